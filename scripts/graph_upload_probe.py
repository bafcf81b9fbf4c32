"""Does the first replay of a freshly captured multi-step MLP graph cost more than later
ones, and does hipGraphUpload on the graph exec remove that?  Times replays of a
20-step graph (B=65536) on two trainers: one replayed cold, one uploaded first."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from serverless_learn_amd.data.synthetic import make_shard, decode_shard  # noqa: E402
from serverless_learn_amd.models.mlp import FusedMLPTrainer  # noqa: E402

K = 20
dev = torch.device("cuda", 0)
hdr, xi, yi = decode_shard(bytearray(make_shard(65536 * 4, 0, 1, seed=0, dataset="synthetic-mnist")))
x, y = torch.from_numpy(xi).to(dev), torch.from_numpy(yi.copy()).to(dev)
hip = ctypes.CDLL("libamdhip64.so")


def one(upload: bool):
    tr = FusedMLPTrainer(batch=65536, device=dev, seed=0)
    tr.load_shard(x, y)
    for _ in range(3):
        tr.step()
    tr.capture(warmup=0, unroll=K)
    tr.step()
    tr.step()
    torch.cuda.synchronize()
    if upload:
        ex = tr.graph_unrolled.raw_cuda_graph_exec()
        rc = hip.hipGraphUpload(ctypes.c_void_p(ex), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        assert rc == 0, rc
    ts = []
    for _ in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.steps(K)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3 / K)
    return ts


out = {"cold": one(False), "uploaded": one(True), "cold_again": one(False)}
print(json.dumps({k: [round(t, 4) for t in v] for k, v in out.items()}))
