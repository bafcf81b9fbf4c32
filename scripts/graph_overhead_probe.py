"""Where does the fixed cost of one timed multi-step MLP graph replay go?  A 20-step replay
after a synchronize costs ~150 us more GPU time than 20 steps inside a 200-step replay
(profiles/r03_graph).  Variants, each timed by events around the replay (B=65536):

  sync      synchronize, record, replay (the bench's timed region)
  busy      a ~300 us spin kernel queued first, so host submission is hidden
  idle_Xms  synchronize, host sleep X ms, replay
  b2b       10 replays back-to-back, one event pair around all
  split     a 1-step graph then a 19-step graph (the GPU starts while the rest is submitted)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from serverless_learn_amd.data.synthetic import decode_shard, make_shard  # noqa: E402
from serverless_learn_amd.models.mlp import FusedMLPTrainer  # noqa: E402

dev = torch.device("cuda", 0)
hdr, xi, yi = decode_shard(bytearray(make_shard(65536 * 4, 0, 1, seed=0, dataset="synthetic-mnist")))
x, y = torch.from_numpy(xi).to(dev), torch.from_numpy(yi.copy()).to(dev)
K = 20


def trainer(unroll):
    tr = FusedMLPTrainer(batch=65536, device=dev, seed=0)
    tr.load_shard(x, y)
    for _ in range(3):
        tr.step()
    tr.capture(warmup=0, unroll=unroll)
    tr.steps(unroll)
    torch.cuda.synchronize()
    return tr


def timed(fn, pre=None, idle_s=0.0, reps=5):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        if idle_s:
            time.sleep(idle_s)
        if pre:
            pre()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        out.append((round(e0.elapsed_time(e1) * 1e3, 1), round((time.perf_counter() - t0) * 1e6, 1)))
    return out


res = {}
tr = trainer(K)
g = tr.graph_unrolled
res["sync"] = timed(g.replay)
res["busy"] = timed(g.replay, pre=lambda: torch.cuda._sleep(600_000))
for ms in (1, 10, 100):
    res[f"idle_{ms}ms"] = timed(g.replay, idle_s=ms / 1000.0)
res["b2b_10"] = timed(lambda: [g.replay() for _ in range(10)], reps=3)
res["sync_again"] = timed(g.replay)
del tr
torch.cuda.empty_cache()
t19 = trainer(19)  # capture() also keeps the 1-step graph
res["split_1_19"] = timed(lambda: (t19.graph.replay(), t19.graph_unrolled.replay()))
res["unsplit_19"] = timed(t19.graph_unrolled.replay)
summary = {k: {"gpu_us_min": min(v[0] for v in vals), "wall_us_min": min(v[1] for v in vals), "all": vals}
           for k, vals in res.items()}
print(json.dumps(summary))
