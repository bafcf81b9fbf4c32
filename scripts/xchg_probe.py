#!/usr/bin/env python3
"""Fixed per-step cost of the MLP's xGMI gradient exchange on one GPU.

A one-rank XgmiExchange runs the multi-GPU step's exact launch sequence -- slab reduction into
the exchange slot that publishes the step, (two-shot: reduce-scatter that waits and publishes,)
update kernel that waits and reads the slots back; or the round-5 sequence with the one-wave
barrier kernel(s) in between -- with no peer, so the difference to the 1-GPU step (slab reduction
fused with the update) is the exchange's fixed cost.  Graph-replayed K-step regions, modes
interleaved; one JSON line per mode.  Kernel times: run under rocprofv3 --kernel-trace --stats."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main() -> int:
    from serverless_learn_amd.data.synthetic import make_mnist_like
    from serverless_learn_amd.models.mlp import FusedMLPTrainer
    from serverless_learn_amd.parallel.xgmi import XgmiExchange

    B = 65536
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    x, y = make_mnist_like(B * 4, seed=0)
    x, y = torch.from_numpy(x), torch.from_numpy(y)
    modes = {}
    # inline synchronisation (the default since round 6: the reduce publishes, the update waits
    # per workgroup) against the round-5 protocol with its one-wave barrier kernel(s)
    for mode in ("sgd", "xgmi_one_shot", "xgmi_two_shot", "xgmi_one_shot_barrier", "xgmi_two_shot_barrier"):
        tr = FusedMLPTrainer(batch=B, device=dev)
        tr.load_shard(x, y)
        if mode != "sgd":
            os.environ["SL_XGMI_BARRIER"] = "1" if mode.endswith("_barrier") else "0"
            ex = XgmiExchange(tr.n_pad, 0, 1, dev, lambda b: [b], lambda ok: ok, two_shot="two_shot" in mode)
            tr.enable_xgmi(ex)
        tr.step()
        tr.capture(warmup=1, unroll=K)
        modes[mode] = tr
    out = {m: [] for m in modes}
    for _ in range(reps):
        for m, tr in modes.items():
            tr.steps(K)  # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.steps(K)
            torch.cuda.synchronize()
            out[m].append((time.perf_counter() - t0) / K * 1e6)
    base = min(out["sgd"])
    for m, v in out.items():
        print(json.dumps({"mode": m, "us_per_step": [round(t, 2) for t in v], "best": round(min(v), 2),
                          "over_sgd_us": round(min(v) - base, 2)}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
