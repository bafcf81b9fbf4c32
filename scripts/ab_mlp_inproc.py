#!/usr/bin/env python3
"""In-process interleaved A/B of MLP step configurations (cdna_hip_programming.md rule 24).

Separate bench processes on one box spread by +-2-3 %, more than the effects being
measured.  Here one trainer on one batch re-captures its step graph for each arm and the
arms alternate over R rounds of K timed steps; medians and per-round ratios are printed.

Arms: rows-kernel tile heights ("--bm 64,128") or weight-gradient split-K slice counts
("--slices 28,24", one trainer per arm).  Kernel libraries cannot be loaded side by side in one
process: use scripts/ab_env.sh for those.
Usage: python scripts/ab_mlp_inproc.py [--bm 64,128 | --slices 28,24] [--rounds 8] [--steps 50]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from serverless_learn_amd.data.synthetic import make_mnist_like
from serverless_learn_amd.models.mlp import FusedMLPTrainer
from serverless_learn_amd.ops import _native

ap = argparse.ArgumentParser()
ap.add_argument("--bm", default="64,128")
ap.add_argument("--slices", default=None, help="comma list of weight-gradient split-K slice counts, one trainer each")
ap.add_argument("--rounds", type=int, default=8)
ap.add_argument("--steps", type=int, default=50)
ap.add_argument("--batch", type=int, default=65536)
a = ap.parse_args()
arms = [int(v) for v in (a.slices or a.bm).split(",")]
B = a.batch
ap_nb = int(os.environ.get("SL_AB_BATCHES", "4"))  # shard size in batches (4: X streams from HBM, as in bench.py)
x, y = make_mnist_like(B * ap_nb, seed=0)
xs, ys = torch.from_numpy(x), torch.from_numpy(y)
if a.slices:
    trs = {}
    for arm in arms:
        trs[arm] = FusedMLPTrainer(batch=B, device="cuda:0", slices=arm)
        trs[arm].load_shard(xs, ys)
        print(arm, "->", trs[arm].slices, file=sys.stderr)
else:
    tr = FusedMLPTrainer(batch=B, device="cuda:0")
    tr.load_shard(xs, ys)
t = {bm: [] for bm in arms}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(a.rounds):
    for bm in arms:
        if a.slices:
            tr = trs[bm]
        else:
            _native.call("sl_mlp_set_rows_bm", bm)
        tr.graph = None
        tr._lc = None
        tr._lkey = None
        tr.capture(warmup=2, unroll=a.steps)
        tr.steps(a.steps)  # warm
        torch.cuda.synchronize()
        e0.record()
        tr.steps(a.steps)
        e1.record()
        torch.cuda.synchronize()
        t[bm].append(e0.elapsed_time(e1) / a.steps * 1e3)  # us per step
res = {str(bm): {"median_us": statistics.median(v), "min_us": min(v), "all": [round(u, 2) for u in v]} for bm, v in t.items()}
if len(arms) == 2:
    ratios = [t[arms[0]][i] / t[arms[1]][i] for i in range(a.rounds)]
    res["ratio_%s_over_%s" % (arms[0], arms[1])] = {"median": statistics.median(ratios), "all": [round(q, 4) for q in ratios]}
print(json.dumps(res, indent=1))
