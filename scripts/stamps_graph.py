#!/usr/bin/env python3
"""Diagnostic: where one graph-replayed MLP step's time goes, on the GPU's own 100 MHz clock.

The rows, weight-gradient and SGD kernels stamp s_memrealtime (chip-wide) when each workgroup
starts and ends. With the stamp buffers set before capture, every replay of a 20-step unrolled
graph (bench.py's form) rewrites them. The last step's values give each launch's span (first
workgroup start to last workgroup end) and the gaps between launches. CUDA events around 10
replays give the step time; what the spans and in-step gaps do not cover is the boundary from
one step's SGD to the next step's rows."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from serverless_learn_amd.data.synthetic import make_mnist_like
from serverless_learn_amd.models.mlp import FusedMLPTrainer
from serverless_learn_amd.ops import _native

B = 65536
UNROLL = 20
x, y = make_mnist_like(B * 4, seed=0)
tr = FusedMLPTrainer(batch=B, device="cuda:0")
tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
bm = _native.lib().sl_mlp_rows_bm(B)
n_rows, n_wg, n_sgd = B // bm, 9 * tr.slices, int(_native.lib().sl_mlp_sgd_wgs())
dev = "cuda:0"
st_r = torch.zeros(n_rows * 20, dtype=torch.int64, device=dev)
st_w = torch.zeros(n_wg * 6, dtype=torch.int64, device=dev)
st_s = torch.zeros(n_sgd * 2, dtype=torch.int64, device=dev)
_native.call("sl_mlp_set_stamps", st_r.data_ptr())
_native.call("sl_mlp_set_wg_stamps", st_w.data_ptr())
_native.call("sl_mlp_set_sgd_stamps", st_s.data_ptr())
tr._lc = None; tr._lkey = None
tr.capture(warmup=2, unroll=UNROLL)
_native.call("sl_mlp_set_stamps", None)
_native.call("sl_mlp_set_wg_stamps", None)
_native.call("sl_mlp_set_sgd_stamps", None)
for _ in range(5):
    tr.steps(UNROLL)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 10
e0.record()
for _ in range(reps):
    tr.steps(UNROLL)
e1.record()
torch.cuda.synchronize()
step_us = e0.elapsed_time(e1) * 1000.0 / (reps * UNROLL)

r = st_r.view(-1, 20).cpu().double()
w = st_w.view(-1, 6).cpu().double()
s = st_s.view(-1, 2).cpu().double()
assert bool((s[:, 0] > 0).all()) and bool((w[:, 4] > 0).all()) and bool((r[:, 16] > 0).all()), "stamps missing"
spans = {"rows": (r[:, 16], r[:, 17]), "wgrad": (w[:, 4], w[:, 5]), "sgd": (s[:, 0], s[:, 1])}
t0 = float(r[:, 16].min())
print(f"step (events, {reps} x {UNROLL}-step graph): {step_us:.1f} us")
prev_end, covered = None, 0.0
for name, (a, b) in spans.items():
    a0, b1 = (float(a.min()) - t0) * 0.01, (float(b.max()) - t0) * 0.01  # 100 MHz ticks -> us
    med = float((b - a).median()) * 0.01
    gap = f"  gap after previous {a0 - prev_end:5.2f} us" if prev_end is not None else ""
    print(f"{name:6s} first start {a0:7.2f}  last end {b1:7.2f}  span {b1 - a0:6.2f} us  "
          f"median WG {med:6.2f} us  last start {(float(a.max()) - t0) * 0.01:7.2f}{gap}")
    if prev_end is not None:
        covered += a0 - prev_end
    covered += b1 - a0
    prev_end = b1
print(f"in-step spans + gaps {covered:.2f} us; rest of the step (SGD end -> next rows start) "
      f"{step_us - covered:.2f} us")
