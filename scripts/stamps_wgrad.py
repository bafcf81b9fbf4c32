#!/usr/bin/env python3
"""Diagnostic: per-stage s_memtime stamps of the MLP weight gradient's dW2 loop (slice 0, first
dW2 tile, wave 0).  Prints the median cycles of each phase over the steady-state stages."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from serverless_learn_amd.data.synthetic import make_mnist_like
from serverless_learn_amd.models.mlp import FusedMLPTrainer
from serverless_learn_amd.ops import _native

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
x, y = make_mnist_like(B * 2, seed=0)
tr = FusedMLPTrainer(batch=B, device="cuda:0")
tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
for _ in range(5):
    tr.step()
st = torch.zeros(64 * 8, dtype=torch.int64, device="cuda:0")
_native.call("sl_mlp_set_wg_stamps", st.data_ptr())
tr._lc = None; tr._lkey = None
for _ in range(3):
    tr.step()
torch.cuda.synchronize()
_native.call("sl_mlp_set_wg_stamps", None)
s = st.view(64, 8)[:, :6].cpu().double()
n = int((s[:, 0] != 0).sum())
s = s[:n]
names = ["wait+barrier+issue", "k0 MFMAs+reads", "mid lgkm wait", "k1 MFMAs+recompute", "finish+end wait"]
d = s[:, 1:] - s[:, :-1]
step = s[1:, 0] - s[:-1, 0]
print(f"stages {n}  median cycles per stage {float(step[2:-2].median()):.0f}")
for i, nm in enumerate(names):
    print(f"  {nm:22s} median {float(d[2:-2, i].median()):7.0f}  mean {float(d[2:-2, i].mean()):7.0f}")
