#!/usr/bin/env python3
"""Diagnostic: per-workgroup s_memtime stamps of the MLP weight gradient (mlp_wgrad_kernel):
main-loop and total cycles per tile kind (dW1 tiles 0-6, dW2 tiles 7-8) for a steady-state step."""
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
nwg = 9 * tr.slices
st = torch.zeros(nwg * 6, dtype=torch.int64, device="cuda:0")
_native.call("sl_mlp_set_wg_stamps", st.data_ptr())
tr._lc = None; tr._lkey = None
for _ in range(3):
    tr.step()
torch.cuda.synchronize()
_native.call("sl_mlp_set_wg_stamps", None)
s = st.view(nwg, 6).cpu().double()
t0 = s[:, 0].min()
tile = torch.arange(nwg) % 9
for name, sel in (("dW1 tiles 0-5", tile < 6), ("dW1 tile 6 (16 cols)", tile == 6), ("dW2 tiles", tile >= 7)):
    v = s[sel]
    print(f"{name:22s} n={int(sel.sum()):3d}  main loop median {float((v[:, 1] - v[:, 0]).median()):8.0f}  "
          f"max {float((v[:, 1] - v[:, 0]).max()):8.0f}  total median {float((v[:, 2] - v[:, 0]).median()):8.0f}  "
          f"start spread {float((v[:, 0] - t0).max()):6.0f}  end max {float((v[:, 2] - t0).max()):8.0f}")
r = s[:, 5] - s[:, 4]
mhz = (s[:, 2] - s[:, 0]) / (r / 100.0)
print(f"shader clock MHz over each WG: median {float(mhz.median()):.0f}  min {float(mhz.min()):.0f}  "
      f"max {float(mhz.max()):.0f};  first start -> last end {float(s[:, 5].max() - s[:, 4].min()) * 10:.0f} ns")
