#!/usr/bin/env python3
"""Diagnostic: MLP gradient determinism + accuracy at a large batch on the GPU.

Runs compute_grads() several times on the same batch and parameters, reports the max
difference between runs (the fused kernels are deterministic: it must be 0) and the
error against the fp32 reference.  Then trains K steps twice from the same start and
compares the final parameters.
Usage: python scripts/check_mlp_det.py [batch] [bm]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from serverless_learn_amd.data.synthetic import make_mnist_like
from serverless_learn_amd.models import mlp as M
from serverless_learn_amd.ops import _native

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
bm = int(sys.argv[2]) if len(sys.argv) > 2 else 0
_native.call("sl_mlp_set_rows_bm", bm)
print("rows bm", _native.lib().sl_mlp_rows_bm(B))
x, y = make_mnist_like(B * 4, seed=3)
x, y = torch.from_numpy(x), torch.from_numpy(y)
flat = M.init_params(2)
tr = M.FusedMLPTrainer(batch=B, flat=flat, momentum=0.0)
tr.load_shard(x, y)
gs = []
for i in range(4):
    tr.cursor.zero_()
    gs.append(tr.compute_grads().clone())
torch.cuda.synchronize()
for i in range(1, 4):
    print(f"run {i} vs 0: max |diff| {float((gs[i] - gs[0]).abs().max()):.3e}")
g = gs[0].cpu()
_, _, gref = M.reference_grads(flat, x[:B], y[:B], 1.0 / B)
for name, shape, off, n in M.param_layout():
    a, b = g[off:off + n], gref[off:off + n]
    print(f"{name:10s} rel-norm err {float((a - b).norm() / b.norm()):.3e}  finite {bool(torch.isfinite(a).all())}")


def train(k):
    t = M.FusedMLPTrainer(batch=B, flat=flat, momentum=0.9)
    t.load_shard(x, y)
    for _ in range(k):
        t.step()
    torch.cuda.synchronize()
    return t.params.clone(), t.stats()


p1, s1 = train(30)
p2, s2 = train(30)
print(f"train 30 steps twice: max |dparam| {float((p1 - p2).abs().max()):.3e}  loss {s1.loss:.4f} / {s2.loss:.4f}")
