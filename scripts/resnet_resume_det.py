#!/usr/bin/env python3
"""Exact resume of the ResNet engine in the deterministic kernel build (SL_DETERMINISTIC=1):
train k steps, save through the checkpoint byte format (parameters + momentum + cursor +
BatchNorm running statistics), restore into a fresh engine with another seed, and run m more
steps in both.  Prints JSON; with the deterministic build the two must be bit-identical
(parameters, momentum, running statistics, cursor).
Usage: SL_DETERMINISTIC=1 python scripts/resnet_resume_det.py [batch] [k] [m]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from serverless_learn_amd.ckpt import format as ckfmt
from serverless_learn_amd.data.synthetic import make_cifar_like
from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer
from serverless_learn_amd.ops import cnn as K

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 32
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
m = int(sys.argv[3]) if len(sys.argv) > 3 else 2
x, y = make_cifar_like(4 * batch, seed=5)
x, y = torch.from_numpy(x), torch.from_numpy(y)
a = FusedResNetTrainer(batch=batch, device="cuda:0", seed=2)
a.load_shard(x, y)
for _ in range(k):
    a.step()
n = a.n_params
buf = ckfmt.encode(a.get_flat().cpu().numpy(), {"model": a.model_name, "step": k}, a.mom[:n].cpu().numpy(),
                   a.state_extra())
meta, params, mom, extra = ckfmt.decode_full(buf)
b = FusedResNetTrainer(batch=batch, device="cuda:0", seed=7)
b.load_shard(x, y)
b.set_flat(torch.from_numpy(params))
b.mom[:n].copy_(torch.from_numpy(mom))
b.load_state_extra(extra)
for _ in range(m):
    a.step()
    b.step()
torch.cuda.synchronize()
stats_equal = all(torch.equal(rm, b.running_stats()[name][0]) and torch.equal(rv, b.running_stats()[name][1])
                  for name, (rm, rv) in a.running_stats().items())
pa, pb = a.get_flat(), b.get_flat()
print(json.dumps({"deterministic_build": K.deterministic(), "batch": batch, "k": k, "m": m,
                  "params_identical": bool(torch.equal(pa, pb)), "mom_identical": bool(torch.equal(a.mom, b.mom)),
                  "running_stats_identical": bool(stats_equal),
                  "cursor": [int(a.cursor.item()), int(b.cursor.item())],
                  "param_max_diff": float((pa - pb).abs().max()), "finite": bool(torch.isfinite(pa).all())}))
