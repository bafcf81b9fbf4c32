#!/usr/bin/env python3
"""Run-to-run reproducibility of the ResNet-18 engine: two fresh engines from the same
seed train K steps on the same data; prints JSON with the max parameter / gradient
difference and whether they are bit-identical.  With SL_DETERMINISTIC=1 the
deterministic kernel build is loaded (fixed-point cross-workgroup sums, no split-K
atomics) and the runs must be identical; the default build shows its fp32-atomic noise.
Usage: [SL_DETERMINISTIC=1] python scripts/resnet_det_check.py [batch] [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from serverless_learn_amd.data.synthetic import make_cifar_like
from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer
from serverless_learn_amd.ops import cnn as K

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 64
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
x, y = make_cifar_like(batch * 2, seed=1)
runs = []
for _ in range(2):
    tr = FusedResNetTrainer(batch=batch, device="cuda:0", seed=7)
    tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
    g = tr.compute_grads().clone()
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    runs.append((g, tr.get_flat().clone(), tr.stats().loss))
(g0, p0, l0), (g1, p1, l1) = runs
print(json.dumps({"deterministic_build": K.deterministic(), "batch": batch, "steps": steps,
                  "grad_identical": bool(torch.equal(g0, g1)), "params_identical": bool(torch.equal(p0, p1)),
                  "grad_max_diff": float((g0 - g1).abs().max()), "param_max_diff": float((p0 - p1).abs().max()),
                  "grad_cos": float(torch.nn.functional.cosine_similarity(g0.double(), g1.double(), dim=0)),
                  "loss": [l0, l1], "finite": bool(torch.isfinite(p0).all())}))
