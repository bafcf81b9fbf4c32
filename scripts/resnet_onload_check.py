#!/usr/bin/env python3
"""Trains the ResNet-18 engine K steps from a fixed seed and prints JSON with a hash of the
final parameters and the number of blocks on the BN-on-load path (SL_BN_ONLOAD).  Run under
SL_DETERMINISTIC=1 with SL_BN_ONLOAD=1 and =0: the hashes must agree
(tests/test_cnn_gpu.py::test_resnet_engine_bn_on_load_is_bit_identical_in_deterministic_build).
Usage: SL_DETERMINISTIC=1 SL_BN_ONLOAD=0|1 python scripts/resnet_onload_check.py [batch] [steps]"""
import hashlib
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
tr = FusedResNetTrainer(batch=batch, device="cuda:0", seed=7)
tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
for _ in range(steps):
    tr.step()
torch.cuda.synchronize()
p = tr.get_flat().cpu()
print(json.dumps({"deterministic_build": K.deterministic(), "bn_onload": tr.bn_onload,
                  "bnin_blocks": sum(bool(st["bnin"]) for st in tr.blocks), "stem_onload": tr.stem_onload, "batch": batch, "steps": steps,
                  "param_hash": hashlib.sha256(p.numpy().tobytes()).hexdigest()[:16], "loss": tr.stats().loss,
                  "finite": bool(torch.isfinite(p).all())}))
