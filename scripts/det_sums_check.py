#!/usr/bin/env python3
"""Range check of the cross-workgroup sums (csrc/kernels/common.h fix_add): the BatchNorm
statistics a conv epilogue accumulates, for outputs of a large magnitude (sum of squares far
past 2^31, where a single 2^-32 fixed-point int64 used to wrap) and of a tiny one (where a
coarse scale would round the values away), against fp64 sums of the stored outputs.
Prints one JSON line.  Run with SL_DETERMINISTIC=1 for the fixed-point build.
Usage: [SL_DETERMINISTIC=1] python scripts/det_sums_check.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from serverless_learn_amd.ops import cnn as K

DEV = torch.device("cuda", 0)


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


out = {"deterministic_build": K.deterministic()}
torch.manual_seed(3)
n, h, c = 64, 32, 64
x = torch.randn(n, h, 32, c, device=DEV).to(torch.bfloat16)
w0 = torch.randn(c, 3, 3, c, device=DEV) / 24
for name, scale in (("large", 400.0), ("tiny", 1e-5)):
    w = (w0 * scale).to(torch.bfloat16)
    y = torch.empty_like(x)
    s = torch.zeros(K.rsum_floats(2 * c), device=DEV)
    K.conv_fwd(x, w, c, 3, 1, 1, y=y, stats=s)
    torch.cuda.synchronize()
    st = K.rsum_result(s, 2 * c).clone()
    yf = y.double().reshape(-1, c)
    ref_s, ref_q = yf.sum(0), (yf * yf).sum(0)
    out[name] = {"sumsq_max": float(ref_q.max()), "rel_sum": rel(st[:c], ref_s), "rel_sumsq": rel(st[c:], ref_q),
                 "finite": bool(torch.isfinite(st).all())}
print(json.dumps(out))
