#!/usr/bin/env python3
"""Time the ResNet-18 stage-2 downsample data gradient (3x3 / stride 2 into 64 channels, B = 1024,
the four parity-class launches of ``conv_dgrad``) in its variants, to split its cost between the
GEMM and the fused epilogue work: plain, + residual add, + fused BN backward (mask + sums), + both.

    python scripts/dgrad_probe.py [--batch 1024] [--reps 30] [--h 32 --cin 64 | --h 16 --cin 128 | --h 8 --cin 256]

Prints one JSON line of microseconds per call (CUDA events around ``reps`` back-to-back calls).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--h", type=int, default=32, help="input (dx) height = width: 32 / 16 / 8 = stage 2 / 3 / 4")
    ap.add_argument("--cin", type=int, default=64)
    args = ap.parse_args()
    from serverless_learn_amd.ops import cnn as K

    dev = "cuda"
    n, h, c = args.batch, args.h, args.cin
    cout = 2 * c
    oh = h // 2
    g = torch.Generator(device="cpu").manual_seed(0)
    dy = torch.randn(n, oh, oh, cout, generator=g).to(dev, torch.bfloat16)
    wt = (torch.randn(c, 9, cout, generator=g) / math.sqrt(9 * cout)).to(dev, torch.bfloat16).reshape(-1)
    add = torch.randn(n, h, h, c, generator=g).to(dev, torch.bfloat16)
    xb = torch.randn(n, h, h, c, generator=g).to(dev, torch.bfloat16)
    coef = torch.randn(4 * c, generator=g).to(dev)
    sums = torch.zeros(K.rsum_floats(2 * c), device=dev)
    dx = torch.empty(n, h, h, c, dtype=torch.bfloat16, device=dev)

    def timed(fn) -> float:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / args.reps

    bn = dict(x=xb, mask_coef=coef, sums=sums)
    out = {
        "shape": {"batch": n, "h": h, "cin": c, "cout": cout, "k": 3, "stride": 2},
        "plain_us": timed(lambda: K.conv_dgrad(dy, wt, c, 3, 2, 1, dx)),
        "add_us": timed(lambda: K.conv_dgrad(dy, wt, c, 3, 2, 1, dx, add=add)),
        "bn_us": timed(lambda: K.conv_dgrad(dy, wt, c, 3, 2, 1, dx, bn=bn)),
        "add_bn_us": timed(lambda: K.conv_dgrad(dy, wt, c, 3, 2, 1, dx, add=add, bn=bn)),
    }
    # bytes every variant must move at least: dx written, dy read once (+ add, + BN input x read)
    mb = lambda t: t.numel() * t.element_size() / 1e6  # noqa: E731
    out["min_mb"] = {"plain": round(mb(dx) + mb(dy), 1), "add_bn": round(3 * mb(dx) + mb(dy), 1)}
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in out.items()}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
