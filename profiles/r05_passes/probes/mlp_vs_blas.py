#!/usr/bin/env python3
"""The bar for the hand-written MLP kernels: hipBLASLt (torch.matmul, bf16) on the GEMM shapes
of one MLP training step at B = 65,536 (784-256-256-10).

Times each shape by events over back-to-back repetitions (after warm-up) and prints one JSON
line: per-shape us and TFLOP/s, and the sum over the step's GEMMs -- what a library-GEMM step
would cost before any of the elementwise work (bias, ReLU, softmax-CE, masks, SGD) that the
fused kernels do in their epilogues.

usage: python scripts/mlp_vs_blas.py [batch] [reps]"""
import json
import sys

import torch

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda", 0)
bf = torch.bfloat16
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*shape):
    return torch.randn(*shape, device=dev, dtype=bf, generator=g)


X, H1, dH2, dH1, dZ = rnd(B, 784), rnd(B, 256), rnd(B, 256), rnd(B, 256), rnd(B, 16)
W1, W2, W3 = rnd(256, 784), rnd(256, 256), rnd(16, 256)
shapes = {
    # name: (callable, flop)
    "l1_fwd  X[B,784] W1^T": (lambda: X @ W1.t(), 2 * B * 784 * 256),
    "l2_fwd  H1[B,256] W2^T": (lambda: H1 @ W2.t(), 2 * B * 256 * 256),
    "l3_fwd  H2[B,256] W3^T(16)": (lambda: H1 @ W3.t(), 2 * B * 256 * 16),
    "l3_bwd  dZ[B,16] W3": (lambda: dZ @ W3, 2 * B * 16 * 256),
    "l2_bwd  dH2[B,256] W2": (lambda: dH2 @ W2, 2 * B * 256 * 256),
    "dW1     dH1^T X": (lambda: dH1.t() @ X, 2 * B * 784 * 256),
    "dW2     dH2^T H1": (lambda: dH2.t() @ H1, 2 * B * 256 * 256),
    "dW3     dZ^T H2": (lambda: dZ.t() @ H1, 2 * B * 256 * 16),
}
out = {"batch": B, "reps": reps, "shapes": {}}
total_us = total_flop = 0.0
for name, (fn, flop) in shapes.items():
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    out["shapes"][name] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1)}
    total_us += us
    total_flop += flop
out["sum_us"] = round(total_us, 2)
out["sum_tflops"] = round(total_flop / total_us / 1e6, 1)
out["samples_per_s_gemms_only"] = round(B / (total_us * 1e-6), 1)
print(json.dumps(out))
