"""Throughput of the engine's implicit-GEMM 3x3 convolutions against hipBLASLt (torch.matmul on
the equivalent [M, K] x [K, N] GEMM) and MIOpen (F.conv2d, channels-last bf16) on the
ResNet-18 stage shapes at B = 1024.  Prints one JSON line per shape (TFLOP/s each)."""
import json
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from serverless_learn_amd.ops import cnn  # noqa: E402


def clock(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    dev = torch.device("cuda", 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    for h, c in ((32, 64), (16, 128), (8, 256), (4, 512)):
        x = torch.randn(B, h, h, c, device=dev).to(torch.bfloat16)
        w = (torch.randn(c, 3, 3, c, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.empty(B, h, h, c, device=dev, dtype=torch.bfloat16)
        stats = torch.zeros(cnn.rsum_floats(2 * c), device=dev)
        flop = 2.0 * B * h * h * c * c * 9
        t_eng = clock(lambda: cnn.conv_fwd(x, w.view(c, -1), c, 3, 1, 1, y=y, stats=stats))
        a = torch.randn(B * h * h, 9 * c, device=dev).to(torch.bfloat16)
        bm = torch.randn(9 * c, c, device=dev).to(torch.bfloat16)
        t_blas = clock(lambda: a @ bm)
        xn = x.permute(0, 3, 1, 2)  # NCHW view of NHWC memory = channels_last
        wn = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        try:
            t_miopen = clock(lambda: F.conv2d(xn, wn, padding=1), reps=10)
        except Exception as e:  # noqa: BLE001
            t_miopen = float("nan")
            print(f"miopen: {e}", file=sys.stderr)
        # numerics: engine vs torch on a slice
        ref = F.conv2d(xn[:8].float(), w.permute(0, 3, 1, 2).float(), padding=1).permute(0, 2, 3, 1)
        err = float((y[:8].float() - ref).abs().max() / ref.abs().max())
        print(json.dumps({"h": h, "c": c, "B": B, "gflop": round(flop / 1e9, 1),
                          "engine_us": round(t_eng * 1e6, 1), "engine_tflops": round(flop / t_eng / 1e12, 1),
                          "hipblaslt_gemm_us": round(t_blas * 1e6, 1), "hipblaslt_tflops": round(flop / t_blas / 1e12, 1),
                          "miopen_us": round(t_miopen * 1e6, 1), "miopen_tflops": round(flop / t_miopen / 1e12, 1),
                          "engine_rel_err": round(err, 4)}), flush=True)


if __name__ == "__main__":
    main()
