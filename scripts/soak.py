#!/usr/bin/env python3
"""Stability soak of the 1-GPU training step (graph-replayed, bench.py's engine path) for a
fixed wall time.  One JSON line per interval (~20 s): steps, interval samples/s, loss, device
memory.  At the end, one summary line: interval throughput min / median / max, whether the
loss stayed finite, and how much device memory grew.

usage: python scripts/soak.py --model mlp|resnet18 --seconds 600 [--batch B] [--interval 20]
"""
import argparse
import json
import math
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=("mlp", "resnet18"), default="mlp")
    ap.add_argument("--seconds", type=float, default=600.0)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--interval", type=float, default=20.0)
    ap.add_argument("--chunk", type=int, default=None, help="steps per replay burst between clock reads")
    a = ap.parse_args()
    mlp = a.model == "mlp"
    B = a.batch or (65536 if mlp else 1024)
    chunk = a.chunk or (20 if mlp else 8)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)

    from serverless_learn_amd.data.device_synth import synth_on_device

    x, y = synth_on_device("mnist" if mlp else "cifar", B * 4, seed=0, device=dev)
    if mlp:
        from serverless_learn_amd.models.mlp import FusedMLPTrainer
        tr = FusedMLPTrainer(batch=B, device=dev, lr=0.1, momentum=0.9, world_size=1, seed=0)
    else:
        from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer
        tr = FusedResNetTrainer(batch=B, device=dev, lr=0.1, momentum=0.9, world_size=1, seed=0)
    tr.load_shard(x, y)
    for _ in range(3):
        tr.step()
    if mlp:
        tr.capture(warmup=0, unroll=chunk)
    else:
        tr.capture(warmup=0)
    run = getattr(tr, "steps", None) or (lambda n: [tr.step() for _ in range(n)])
    run(chunk)
    torch.cuda.synchronize()
    mem0 = torch.cuda.memory_allocated(dev)

    rates, losses, nonfinite = [], [], 0
    total = 0
    t_start = time.perf_counter()
    t_end = t_start + a.seconds
    while time.perf_counter() < t_end:
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < a.interval and time.perf_counter() < t_end:
            run(chunk)
            n += chunk
            if n % (chunk * 16) == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        total += n
        loss = float(tr.stats().loss)
        finite = math.isfinite(loss)
        nonfinite += 0 if finite else 1
        rates.append(B * n / dt)
        losses.append(loss)
        print(json.dumps({"t_s": round(time.perf_counter() - t_start, 1), "steps": total,
                          "samples_per_s": round(B * n / dt, 1), "loss": round(loss, 5) if finite else str(loss),
                          "mem_mb": round(torch.cuda.memory_allocated(dev) / 2**20, 1)}), flush=True)
    summary = {"summary": True, "model": a.model, "batch": B, "seconds": round(time.perf_counter() - t_start, 1),
               "steps": total, "intervals": len(rates),
               "samples_per_s_min": round(min(rates), 1), "samples_per_s_median": round(statistics.median(rates), 1),
               "samples_per_s_max": round(max(rates), 1), "loss_first": losses[0], "loss_last": losses[-1],
               "nonfinite_intervals": nonfinite,
               "mem_growth_mb": round((torch.cuda.memory_allocated(dev) - mem0) / 2**20, 2)}
    print(json.dumps(summary), flush=True)
    return 0 if nonfinite == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
