#!/usr/bin/env python3
"""Diagnostic: where the bench's timed region loses against the steady-state step.

bench.py times K steps as one replay of a K-step graph, bracketed by synchronize() and a
host clock.  This probe times the same replay three ways on one trainer: (a) host clock
around sync/replay/sync after the GPU went idle (the bench form), (b) CUDA events around a
replay that follows another replay (steady state), (c) the host clock around two
back-to-back replays (fixed per-region cost = (c) - 2 x (b)).  Prints JSON (us per step).
Usage: python scripts/timed_region_probe.py [K] [reps]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from serverless_learn_amd.data.synthetic import make_mnist_like
from serverless_learn_amd.models.mlp import FusedMLPTrainer

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
B = 65536
x, y = make_mnist_like(B * 4, seed=0)
tr = FusedMLPTrainer(batch=B, device="cuda:0")
tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
for _ in range(3):
    tr.step()
tr.capture(warmup=0, unroll=K)
tr.steps(K)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
bench_form, steady, double = [], [], []
for _ in range(reps):
    time.sleep(0.05)  # GPU idle, as after the bench's setup
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.steps(K)
    torch.cuda.synchronize()
    bench_form.append((time.perf_counter() - t0) / K * 1e6)
    tr.steps(K)
    e0.record()
    tr.steps(K)
    e1.record()
    torch.cuda.synchronize()
    steady.append(e0.elapsed_time(e1) / K * 1e3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.steps(K)
    tr.steps(K)
    torch.cuda.synchronize()
    double.append((time.perf_counter() - t0) / (2 * K) * 1e6)
med = statistics.median
print(json.dumps({"K": K, "bench_form_us": round(med(bench_form), 2), "steady_events_us": round(med(steady), 2),
                  "two_replays_host_us": round(med(double), 2),
                  "fixed_per_region_us": round((med(double) * 2 * K - 2 * K * med(steady)) / 1, 1),
                  "bench_form_all": [round(v, 1) for v in bench_form]}))
