#!/usr/bin/env python3
"""Probe: one-rank RCCL group; time the MLP step eager (kernels + all_reduce hook) vs captured
in a hipGraph with the all_reduce inside.  Usage: python scripts/graph_nccl_probe.py [batch]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
import torch
import torch.distributed as dist

from serverless_learn_amd.data.synthetic import make_mnist_like
from serverless_learn_amd.models.mlp import FusedMLPTrainer

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
x, y = make_mnist_like(B * 2, seed=0)
tr = FusedMLPTrainer(batch=B, device=dev)
tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
tr.allreduce = lambda g: dist.all_reduce(g)


def timeit(n=200):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        tr.step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


for _ in range(10):
    tr.step()
print(f"eager+allreduce: {timeit():.1f} us/step")
tr.allreduce = None
for _ in range(5):
    tr.step()
print(f"eager, no allreduce: {timeit():.1f} us/step")
tr.allreduce = lambda g: dist.all_reduce(g)
tr.capture(warmup=2)
print(f"graph+allreduce: {timeit():.1f} us/step")
print(f"loss {tr.stats().loss:.4f}")
dist.destroy_process_group()
