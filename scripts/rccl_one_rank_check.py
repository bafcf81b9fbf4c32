#!/usr/bin/env python3
"""RCCL on the hardware with one rank (the one GPU a box has): a ``ProcessGroupNCCL`` of world 1
drives the engines' data-parallel hooks, eager and captured in a hipGraph, and the results are
compared bit for bit with the hook-free step (a one-rank SUM all-reduce leaves the gradient as
it is).  Run with SL_DETERMINISTIC=1 so that the ResNet engine's kernels are bit-reproducible.

  MLP:    allreduce hook = dist.all_reduce (reduce -> RCCL -> update kernels), 2 eager steps,
          then a captured 3-step graph (the RCCL kernel inside the graph), vs a trainer whose
          hook is a no-op (the same kernels without the collective).
  ResNet: bucket_hook = dist.all_reduce(view, async_op=True) during backward + bucket_wait
          before the update, eager then hipGraph-captured, vs a hook-free engine.

Prints one JSON line.  Usage: SL_DETERMINISTIC=1 python scripts/rccl_one_rank_check.py"""
import json
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if "MASTER_PORT" not in os.environ:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    s.close()
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
import torch
import torch.distributed as dist

from serverless_learn_amd.data.synthetic import make_cifar_like, make_mnist_like
from serverless_learn_amd.models.mlp import FusedMLPTrainer
from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer
from serverless_learn_amd.ops import cnn as K

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
out = {"backend": dist.get_backend(), "world": dist.get_world_size(), "deterministic_build": K.deterministic()}

# ---- MLP: all-reduce hook ----
B = 2048
x, y = make_mnist_like(4 * B, seed=3)
x, y = torch.from_numpy(x), torch.from_numpy(y)
a = FusedMLPTrainer(batch=B, device=dev, seed=1)
b = FusedMLPTrainer(batch=B, device=dev, seed=1)
a.allreduce = lambda g: None
b.allreduce = lambda g: dist.all_reduce(g)
for t in (a, b):
    t.load_shard(x, y)
for _ in range(2):
    a.step()
    b.step()
torch.cuda.synchronize()
out["mlp_eager_identical"] = bool(torch.equal(a.get_flat(), b.get_flat()))
b.capture(warmup=0, unroll=3)
for _ in range(3):
    a.step()
b.steps(3)
torch.cuda.synchronize()
out["mlp_graph_identical"] = bool(torch.equal(a.get_flat(), b.get_flat()) and torch.equal(a.mom, b.mom))
out["mlp_cursor"] = [int(a.cursor.item()), int(b.cursor.item())]
del a, b

# ---- ResNet: bucketed async all-reduces during backward ----
Bc = 32
xc, yc = make_cifar_like(4 * Bc, seed=5)
xc, yc = torch.from_numpy(xc), torch.from_numpy(yc)
ra = FusedResNetTrainer(batch=Bc, device=dev, seed=2)
rb = FusedResNetTrainer(batch=Bc, device=dev, seed=2)
rb.bucket_bytes = 4 << 20
rb.bucket_hook = lambda view: dist.all_reduce(view, async_op=True)
rb.bucket_wait = lambda works: [w.wait() for w in works]
for t in (ra, rb):
    t.load_shard(xc, yc)
nb = []
orig = rb.bucket_hook
rb.bucket_hook = lambda view: (nb.append(view.numel()), orig(view))[1]
for _ in range(2):
    ra.step()
    rb.step()
torch.cuda.synchronize()
rb.bucket_hook = orig
out["resnet_buckets_per_step"] = len(nb) // 2
out["resnet_eager_identical"] = bool(torch.equal(ra.get_flat(), rb.get_flat()))
rb.capture(warmup=0)
for _ in range(2):
    ra.step()
    rb.step()
torch.cuda.synchronize()
out["resnet_graph_identical"] = bool(torch.equal(ra.get_flat(), rb.get_flat()) and torch.equal(ra.mom, rb.mom))
out["resnet_cursor"] = [int(ra.cursor.item()), int(rb.cursor.item())]
out["finite"] = bool(torch.isfinite(rb.get_flat()).all())
dist.destroy_process_group()
print(json.dumps(out))
