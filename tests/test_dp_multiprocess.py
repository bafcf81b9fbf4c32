"""Multi-process data parallelism on CPU (gloo, world_size 2) vs single-process training."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from serverless_learn_amd.data.synthetic import make_mnist_like
from serverless_learn_amd.models import mlp as M
from serverless_learn_amd.parallel.dp import ElasticGroup

pytestmark = pytest.mark.slow

STEPS, BATCH = 8, 128


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_path):
    import torch.distributed as dist

    if rank == 0:
        store = dist.TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False)  # noqa: F841
    g = ElasticGroup(device=torch.device("cpu"), timeout_s=30)
    assert g.reform(1, rank, world, f"127.0.0.1:{port}")
    x, y = make_mnist_like(BATCH * world * STEPS, seed=1)
    x = torch.from_numpy(x).view(STEPS, world, BATCH, -1)[:, rank].reshape(-1, 784)
    y = torch.from_numpy(y).view(STEPS, world, BATCH)[:, rank].reshape(-1)
    tr = M.CPUTrainer(batch=BATCH, lr=0.1, momentum=0.9, world_size=world, seed=3)
    tr.load_shard(x, y)
    tr.allreduce = g.allreduce_
    for _ in range(STEPS):
        tr.step()
    torch.save(tr.params, out_path)
    g.teardown()


def test_gloo_dp_matches_single_process(tmp_path):
    world = 2
    port = _free_port()
    outs = [str(tmp_path / f"r{r}.pt") for r in range(world)]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, outs[r])) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    p0, p1 = (torch.load(o, weights_only=True) for o in outs)
    assert torch.equal(p0, p1)
    # single process, global batch = world * BATCH, same sample order
    x, y = make_mnist_like(BATCH * world * STEPS, seed=1)
    ref = M.CPUTrainer(batch=BATCH * world, lr=0.1, momentum=0.9, seed=3)
    ref.load_shard(torch.from_numpy(x), torch.from_numpy(y))
    for _ in range(STEPS):
        ref.step()
    assert torch.allclose(p0, ref.params, atol=3e-4, rtol=1e-3), (p0 - ref.params).abs().max()


def _resnet_rank_main(rank, world, port, out_path):
    import torch.distributed as dist

    from serverless_learn_amd.data.synthetic import make_cifar_like
    from serverless_learn_amd.models.resnet import CPUResNetTrainer

    torch.set_num_threads(2)
    if rank == 0:
        store = dist.TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False)  # noqa: F841
    g = ElasticGroup(device=torch.device("cpu"), timeout_s=60)
    assert g.reform(1, rank, world, f"127.0.0.1:{port}")
    x, y = make_cifar_like(8, seed=10 + rank)
    tr = CPUResNetTrainer(batch=4, lr=0.05, world_size=world, seed=5)
    tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
    tr.allreduce = g.allreduce_
    for _ in range(2):
        tr.step()
    torch.save(tr.params, out_path)
    g.teardown()


def test_gloo_dp_resnet_ranks_stay_identical(tmp_path):
    """Different data per rank, one all-reduced gradient: replicas must not drift."""
    world = 2
    port = _free_port()
    outs = [str(tmp_path / f"r{r}.pt") for r in range(world)]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_resnet_rank_main, args=(r, world, port, outs[r])) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    p0, p1 = (torch.load(o, weights_only=True) for o in outs)
    assert torch.equal(p0, p1)
    from serverless_learn_amd.models.resnet import init_params, resnet18_spec

    assert not torch.equal(p0, init_params(resnet18_spec(), 5))
