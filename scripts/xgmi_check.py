#!/usr/bin/env python3
"""Multi-rank check of the xGMI exchange (parallel/xgmi.py, csrc/kernels/xgmi.*).

Launched by tests/test_xgmi_gpu.py as
``torchrun --nproc-per-node W scripts/xgmi_check.py [--same-device] [--two-shot]``: every rank
maps every other rank's exchange buffer over IPC (on one GPU the ranks share the
device -- the same code path minus the xGMI links).  Checks, per rank:

0. the setup-time probe (``parallel.xgmi.probe``) passes;
1. the generic all-reduce (one-shot, or reduce-scatter + all-gather with ``--two-shot``) equals the rank-order fp32 sum, over several
   calls (both slot parities, device-side step counter);
2. the MLP step with the all-reduce fused into its update kernel gives exactly the
   parameters of the same step with gloo's all-reduce of the reduced gradient,
   eager and replayed from an 8-step hipGraph, and all replicas stay bit-identical;
3. no barrier timed out;
4. ``XgmiExchange.abort()`` ends a wait on peers that never signal within 3 s (processes with
   HIP's default 4 hardware queues: the 2-rank runs).
Prints ``XGMI_CHECK_OK rank=R`` on success; any failure raises (non-zero exit).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.distributed as dist


def _same(p, q, msg):
    """Bit-exact: the reference sums in rank order, as the kernel does."""
    if not torch.equal(p, q):
        bad = (p != q).nonzero().flatten()
        raise AssertionError(f"{msg}: {bad.numel()} params differ, first {bad[:8].tolist()}, "
                             f"max |diff| {(p - q).abs().max().item():.3e}")


def main() -> int:
    same = "--same-device" in sys.argv
    two = "--two-shot" in sys.argv
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0 if same else int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    from serverless_learn_amd.data.synthetic import make_mnist_like
    from serverless_learn_amd.models.mlp import FusedMLPTrainer
    from serverless_learn_amd.parallel.xgmi import XgmiExchange, dist_collectives

    # 0. the setup-time probe bench.py and the worker run before trusting the exchange
    from serverless_learn_amd.parallel.xgmi import probe
    bad = probe(rank, world, dev, *dist_collectives())
    assert bad == "", bad

    # 1. generic all-reduce
    n = 100_000
    ex = XgmiExchange(n, rank, world, dev, *dist_collectives(), two_shot=two)
    for it in range(5):
        gens = [torch.Generator().manual_seed(1000 * it + q) for q in range(world)]
        parts = [torch.randn(n, generator=g) for g in gens]
        expect = parts[0].clone()
        for q in range(1, world):
            expect += parts[q]
        t = parts[rank].to(dev)
        ex.allreduce_(t)
        torch.cuda.synchronize()
        assert torch.equal(t.cpu(), expect), f"generic allreduce mismatch at call {it}"
    assert not ex.error() and ex.steps_done() == 5, (ex.error(), ex.steps_done())
    dist.barrier()
    torch.cuda.synchronize()
    ex.close()

    # 2. MLP: fused xGMI update == the host all-reduce path, bit for bit
    B = 256
    x, y = make_mnist_like(B * 4, seed=rank + 1)
    xt, yt = torch.from_numpy(x), torch.from_numpy(y)
    a = FusedMLPTrainer(batch=B, device=dev, world_size=world, seed=0)
    b = FusedMLPTrainer(batch=B, device=dev, world_size=world, seed=0)
    a.load_shard(xt, yt)
    b.load_shard(xt, yt)
    xa = XgmiExchange(a.n_pad, rank, world, dev, *dist_collectives(), two_shot=two)
    a.enable_xgmi(xa)

    def host_allreduce(g):
        """Reference all-reduce through host memory, summing in rank order as the kernel does."""
        parts = [torch.empty(g.numel()) for _ in range(world)]
        dist.all_gather(parts, g.cpu())
        acc = parts[0].clone()
        for q in range(1, world):
            acc += parts[q]
        g.copy_(acc.to(g.device))

    def b_step():
        """b's step by hand, keeping its local gradient for the diagnostics."""
        b._rows(True)
        b._wgrad()
        b._sgd(1, from_grad=False, grad_out=True, bump=False)
        g_loc = b.grad.clone()
        host_allreduce(b.grad)
        b._sgd(2, from_grad=True, grad_out=False)
        return g_loc

    for step in range(12):
        g_loc = b_step()
        a.step()
        torch.cuda.synchronize()
        assert not xa.error(), f"xgmi barrier timed out at step {step}"
        bad = torch.tensor([0 if torch.equal(a.params, b.params) else 1])
        dist.all_reduce(bad)  # every rank takes the diagnostics branch together (it has collectives)
        if bad.item():
            n = g_loc.numel()
            parity = (step + 1) & 1
            peers = [torch.empty(n) for _ in range(world)]
            dist.all_gather(peers, g_loc.cpu())
            for q in range(world):
                v = xa.peek(q, parity, n, True).cpu()
                print(f"DIAG step={step} rank={rank} slot_of={q} parity={parity} "
                      f"diff_vs_local_of_q={(v - peers[q]).abs().max().item():.3e}", flush=True)
        _same(a.params, b.params, f"eager step {step}: xgmi != host all-reduce")
    b.allreduce = host_allreduce
    a.capture(warmup=0, unroll=8)  # records only: nothing runs during capture
    a.steps(16)
    torch.cuda.synchronize()
    done = xa.steps_done()
    assert done == 28, done
    for _ in range(16):
        b.step()
    torch.cuda.synchronize()
    _same(a.params, b.params, "graph replay: xgmi != host all-reduce")
    # replicas identical across ranks
    flat = a.params.detach().cpu()
    ref = flat.clone()
    dist.broadcast(ref, 0)
    assert torch.equal(flat, ref), "replicas diverged"
    assert not xa.error(), "an xgmi barrier timed out"
    dist.barrier()
    torch.cuda.synchronize()
    xa.close()
    # 4. host abort: rank 0 starts an exchange that no peer joins; XgmiExchange.abort() must end
    # its wait at once (the elastic runtime calls it on a broken group) instead of at the 10 s timeout
    # (only with HIP's default 4 hardware queues: capped ranks may share one queue with the spinner)
    import time
    xb = XgmiExchange(1024, rank, world, dev, *dist_collectives(), two_shot=False)
    if rank == 0 and int(os.environ.get("GPU_MAX_HW_QUEUES") or 4) >= 4:
        t = torch.ones(1024, device=dev)
        xb.allreduce_(t)
        time.sleep(0.3)  # the barrier is spinning on the peers by now
        t0 = time.monotonic()
        xb.abort()
        torch.cuda.synchronize()
        waited = time.monotonic() - t0
        assert xb.error() and waited < 3.0, (xb.error(), waited)
        print(f"XGMI_ABORT rank=0 drained_s={waited:.3f}", flush=True)
    dist.barrier()  # rank 0's kernels are done with every peer's buffer before anyone unmaps
    xb.close()
    print(f"XGMI_CHECK_OK rank={rank} two_shot={two} steps={done} loss={a.stats().loss:.4f}", flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
