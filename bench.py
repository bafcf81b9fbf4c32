#!/usr/bin/env python3
"""Headline benchmark: samples/sec (whole node), 3-layer MLP on synthetic MNIST.

Metric and config come from BASELINE.json ("samples/sec (whole node), 3-layer
MLP on synthetic MNIST, 1/2/4/8 workers").  One process per GPU (torchrun sets
RANK/LOCAL_RANK/WORLD_SIZE); each rank is one worker that

  1. receives its data shard (default: over the real gRPC data plane -- an
     in-process file server streams it as 1 MB ``Chunk``s to a ``ReceiveFile``
     handler, which parses each chunk in place into a pinned (hipHostMalloc) ring
     slot and hipMemcpyAsync's it into HBM, the worker's own ingest path; the
     JSON reports that stream's GB/s as ``ingest_gbps``, shard synthesis timed
     apart; ``--ingest local`` skips gRPC),
  2. trains the model with the hand-written HIP kernels (bf16 MFMA, fp32
     master weights, momentum SGD) -- every timed step is a full forward +
     backward + (RCCL all-reduce) + optimizer step,
  3. reports whole-job samples/s = global_batch * steps / max-over-ranks time.

``--model resnet18`` runs BASELINE config 4 instead (ResNet-18-shaped CNN on
synthetic CIFAR-shaped 32x32x3 data, implicit-GEMM convolutions), with the
gradient all-reduce bucketed and overlapped with backward.

Weak scaling: the per-GPU batch is fixed as N grows (MLP default 65,536 rows
per GPU; ``--batch 16384`` reproduces the smaller configuration).  The reference publishes
no number; ``vs_baseline`` is against the reference's derived
data-delivery ceiling of 25,478 samples/s per worker (BASELINE.md row
"Derived: data-delivery ceiling"), i.e. 25,478 * N.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

REF_CEILING_PER_WORKER = 25478.0
METRIC = "samples/sec (whole node), 3-layer MLP on synthetic MNIST, 1/2/4/8 workers"
METRIC_CNN = "samples/sec (whole node), ResNet-18-shaped CNN on synthetic CIFAR-shaped data, 1/2/4/8 workers"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--model", choices=["mlp", "resnet18"], default="mlp")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (MLP: multiple of 64)")
    ap.add_argument("--shard-batches", type=int, default=None, help="batches resident per worker shard")
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto")
    ap.add_argument("--unroll", type=int, default=0,
                    help="MLP: steps per hipGraph replay (each step still runs all its kernels on its own batch); "
                         "0 = the timed step count itself when <= 256 (one replay times exactly K steps), else 8")
    ap.add_argument("--ingest", choices=["grpc", "local", "device"], default="grpc",
                    help="grpc: file server -> ReceiveFile -> pinned ring -> HBM; local: host-generated shard; "
                         "device: shard synthesised in HBM by the Philox kernel (K8)")
    ap.add_argument("--bucket-mb", type=float, default=16.0, help="CNN all-reduce bucket size")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl (= RCCL over xGMI, the production path); gloo only to rehearse several ranks "
                         "sharing one GPU (RCCL refuses duplicate devices)")
    ap.add_argument("--allreduce", choices=["auto", "xgmi", "xgmi2", "pg"], default="auto",
                    help="MLP gradient all-reduce for N>1: xgmi = one-shot over IPC-mapped peer buffers fused "
                         "into the update kernel (hipGraph-capturable); xgmi2 = two-shot (reduce-scatter + "
                         "all-gather) through the same buffers; pg = the process group's all-reduce (RCCL); "
                         "auto = the fastest of the three, timed before the timed region")
    ap.add_argument("--autotune", type=int, default=6,
                    help="--allreduce auto with N>1: untimed steps per candidate (xGMI one-shot, xGMI two-shot, "
                         "the process group) before the timed region; the fastest is timed (0 = keep one-shot xGMI)")
    ap.add_argument("--oversubscribe", action="store_true",
                    help="allow --gpus N on fewer than N visible devices (ranks share GPUs: rehearsal only, "
                         "needs --dist-backend gloo)")
    ap.add_argument("--runtime", action="store_true",
                    help="train through the runtime roles instead of the bare engine: an in-process file "
                         "server, master and worker (gRPC control + data plane, the worker's hipGraph "
                         "chunks, its logging and feedback); 1 GPU")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="--runtime: steps per worker graph chunk (0: the runtime's default, config.py)")
    ap.add_argument("--settle", type=float, default=0.3,
                    help="after the timed region (1 GPU, graph mode): replay the same K-step graph back-to-back "
                         "for this many seconds and report the last replay as settled_* fields (informative; the "
                         "headline value is the timed region).  0 disables")
    ap.add_argument("--graph-collectives", action="store_true",
                    default=os.environ.get("SL_GRAPH_COLLECTIVES", "0") == "1",
                    help="N>1 with RCCL: capture the process group's collectives (the MLP all-reduce hook, the "
                         "ResNet bucket all-reduces) into the step hipGraph.  Opt-in, as in the runtime worker, "
                         "until a real multi-GPU run pins captured multi-rank RCCL; the default steps RCCL "
                         "eagerly (the xGMI exchange has no host collective and is always captured)")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args(argv)
    mlp = a.model == "mlp"
    a.steps = a.steps if a.steps is not None else (200 if mlp else 30)
    a.warmup = a.warmup if a.warmup is not None else (20 if mlp else 5)
    # MLP: 65,536 rows per GPU -- 1,024 row blocks, i.e. 4 per CU (16,384 leaves one per CU and the
    # step latency-bound); the shard (4 batches, 205 MB u8) is a sliver of the 288 GB of HBM.
    # ResNet-18: 1,024 images per GPU (82 K img/s vs 71 K at 512 and 54 K at 256 on one MI355X;
    # ~3 GB of activations).
    a.batch = a.batch or (65536 if mlp else 1024)
    a.unroll = a.unroll or (a.steps if a.steps <= 256 else 8)
    a.shard_batches = a.shard_batches or (4 if mlp else 4)
    a.lr = a.lr if a.lr is not None else (0.05 if mlp else 0.1)
    return a


class ReplicaDivergence(RuntimeError):
    """The replicas still differ after the re-timed fallback: no number may be reported."""


_T0 = time.perf_counter()


def _progress(msg: str) -> None:
    """SL_BENCH_PROGRESS=1: one stderr line per phase (diagnosing slow or stuck multi-rank runs)."""
    if os.environ.get("SL_BENCH_PROGRESS") == "1":
        print(f"[bench rank {os.environ.get('RANK', '0')} +{time.perf_counter() - _T0:.1f}s] {msg}",
              file=sys.stderr, flush=True)


def verify_replicas(check, retime, exchange_failed=lambda: False):
    """The N>1 safety net, for EVERY gradient-exchange path (xGMI one-/two-shot, RCCL captured or
    eager, gloo).  ``check()`` is True iff every replica holds bit-identical weights (decided by an
    all-reduce, so every rank takes the same branch); ``exchange_failed()`` is True iff the xGMI
    exchange recorded a barrier timeout on any rank.  On either failure ``retime()`` re-syncs every
    rank from rank 0 and times the K steps again with the process group's all-reduce, uncaptured,
    returning the new elapsed time.  Returns (replicas_identical, fallback reason or None, re-timed
    elapsed or None); raises :class:`ReplicaDivergence` when the replicas differ even then.

    The reference applies a gossip reply even when the RPC failed (/root/reference/src/worker.cc:153-165);
    this is the guard against the data-parallel version of that failure mode."""
    ok, failed = check(), exchange_failed()
    if ok and not failed:
        return True, None, None
    reason = "barrier timeout" if failed else "replicas diverged"
    elapsed = retime()
    if not check():
        raise ReplicaDivergence(f"{reason}; the replicas still diverge after re-timing with the uncaptured "
                                "process-group all-reduce")
    return True, reason, elapsed


def _free_port() -> int:
    from serverless_learn_amd.utils.ports import reserve_port

    return reserve_port()


def visible_devices() -> int:
    """GPUs this process could use.  ``torch.cuda.device_count()`` does not initialise the
    GPU on this image, so the launcher parent stays GPU-free before it spawns its ranks."""
    import torch

    return int(torch.cuda.device_count())


def launch_ranks(args, argv) -> int:
    """``--gpus N`` without a launcher: spawn N rank processes (one per GPU, the same
    command line under ``torch.distributed.run``) and exit with their status.  Nothing
    here touches the GPU, so the children are started from a parent that never
    initialised HIP.  Rank 0 prints the one JSON line; it reaches our stdout unchanged.

    The reference starts one ``worker ADDR`` process per worker by hand
    (/root/reference/src/worker.cc:233-258); this is the benchmark's equivalent."""
    import subprocess

    n_dev = visible_devices()
    if n_dev < args.gpus and not args.oversubscribe:
        print(f"bench.py: --gpus {args.gpus} but only {n_dev} GPU(s) visible; refusing to report a "
              f"{args.gpus}-GPU number (pass --oversubscribe --dist-backend gloo to rehearse ranks "
              "sharing GPUs)", file=sys.stderr)
        return 2
    if n_dev < args.gpus and args.dist_backend != "gloo":
        print("bench.py: --oversubscribe needs --dist-backend gloo (RCCL refuses ranks sharing a device)",
              file=sys.stderr)
        return 2
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    env["SL_BENCH_LAUNCHED"] = "1"
    # ranks sharing a GPU (rehearsal): keep their hardware queues within the GPU's budget
    from serverless_learn_amd.utils.gpu_share import share_gpu_env

    share_gpu_env(env, -(-args.gpus // max(n_dev, 1)))
    p = subprocess.run(cmd, env=env)
    return p.returncode


def record(args, *, world, elapsed, model_name, n_params, use_graph, collective, first_loss, st, t_ingest,
           ingest_stats, replicas_identical, n_dev) -> dict:
    """The one JSON line (driver contract: whole-job value, max-over-ranks time)."""
    import torch.distributed as dist

    mlp = args.model == "mlp"
    B = args.batch
    global_batch = B * world
    value = global_batch * args.steps / elapsed
    out = {
        "metric": METRIC if mlp else METRIC_CNN,
        "value": round(value, 1),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / (REF_CEILING_PER_WORKER * world), 2),
        "dtype": "bf16",
        "data": f"synthetic (seeded {'MNIST' if mlp else 'CIFAR'}-shaped u8 shards, random-init weights)",
        "config": {
            "model": model_name,
            "params": n_params,
            "global_batch": global_batch,
            "per_gpu_batch": B,
            "seq_len": None,
            "parallelism": f"dp{world}",
            "optimizer": f"sgd(lr={args.lr}, momentum={args.momentum}) fp32 master",
            "hipgraph": use_graph,
            "steps_per_graph": (args.unroll if mlp else 1) if use_graph else 0,
            "ingest": args.ingest,
            "collective_backend": collective,
        },
        "baseline_note": "reference publishes no number; vs_baseline is vs its derived data-delivery "
                         "ceiling of 25,478 samples/s/worker (BASELINE.md)",
        "train_loss_first": None if first_loss is None else round(first_loss, 4),
        "train_loss_last": round(st.loss, 4),
        "train_acc_last": round(st.accuracy, 4),
        "ingest_s": round(t_ingest, 3),
        "ingest": ingest_stats or None,
        "ingest_gbps": ingest_stats.get("gbps"),
        "replicas_identical": replicas_identical,
        "dist": {
            "world_size": dist.get_world_size() if world > 1 else 1,
            "backend": dist.get_backend() if world > 1 else None,
            "collective_backend": collective,
            "devices_visible": n_dev,
            "ranks_share_gpus": world > n_dev,
            "launcher": "bench.py" if os.environ.get("SL_BENCH_LAUNCHED") else ("torchrun" if world > 1 else None),
        },
    }
    return out


def runtime_bench(args, dev) -> tuple[float, dict, object]:
    """``--runtime``: the reference's three roles end-to-end on this GPU (file_server.cc,
    master.cc, worker.cc).  The file server streams the shard to the worker over gRPC, the
    master tracks it, and the worker trains from hipGraph chunks on its own thread with its
    periodic logs / group metrics / feedback.  ``Worker.hold_at`` pauses it exactly at a step
    once its device work has drained: hold at W, release to W + K, and the K steps between
    are timed.  Returns (seconds, runtime info, the worker's trainer)."""
    from serverless_learn_amd.proto import messages as pb
    from serverless_learn_amd.config import Config
    from serverless_learn_amd.runtime.local_cluster import LocalCluster, fast_config

    cfg = fast_config(device=str(dev), model=args.model, batch=args.batch,
                      shard_records=args.batch * args.shard_batches, log_every=64,
                      graph_steps=args.graph_steps or Config().graph_steps,
                      lr=args.lr, momentum=args.momentum, rpc_timeout_s=30.0, checkup_interval_ms=500,
                      dataset="synthetic-mnist" if args.model == "mlp" else "synthetic-cifar")
    c = LocalCluster(cfg)
    w = None
    try:
        w = c.add_worker(sync="none")
        t_ingest = time.perf_counter()
        w.hold_at = args.warmup
        if not c.wait_for(lambda: w.held_step == args.warmup, 600, interval=0.001):
            raise RuntimeError(f"runtime worker never reached warmup step {args.warmup} (state {w.state})")
        t_ingest = time.perf_counter() - t_ingest
        t0 = time.perf_counter()
        w.hold_at = args.warmup + args.steps
        if not c.wait_for(lambda: w.held_step == args.warmup + args.steps, 600, interval=0.0002):
            raise RuntimeError(f"runtime worker stalled at step {w.step} (state {w.state})")
        elapsed = time.perf_counter() - t0
        fb = pb.FlowFeedback.FromString(w._check_up(pb.PeerList().SerializeToString(), None))
        info = {"roles": ["file_server", "master", "worker"], "worker_graph_chunks": w.graph_chunks,
                "worker_feedback_samples_per_sec": round(fb.samples_per_sec, 1),
                "master_job": c.master.job_metrics(), "bytes_ingested": w.bytes_ingested,
                "warmup_incl_shard_s": round(t_ingest, 3), "log_every": cfg.log_every,
                "graph_steps": cfg.graph_steps}
        return elapsed, info, w.trainer
    finally:
        if w is not None:
            w.hold_at = None
        c.stop()


def main(argv=None) -> int:
    args = parse(argv)
    if args.runtime and args.gpus != 1:
        print("bench.py: --runtime runs the roles in one process on one GPU (--gpus 1)", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, argv)

    import torch
    import torch.distributed as dist

    from serverless_learn_amd.data.synthetic import decode_shard, make_shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)
        return 2
    n_dev = visible_devices()
    if n_dev < 1:
        print("bench.py: no GPU visible", file=sys.stderr)
        return 2
    if local_rank >= n_dev and not (args.oversubscribe and args.dist_backend == "gloo"):
        print(f"bench.py: local rank {local_rank} but only {n_dev} GPU(s) visible (ranks would share a "
              "device; pass --oversubscribe --dist-backend gloo to rehearse that)", file=sys.stderr)
        return 2
    local_dev = local_rank % n_dev
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    mlp = args.model == "mlp"
    if args.runtime:
        elapsed, rt_info, tr = runtime_bench(args, dev)
        out = record(args, world=1, elapsed=elapsed,
                     model_name="mlp-784-256-256-10" if mlp else "resnet18-cifar (11.17M params)",
                     n_params=tr.n_params if mlp else tr.spec.n_logical, use_graph=True, collective=None, first_loss=None, st=tr.stats(),
                     t_ingest=rt_info["warmup_incl_shard_s"], ingest_stats={}, replicas_identical=None, n_dev=n_dev)
        out["config"]["ingest"] = "grpc (file server role)"
        out["config"]["mode"] = "runtime"
        out["config"]["steps_per_graph"] = rt_info["graph_steps"]
        out["runtime"] = rt_info
        print(json.dumps(out), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(json.dumps(out) + "\n")
        return 0
    dataset = "synthetic-mnist" if mlp else "synthetic-cifar"
    B = args.batch
    n_records = B * args.shard_batches

    # ---- 1. shard delivery -------------------------------------------------
    ingest_stats: dict = {}
    t_ingest = time.perf_counter()
    if args.ingest == "device":
        from serverless_learn_amd.data.device_synth import synth_on_device

        x, y = synth_on_device("mnist" if mlp else "cifar", n_records, seed=rank, device=dev)
    elif args.ingest == "grpc":
        # the north-star data plane: the file server streams the shard as 1 MB Chunks, the
        # receiving handler parses each in place into a pinned ring slot and hipMemcpyAsync's
        # it into HBM (csrc/core/ingest.cpp); x / y are views of that device buffer
        from serverless_learn_amd.data.synthetic import HEADER_SIZE, decode_header
        from serverless_learn_amd.runtime.local_cluster import fetch_shard_via_grpc

        buf = fetch_shard_via_grpc(n_records=n_records, shard_index=rank, num_shards=world, seed=0,
                                   dataset=dataset, device=local_dev, stats=ingest_stats)
        hdr = decode_header(buf[:HEADER_SIZE].cpu().numpy().tobytes())
        n, d = hdr["n"], hdr["height"] * hdr["width"] * hdr["channels"]
        x = buf[HEADER_SIZE:HEADER_SIZE + n * d].view(n, d)
        y = buf[HEADER_SIZE + n * d:HEADER_SIZE + n * d + n]
    else:
        host_buf = make_shard(n_records, shard_index=rank, num_shards=world, seed=0, dataset=dataset)
        hdr, images, labels = decode_shard(bytearray(host_buf))
        x = torch.from_numpy(images).pin_memory().to(dev, non_blocking=True)
        y = torch.from_numpy(labels.copy()).pin_memory().to(dev, non_blocking=True)
    torch.cuda.synchronize()
    t_ingest = time.perf_counter() - t_ingest
    _progress(f"shard ready ({n_records} records)")

    # ---- 2. engine ----------------------------------------------------------
    if mlp:
        from serverless_learn_amd.models.mlp import FusedMLPTrainer, N_PARAMS

        tr = FusedMLPTrainer(batch=B, device=dev, lr=args.lr, momentum=args.momentum, world_size=world, seed=0)
        n_params, model_name = N_PARAMS, "mlp-784-256-256-10"
        if os.environ.get("SL_CLOCK_PROBE") == "1":  # diagnostics: per-step wall time + shader clock
            tr.enable_clock_probe()
    else:
        from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer

        tr = FusedResNetTrainer(batch=B, device=dev, lr=args.lr, momentum=args.momentum, world_size=world, seed=0)
        n_params, model_name = tr.spec.n_logical, "resnet18-cifar (11.17M params)"
    xg = None
    collective = None
    if world > 1:
        # identical start: broadcast rank 0's weights
        flat = tr.get_flat()
        dist.broadcast(flat, 0)
        tr.set_flat(flat)
        collective = "rccl" if args.dist_backend == "nccl" else "gloo"
        if mlp and args.allreduce in ("auto", "xgmi", "xgmi2"):
            from serverless_learn_amd.parallel.xgmi import XgmiExchange, dist_collectives, probe

            try:
                bad = probe(rank, world, dev, *dist_collectives())
                if bad:
                    raise RuntimeError("exchange probe failed: " + bad)
                xg = XgmiExchange(tr.n_pad, rank, world, dev, *dist_collectives(),
                                  two_shot=args.allreduce == "xgmi2")
                tr.enable_xgmi(xg)
                collective = "xgmi-ipc-two-shot" if xg.two_shot else "xgmi-ipc"
            except RuntimeError as e:
                if args.allreduce in ("xgmi", "xgmi2"):
                    raise
                print(f"xgmi all-reduce unavailable, using the process group: {e}", file=sys.stderr)
        if mlp and xg is None:
            tr.allreduce = lambda g: dist.all_reduce(g)
        else:
            tr.bucket_bytes = int(args.bucket_mb * (1 << 20))
            tr.bucket_hook = lambda view: dist.all_reduce(view, async_op=True)
            tr.bucket_wait = lambda handles: [h.wait() for h in handles]
    tr.load_shard(x, y)
    _progress("engine ready")

    # the xGMI exchange needs no host sync, so the N>1 MLP step is graph-captured like N=1; RCCL
    # collectives (the MLP all-reduce hook, the ResNet bucket all-reduces and their waits) are
    # stream-ordered device work and are captured into the step graph as well
    # (tests/test_rccl_gpu.py: captured RCCL steps bit-identical to the hook-free step).  gloo
    # collectives run on the host and keep the eager step.
    graph_pg = args.dist_backend == "nccl" and (world == 1 or args.graph_collectives)
    use_graph = args.graph == "on" or (args.graph == "auto" and (world == 1 or xg is not None or graph_pg))
    warm_eager = min(args.warmup, 3)
    for i in range(warm_eager):
        tr.step()
        _progress(f"eager warm-up step {i + 1}")
    run = getattr(tr, "steps", None) or (lambda n: [tr.step() for _ in range(n)])
    if use_graph:
        try:
            if mlp:
                tr.capture(warmup=0, unroll=args.unroll)
            else:
                tr.capture(warmup=0)
        except RuntimeError as e:
            if not (graph_pg and world > 1 and xg is None):
                raise
            # a multi-rank RCCL capture the runtime refuses: the timed steps run eagerly
            print(f"RCCL step capture failed, stepping eagerly: {e}", file=sys.stderr)
            tr.drop_graphs()
            graph_pg = use_graph = False

    def upload_graph():
        # upload the K-step executable graph before the clock starts, as any graph about to be
        # replayed in a loop is (hipGraphUpload); otherwise its first replay pays the upload
        if not (use_graph and mlp and getattr(tr, "graph_unrolled", None) is not None and args.steps <= args.unroll):
            return
        try:
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            rc = hip.hipGraphUpload(ctypes.c_void_p(tr.graph_unrolled.raw_cuda_graph_exec()),
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            if rc != 0:
                print(f"hipGraphUpload failed ({rc})", file=sys.stderr)
        except (AttributeError, OSError) as e:
            print(f"graph upload unavailable: {e}", file=sys.stderr)
        torch.cuda.synchronize()

    # SL_BENCH_PRELOAD=1 moves the one-time host work (the first tr.stats() loads torch's
    # reduction kernels lazily: the GPU sits idle ~27 ms there, profiles/r04_a/tr20; the graph
    # upload) before the last warm-up steps instead of after them.  Same-box A/B: no gain
    # (484-496 M vs 496-505 M, profiles/r04_c), so the default keeps the round-3 order.  The
    # warm-up is exactly --warmup steps either way.
    preload = os.environ.get("SL_BENCH_PRELOAD") == "1"
    if preload:
        torch.cuda.synchronize()
        first_loss = tr.stats().loss  # after the eager warm-up steps
        upload_graph()
    run(args.warmup - warm_eager)
    _progress("warm-up done")
    if not preload:
        torch.cuda.synchronize()
        first_loss = tr.stats().loss
        upload_graph()

    def pg_mode(captured: bool = True):
        nonlocal graph_pg
        tr.enable_xgmi(None)
        tr.drop_graphs()
        tr.allreduce = lambda g: dist.all_reduce(g)
        tr.step()  # eager first: anything lazily set up by the collective happens outside capture
        if captured and use_graph and graph_pg:
            try:
                tr.capture(warmup=0, unroll=args.unroll)
                return getattr(tr, "steps", None) or (lambda n: [tr.step() for _ in range(n)])
            except RuntimeError as e:  # a multi-rank RCCL capture the runtime refuses: eager steps
                print(f"RCCL step capture failed, stepping eagerly: {e}", file=sys.stderr)
                tr.drop_graphs()
                graph_pg = False
        return lambda n: [tr.step() for _ in range(n)]

    autotune = None
    if xg is not None and args.allreduce == "auto" and args.autotune > 0:
        # the xGMI exchange is validated on ranks sharing one GPU; on a real node its speed
        # depends on the peer links, so time a few untimed steps of it against the process
        # group's all-reduce and keep the faster (max over ranks decides, identically everywhere)
        def clock(fn, n):
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn(n)
            torch.cuda.synchronize()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item()) / n
        def xgmi_mode(two_shot: bool):
            xg.two_shot = two_shot
            tr.enable_xgmi(xg)
            tr.allreduce = None
            if use_graph:
                tr.capture(warmup=0, unroll=args.unroll)
            fn = getattr(tr, "steps", None) or (lambda n: [tr.step() for _ in range(n)])
            fn(2)
            return fn
        # the graph candidates are timed as the timed region runs them: one replay of the
        # k-step graph (a run of single-step replays behaves differently, e.g. with ranks
        # sharing a GPU)
        n_at = args.unroll if use_graph and args.unroll <= 256 else args.autotune
        t_x = clock(run, n_at)
        run_x2 = xgmi_mode(True)
        t_x2 = clock(run_x2, n_at)
        run_pg = pg_mode()
        pg_graph = use_graph and graph_pg
        run_pg(2)
        n_pg = n_at if pg_graph else args.autotune
        t_p = clock(run_pg, n_pg)
        autotune = {"xgmi_ms": round(t_x * 1e3, 4), "xgmi_two_shot_ms": round(t_x2 * 1e3, 4),
                    "pg_ms": round(t_p * 1e3, 4), "pg_hipgraph": pg_graph, "steps": n_at, "pg_steps": n_pg}
        if t_p < min(t_x, t_x2):
            run, use_graph = run_pg, pg_graph
            collective = "rccl" if args.dist_backend == "nccl" else "gloo"
            xg_keep = xg
            xg = None
        else:
            run = xgmi_mode(t_x2 < t_x)
            collective = "xgmi-ipc-two-shot" if xg.two_shot else "xgmi-ipc"
        torch.cuda.synchronize()

    # ---- 3. timed region ----------------------------------------------------
    def timed() -> float:
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(args.steps)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    force = os.environ.get("SL_BENCH_FORCE_DIVERGE", "")  # tests: "once" / "always" (rank 1 drifts)
    n_checks = [0]

    def replicas_agree() -> bool:
        # every replica must hold the same weights after lock-step DP (checks the exchange too)
        n_checks[0] += 1
        if rank == 1 and (force == "always" or (force == "once" and n_checks[0] == 1)):
            f = tr.get_flat()
            f[0] += 1.0
            tr.set_flat(f)
        ck = tr.get_flat().double()
        lo, hi = ck.clone(), ck.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        return bool(torch.equal(lo, hi))

    if autotune is not None:
        upload_graph()  # the autotune re-captured the chosen mode's graph
    _progress("timed region starts")
    if os.environ.get("SL_BENCH_PROGRESS") == "1" and not (use_graph and mlp):
        run_inner = run

        def run(n):  # diagnostics only: one synchronised step at a time, one line each
            for i in range(n):
                run_inner(1)
                torch.cuda.synchronize()
                _progress(f"step {i + 1} of {n}")
    elapsed = timed()
    _progress(f"timed region done ({elapsed:.3f} s)")
    st_timed = tr.stats()
    replicas_identical, fallback = None, None
    if world > 1:
        def exchange_failed() -> bool:
            bad = torch.tensor([1.0 if (xg is not None and xg.error()) else 0.0], device=dev)
            dist.all_reduce(bad, op=dist.ReduceOp.MAX)
            return bad.item() > 0

        def retime() -> float:
            # never report a number from a broken exchange or diverged replicas: re-sync from rank 0,
            # switch to the process group's all-reduce WITHOUT graph capture and time the K steps again
            nonlocal run, use_graph, collective, st_timed
            print("bench.py: gradient exchange check failed; re-timing with the uncaptured process group",
                  file=sys.stderr)
            flat = tr.get_flat()
            dist.broadcast(flat, 0)
            tr.set_flat(flat)
            if mlp:
                run = pg_mode(captured=False)
            else:  # the bucket hooks stay; only the captured step goes
                tr.drop_graphs()
                run = lambda n: [tr.step() for _ in range(n)]  # noqa: E731
            use_graph, collective = False, ("rccl" if args.dist_backend == "nccl" else "gloo")
            run(3)
            t = timed()
            st_timed = tr.stats()
            return t

        try:
            replicas_identical, fallback, re_elapsed = verify_replicas(replicas_agree, retime, exchange_failed)
        except ReplicaDivergence as e:
            print(f"bench.py: {e}; no number reported", file=sys.stderr)
            return 2
        if re_elapsed is not None:
            elapsed = re_elapsed
    settled = None
    if world == 1 and use_graph and args.settle > 0:
        # Informative only: the same K-step replay, back-to-back for args.settle seconds, then
        # one replay timed the same way.  The gap to the headline is the GPU clock still ramping
        # up from the idle ingest when the timed region starts (profiles/r03_final2).
        t_end = time.perf_counter() + args.settle
        while time.perf_counter() < t_end:
            run(args.steps)
        settled = timed()
    out = record(args, world=world, elapsed=elapsed, model_name=model_name, n_params=n_params,
                 use_graph=use_graph, collective=collective, first_loss=first_loss, st=st_timed,
                 t_ingest=t_ingest, ingest_stats=ingest_stats, replicas_identical=replicas_identical, n_dev=n_dev)
    if settled:
        out["settled_ms_per_step"] = round(settled / args.steps * 1e3, 4)
        out["settled_samples_per_s"] = round(args.batch * args.steps / settled, 1)
    if fallback:
        out["replica_fallback"] = fallback
    if getattr(tr, "probe", None) is not None:
        # per step: wall us between consecutive probes and the shader clock over it (GHz), per XCD
        # where both probes ran a workgroup on that XCD (median over those XCDs)
        import statistics
        steps = tr.clock_probe_steps()
        iv = []
        for (w0_, t0), (w1_, t1) in zip(steps, steps[1:]):
            ghz = [(t1[x][0] - t0[x][0]) / max(1, t1[x][1] - t0[x][1]) * 0.1 for x in t0 if x in t1]
            iv.append([round((w1_ - w0_) / 100.0, 2), round(statistics.median(ghz), 3) if ghz else None])
        w0 = args.warmup  # steps before the timed region
        out["clock_probe"] = {"n": len(steps), "timed_from": w0, "intervals_us_ghz": iv[:w0 + args.steps + 40]}
    if autotune:
        out["allreduce_autotune"] = autotune
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        for ex in (xg, locals().get("xg_keep")):
            if ex is not None:
                ex.close()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
