#!/usr/bin/env python3
"""Does gradient-bucket communication run beside the ResNet-18 backward?

One GPU, B = 1024 (the bench batch), eager steps so every launch goes to the stream it names.
The engine's bucket hook (models/resnet_engine.py: fired when a block's gradient range is
final) launches ``sl_comm_proxy`` -- a few-workgroup read-modify-write over a bucket-sized
scratch buffer, reading the gradient view, the footprint of a ring all-reduce's channel
workgroups -- on a side stream; the optimizer waits for it.  ``--mask-cus k`` runs the compute
on a stream whose CU mask leaves k CUs per XCD to other queues (hipExtStreamCreateWithCUMask).

Prints one JSON line with ms per step.  Run under ``rocprofv3 --kernel-trace --output-format
csv`` and feed the trace to profiles/r05_passes/probes/overlap_trace.py for the overlap fraction.
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def masked_stream(dev, free_per_xcd: int):
    """A compute stream that leaves the LAST ``free_per_xcd`` CUs of every XCD to other queues.
    The mask is one bit per CU in the device's CU order; the 256 CUs are 8 XCDs of 32."""
    hip = ctypes.CDLL("libamdhip64.so")
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    per = n_cu // 8
    bits = [0] * ((n_cu + 31) // 32)
    for cu in range(n_cu):
        if cu % per < per - free_per_xcd:
            bits[cu // 32] |= 1 << (cu % 32)
    mask = (ctypes.c_uint32 * len(bits))(*bits)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(bits)), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    return torch.cuda.ExternalStream(s.value, device=dev), sum(bin(b).count("1") for b in bits)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--proxy", action="store_true", help="bucket hooks launch the comm proxy")
    ap.add_argument("--nwg", type=int, default=16, help="proxy workgroups (a ring all-reduce's channels)")
    ap.add_argument("--passes", type=int, default=4, help="proxy read-modify-write passes per bucket")
    ap.add_argument("--bucket-mb", type=float, default=16.0)
    ap.add_argument("--mask-cus", type=int, default=0, help="CUs per XCD kept free of the compute stream")
    args = ap.parse_args()

    from serverless_learn_amd.data.device_synth import synth_on_device
    from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer
    from serverless_learn_amd.ops import _native as N

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    compute_cus = torch.cuda.get_device_properties(dev).multi_processor_count
    main_stream = torch.cuda.current_stream(dev)
    if args.mask_cus > 0:
        main_stream, compute_cus = masked_stream(dev, args.mask_cus)
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(main_stream):
        x, y = synth_on_device("cifar", args.batch * 4, seed=0, device=dev)
        tr = FusedResNetTrainer(batch=args.batch, device=dev)
        tr.load_shard(x, y)
        tr.bucket_bytes = int(args.bucket_mb * (1 << 20))
        # a bucket holds whole blocks' gradient ranges, so it can exceed bucket_bytes (ResNet-18's
        # last block alone is 18.9 MB): the scratch covers the whole gradient
        scratch = torch.zeros(tr.grad.numel() + 1024, device=dev)
        if args.proxy:
            def hook(view):
                n = view.numel() // 4 * 4
                if n > scratch.numel() or view.data_ptr() % 16:
                    raise RuntimeError(f"bucket of {n} floats does not fit the proxy scratch")
                ev = torch.cuda.Event()
                ev.record(main_stream)
                side.wait_event(ev)
                for _ in range(args.passes):
                    N.call("sl_comm_proxy", scratch.data_ptr(), view.data_ptr(), n, args.nwg, side.cuda_stream)
                return side

            def wait(handles):
                if handles:
                    main_stream.wait_stream(side)
            tr.bucket_hook, tr.bucket_wait = hook, wait
        for _ in range(args.warmup):
            tr.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tr.step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
    print(json.dumps({"ms_per_step": round(dt * 1e3, 4), "samples_per_s": round(args.batch / dt, 1), "proxy": args.proxy,
                      "nwg": args.nwg, "passes": args.passes, "bucket_mb": args.bucket_mb, "mask_cus_per_xcd": args.mask_cus,
                      "compute_cus": compute_cus, "loss": round(tr.stats().loss, 4)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
