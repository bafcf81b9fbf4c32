"""In-process cluster helpers (tests, benchmarks, examples).

``LocalCluster`` starts a master and a file server on ephemeral localhost ports
and any number of workers, all in one process -- the "plumbing" configuration
of BASELINE.json config 1.  ``fetch_shard_via_grpc`` is what ``bench.py`` uses
to deliver a worker's shard over the real data plane before timing starts.
"""
from __future__ import annotations

import threading
import time

import numpy as np

from ..config import Config
from ..proto import messages as pb
from ..wire.codec import chunk_payload
from .file_server import FILE_NUM_MD, FileServer
from .master import Master
from .transport import RpcServer, metadata_dict
from .worker import Worker


def fast_config(**kw) -> Config:
    base = dict(master_addr="127.0.0.1:0", file_server_addr="127.0.0.1:0", checkup_interval_ms=200,
                push_interval_ms=200, gossip_interval_ms=200, simulated_train_interval_ms=100,
                rpc_timeout_s=2.0, max_misses=2, device="cpu", batch=256, shard_records=2048, log_every=10)
    base.update(kw)
    return Config.from_env(**base)


class LocalCluster:
    def __init__(self, cfg: Config | None = None):
        self.cfg = cfg or fast_config()
        self.file_server = FileServer(self.cfg, addr=self.cfg.file_server_addr).start()
        self.cfg.file_server_addr = self.file_server.addr
        self.master = Master(self.cfg, addr=self.cfg.master_addr).start()
        self.cfg.master_addr = self.master.addr
        self.workers: list[Worker] = []

    def add_worker(self, **overrides) -> Worker:
        import dataclasses

        cfg = dataclasses.replace(self.cfg, **overrides)
        w = Worker("127.0.0.1:0", cfg).start()
        self.workers.append(w)
        return w

    def wait_for(self, pred, timeout: float = 30.0, interval: float = 0.05) -> bool:
        t0 = time.monotonic()
        while time.monotonic() - t0 < timeout:
            if pred():
                return True
            time.sleep(interval)
        return False

    def stop(self) -> None:
        for w in self.workers:
            try:
                w.stop(leave=False)
            except Exception:
                pass
        self.master.stop()
        self.file_server.stop()


class _Sink:
    """A minimal Worker-API endpoint that collects one pushed file.

    ``device`` >= 0: the file lands the way a GPU worker lands shards -- every ``Chunk`` is
    parsed in place into a pinned (hipHostMalloc) ring slot and shipped to HBM with
    hipMemcpyAsync on the ring's own stream (csrc/core/ingest.cpp) -- and ``data`` is a
    device tensor.  Otherwise the bytes land in host memory."""

    def __init__(self, device: int = -1):
        self.data = None
        self.device = device
        self.stream_s = 0.0
        self.pinned = False
        self.done = threading.Event()
        self.server = RpcServer("127.0.0.1:0", max_workers=4)
        self.server.add_service("Worker", {"ReceiveFile": self._recv,
                                           "CheckUp": lambda r, c: pb.FlowFeedback().SerializeToString(),
                                           "ExchangeUpdates": lambda r, c: r})
        self.server.start()

    def _recv(self, requests, context):
        md = metadata_dict(context)
        size = int(md.get("sl-file-size", "-1"))
        from .._core import core

        t0 = None
        if size > 0:
            ring = core().IngestRing(4 << 20, 4, self.device)
            if self.device >= 0:
                import torch

                buf = torch.empty(size, dtype=torch.uint8, device=torch.device("cuda", self.device))
                ring.begin(buf.data_ptr(), size, True)
            else:
                buf = np.empty(size, np.uint8)
                ring.begin(buf.ctypes.data, size, False)
            for m in requests:
                if t0 is None:
                    t0 = time.perf_counter()
                ring.feed_chunk(m)
            ring.finish()
            self.pinned = bool(ring.pinned)
        else:
            t0 = time.perf_counter()
            buf = np.frombuffer(b"".join(bytes(chunk_payload(m)) for m in requests), np.uint8)
        self.stream_s = time.perf_counter() - (t0 or time.perf_counter())
        self.data = buf
        self.done.set()
        return pb.ReceiveFileAck(ok=True).SerializeToString()


def fetch_shard_via_grpc(n_records: int, shard_index: int = 0, num_shards: int = 1, seed: int = 0,
                         dataset: str = "synthetic-mnist", device: int = -1, stats: dict | None = None):
    """Serve shard ``shard_index`` from an in-process file server and receive it over gRPC.

    Returns host bytes, or -- with ``device`` >= 0 -- a uint8 device tensor that the pinned
    ingest ring landed in HBM.  ``stats`` (optional dict) receives the data-plane timing:
    ``gen_s`` (shard synthesis on the file server), ``stream_s`` (first chunk to last byte
    in HBM), ``bytes`` and ``gbps`` (bytes / stream_s)."""
    cfg = Config.from_env(file_server_addr="127.0.0.1:0", shard_records=n_records, num_shards=num_shards,
                          seed=seed, dataset=dataset)
    fs = FileServer(cfg, addr="127.0.0.1:0").start()
    sink = _Sink(device)
    try:
        from .transport import Channels

        t0 = time.perf_counter()
        fs.get_file(shard_index)  # synthesise first, so the push below times only the data plane
        gen_s = time.perf_counter() - t0
        ch = Channels()
        raw = ch.unary(fs.addr, "FileServer", "DoPush",
                       pb.Push(recipient_addr=sink.server.addr, file_num=shard_index).SerializeToString(),
                       timeout=600)
        if not pb.PushOutcome.FromString(raw).ok:
            raise RuntimeError("shard push failed")
        ch.close()
        nbytes = int(sink.data.numel() if device >= 0 else sink.data.size)
        if stats is not None:
            stats.update(gen_s=round(gen_s, 4), stream_s=round(sink.stream_s, 4), bytes=nbytes,
                         gbps=round(nbytes / max(sink.stream_s, 1e-9) / 1e9, 3), pinned=sink.pinned,
                         path="grpc Chunk stream -> pinned ring -> hipMemcpyAsync -> HBM" if device >= 0
                         else "grpc Chunk stream -> host")
        return sink.data if device >= 0 else sink.data.tobytes()
    finally:
        sink.server.stop()
        fs.stop()
