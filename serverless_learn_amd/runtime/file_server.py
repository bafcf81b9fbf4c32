"""The file server: shard store + push-based data plane + checkpoint store.

Reference (/root/reference/src/file_server.cc, 165 LoC): one 100,000,000-byte
dummy "file 0" (:40-43, filled at :151-156); ``DoPush`` streams it to the
recipient in 1,000,000-byte ``Chunk``s synchronously inside the RPC
(:103-119, hot loop :69-76) and ``exit(1)``s the whole server on any other
file number (:107-110); ``CheckUp`` returns an empty ``LoadFeedback``
(:122-130).

Here:
* file ``n < CKPT_BASE`` is data shard ``n``: seeded synthetic MNIST-shaped
  records (:mod:`serverless_learn_amd.data.synthetic`), generated on first
  request and cached; with ``dataset="reference-dummy"`` file 0 is the
  reference's dummy file byte for byte (C++ ``reference_dummy_file``);
* files ``>= CKPT_BASE`` are checkpoints uploaded with the additive
  ``FileStore.StoreFile`` RPC (optionally persisted to ``store_dir``);
* an unknown file yields ``PushOutcome{ok=false}`` -- never an exit;
* chunks are zero-copy ``memoryview`` slices serialized by the C++ codec, the
  file number and size go along as call metadata, and pushes to different
  workers run concurrently (the gRPC pool), with per-call deadlines;
* ``CheckUp`` reports load (active pushes, bytes sent, files).
"""
from __future__ import annotations

import os
import threading
import time

from ..config import Config
from ..ckpt.format import CKPT_BASE
from ..data.synthetic import make_shard
from ..proto import messages as pb
from ..utils.log import Logger
from ..utils.metrics import Metrics
from ..wire.codec import chunk_payload, iter_chunks
from .transport import Channels, RpcFailure, RpcServer, metadata_dict

FILE_NUM_MD = "sl-file-num"
FILE_SIZE_MD = "sl-file-size"


class FileServer:
    def __init__(self, config: Config | None = None, addr: str | None = None):
        self.cfg = config or Config.from_env()
        self.addr_requested = addr or self.cfg.file_server_addr
        self.metrics = Metrics("file_server")
        self.log = Logger("file_server", self.addr_requested, self.metrics)
        self.channels = Channels(self.cfg.max_message_bytes, self.cfg.rpc_timeout_s, metrics=self.metrics)
        self._files: dict[int, bytes] = {}
        self._lock = threading.Lock()
        self._gen_locks: dict[int, threading.Lock] = {}
        self.active_pushes = 0
        self.bytes_sent = 0
        self.pushes_ok = 0
        self.pushes_failed = 0
        self.server: RpcServer | None = None
        if self.cfg.store_dir:
            os.makedirs(self.cfg.store_dir, exist_ok=True)
            self._load_store()

    # ---- file store ------------------------------------------------------
    def _load_store(self):
        for name in os.listdir(self.cfg.store_dir):
            if name.startswith("file_") and name.endswith(".bin"):
                num = int(name[5:-4])
                with open(os.path.join(self.cfg.store_dir, name), "rb") as f:
                    self._files[num] = f.read()

    def put_file(self, file_num: int, data: bytes) -> None:
        with self._lock:
            self._files[file_num] = data
        if self.cfg.store_dir:
            path = os.path.join(self.cfg.store_dir, f"file_{file_num}.bin")
            tmp = path + ".tmp"
            with open(tmp, "wb") as f:
                f.write(data)
            os.replace(tmp, path)

    def _num_shards(self) -> int:
        return self.cfg.num_shards if self.cfg.num_shards > 0 else 1 << 20

    def get_file(self, file_num: int) -> bytes | None:
        with self._lock:
            data = self._files.get(file_num)
            if data is not None:
                return data
            if file_num >= CKPT_BASE or file_num >= self._num_shards():
                return None
            if self.cfg.dataset == "reference-dummy" and file_num != 0:
                return None
            gl = self._gen_locks.setdefault(file_num, threading.Lock())
        with gl:  # generate outside the global lock; one generator per file
            with self._lock:
                if file_num in self._files:
                    return self._files[file_num]
            t0 = time.perf_counter()
            if self.cfg.dataset == "reference-dummy":
                from .._core import core

                data = core().reference_dummy_file(self.cfg.dummy_file_length)
            else:
                data = make_shard(self.cfg.shard_records, shard_index=file_num,
                                  num_shards=self.cfg.num_shards, seed=self.cfg.seed, dataset=self.cfg.dataset)
            with self._lock:
                self._files[file_num] = data
            self.log.info("file_ready", file_num=file_num, bytes=len(data), gen_s=round(time.perf_counter() - t0, 3))
            return data

    # ---- push (data plane) -------------------------------------------------
    def push(self, recipient: str, file_num: int, data=None) -> tuple[bool, int, str]:
        data = self.get_file(file_num) if data is None else data
        if data is None:
            return False, 0, f"unknown file {file_num}"
        with self._lock:
            self.active_pushes += 1
        try:
            md = ((FILE_NUM_MD, str(file_num)), (FILE_SIZE_MD, str(len(data))))
            # generous deadline: 1 s + 1 s per 100 MB at a pessimistic 100 MB/s
            timeout = max(self.cfg.rpc_timeout_s, 1.0 + len(data) / 100e6)
            raw = self.channels.stream_unary(recipient, "Worker", "ReceiveFile",
                                             iter_chunks(data, self.cfg.chunk_size), timeout=timeout, metadata=md)
            ok = pb.ReceiveFileAck.FromString(raw).ok
            if ok:
                with self._lock:
                    self.bytes_sent += len(data)
                    self.pushes_ok += 1
            return ok, len(data) if ok else 0, "" if ok else "recipient rejected file"
        except RpcFailure as e:
            with self._lock:
                self.pushes_failed += 1
            return False, 0, str(e)
        finally:
            with self._lock:
                self.active_pushes -= 1

    # ---- RPC handlers --------------------------------------------------------
    def _do_push(self, request: bytes, context) -> bytes:
        req = pb.Push.FromString(request)
        # time the stream on its own: a first request of a file also synthesises it (gen_s),
        # which is not data-plane throughput
        t0 = time.perf_counter()
        data = self.get_file(req.file_num)
        t1 = time.perf_counter()
        if data is None:
            ok, nbytes, err = False, 0, f"unknown file {req.file_num}"
        else:
            ok, nbytes, err = self.push(req.recipient_addr, req.file_num, data)
        dt = time.perf_counter() - t1
        (self.log.info if ok else self.log.warn)("push", to=req.recipient_addr, file_num=req.file_num, ok=ok,
                                                  bytes=nbytes, s=round(dt, 4), gen_s=round(t1 - t0, 4),
                                                  mb_s=round(nbytes / dt / 1e6, 1) if ok and dt > 0 else 0,
                                                  error=err)
        return pb.PushOutcome(ok=ok, bytes=nbytes, error=err).SerializeToString()

    def _check_up(self, request: bytes, context) -> bytes:
        with self._lock:
            fb = pb.LoadFeedback(active_pushes=self.active_pushes, bytes_sent=self.bytes_sent, files=len(self._files))
        return fb.SerializeToString()

    def _store_file(self, requests, context) -> bytes:
        md = metadata_dict(context)
        file_num = int(md.get(FILE_NUM_MD, "0"))
        parts = [bytes(chunk_payload(m)) for m in requests]
        data = b"".join(parts)
        if file_num < CKPT_BASE:
            return pb.PushOutcome(ok=False, error="uploads are restricted to checkpoint file numbers").SerializeToString()
        self.put_file(file_num, data)
        self.log.info("stored", file_num=file_num, bytes=len(data))
        return pb.PushOutcome(ok=True, bytes=len(data)).SerializeToString()

    def _list_files(self, request: bytes, context) -> bytes:
        with self._lock:
            items = sorted((k, len(v)) for k, v in self._files.items())
        return pb.FileList(file_nums=[k for k, _ in items], sizes=[s for _, s in items]).SerializeToString()

    # ---- lifecycle -------------------------------------------------------------
    def start(self) -> "FileServer":
        self.server = RpcServer(self.addr_requested, max_workers=32, max_message_bytes=self.cfg.max_message_bytes,
                                metrics=self.metrics)
        self.server.add_service("FileServer", {"DoPush": self._do_push, "CheckUp": self._check_up})
        self.server.add_service("FileStore", {"StoreFile": self._store_file, "ListFiles": self._list_files})
        self.server.start()
        self.addr = self.server.addr
        self.log.addr = self.addr
        if self.cfg.metrics_port > 0:
            self.metrics.serve(self.cfg.metrics_port)
        self.log.info("serving", dataset=self.cfg.dataset)
        return self

    def stop(self) -> None:
        self.metrics.close()
        if self.server:
            self.server.stop()
        self.channels.close()

    def wait(self) -> None:
        self.server.wait()
