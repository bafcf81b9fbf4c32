"""The worker: ingest, train, heartbeat, gossip -- an ephemeral member.

Reference (/root/reference/src/worker.cc, 258 LoC): ``worker ADDR`` starts its
gRPC service, a gossip thread (which divides by zero before any peer list
arrives, :200/:244), a "training" thread that bumps an empty vector every 2 s
(:221-231), then registers once without retry (:249-252).  ``ReceiveFile``
reads and discards every chunk (:49-61); ``CheckUp`` overwrites the peer list
(:64-77); ``ExchangeUpdates`` mixes the model (:81-100) -- all unsynchronized.

Here a worker:
* registers with retry/backoff, carrying an incarnation id (restart detection)
  and its GPU count;
* lands ``ReceiveFile`` chunks through the native pinned ring straight into
  HBM (data shards) or host memory (checkpoints), then swaps the resident
  shard into the trainer at a step boundary;
* trains the real model (``Config.model``: the MLP or the ResNet-18-shaped CNN):
  the hand-written HIP engines on MI355X (FusedMLPTrainer / FusedResNetTrainer) or the
  torch reference on CPU, or -- ``model="simulate"`` -- the reference's
  vector += 1 every ``simulated_train_interval_ms``;
* synchronizes per ``sync``: ``allreduce`` (RCCL/gloo group re-formed from the
  master's membership epochs, rank 0 broadcasting state after every re-form),
  ``gossip`` (exact reference exchange, random peer, never % 0), ``ps`` (the
  master's parameter server) or ``none``;
* answers ``CheckUp`` with real feedback (step, samples/s, loss, bytes, epoch)
  and checkpoints to the file server every ``checkpoint_every`` steps (rank 0).
"""
from __future__ import annotations

import os
import random
import socket
import sys
import threading
import time

import numpy as np
import torch

from .._core import core
from ..ckpt import format as ckfmt
from ..config import Config
from ..data.synthetic import HEADER_SIZE, MAGIC as SHARD_MAGIC, decode_header
from ..models import make_trainer
from ..parallel.dp import ElasticGroup, GroupBroken
from ..parallel.gossip import GossipState
from ..parallel.ps import PS_CLIENT_MD
from ..proto import messages as pb
from ..utils import trace
from ..utils.fault import FaultInjector
from ..utils.log import Logger
from ..utils.metrics import Metrics
from ..wire.codec import chunk_payload, decode_update, encode_update, iter_chunks
from .file_server import FILE_NUM_MD, FILE_SIZE_MD
from .transport import Channels, RpcFailure, RpcServer, metadata_dict


# RCCL: a collective timeout must raise (so the group can re-form) rather than
# tear the worker down -- the default handler aborts the process.
os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")


def resolve_device(spec: str) -> torch.device:
    if spec == "auto":
        return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(spec)


class ChunkBroken(GroupBroken):
    """A collective failed part-way through a step chunk: ``done`` steps completed first."""

    def __init__(self, done: int, cause: BaseException):
        super().__init__(str(cause))
        self.done, self.cause = done, cause


class Worker:
    def __init__(self, addr: str, config: Config | None = None):
        self.cfg = config or Config.from_env()
        self.addr_requested = addr
        self.addr = addr
        self.metrics = Metrics("worker")
        self.log = Logger("worker", addr, self.metrics)
        self.incarnation = (time.time_ns() ^ (os.getpid() << 20) ^ random.getrandbits(40)) & ((1 << 63) - 1)
        self.device = resolve_device(self.cfg.device)
        self.channels = Channels(self.cfg.max_message_bytes, self.cfg.rpc_timeout_s, metrics=self.metrics)
        self.fault = FaultInjector.from_env()
        self.train_lock = threading.RLock()
        self.view_lock = threading.Lock()
        self.view = {"epoch": 0, "peers": [], "rank": -1, "world": 0, "rendezvous": "", "resume_file": 0}
        self.trainer = None
        self.xgmi = None  # parallel.xgmi.XgmiExchange while an RCCL group of MLP workers is live
        self.gossip: GossipState | None = None
        backend = None if self.cfg.dp_backend == "auto" else self.cfg.dp_backend
        timeout = float(self.cfg.extra.get("dp_timeout_s", self.cfg.dp_timeout_s))
        self.group = ElasticGroup(backend=backend, device=self.device, timeout_s=timeout)
        self.step = 0
        self.samples = 0
        self.loss = float("nan")
        self.rate = 0.0
        self.group_metrics = {"samples_per_sec": 0.0, "loss": 0.0, "accuracy": 0.0, "world": 0}
        self.resumed_step = -1
        self._resume_pulled = 0   # PeerList.resume_file already pulled from the file server
        self.graph_chunks = 0     # graph replays run (tests / feedback)
        self._graph_collectives = False  # the captured step graphs hold the group's collectives
        # SURVEY §5.5 step-time breakdown, per log interval: wall ms per step, the loop's waits
        # per step, and one probed step's device phases (compute / exchange / update, exchange GB/s)
        self.phase_stats = {k: 0.0 for k in ("step_ms", "data_wait_ms", "compute_ms", "exchange_ms", "update_ms",
                                             "exchange_gbps")}
        self._wait_s = 0.0
        self._probe_due = True
        self._pending_phases = None
        self.hold_at = None       # pause training exactly at this step (bench.py --runtime, tests)
        self.held_step = -1       # step the worker is paused at, once its device work has drained
        self._agreed_epoch = -1   # newest membership epoch the whole lock-step group has agreed to see
        self._broken_since = None  # when the live group was first seen broken (monotonic s)
        self._agree_stream = None  # side stream of the epoch agreement on RCCL groups
        self._group_peers: list[str] = []  # membership of the group last formed (exchange abort on eviction)
        self.bytes_ingested = 0
        self._log_param_sum = os.environ.get("SL_LOG_PARAM_SUM", "0") == "1"
        self.files_received: list[int] = []
        self.state = "idle"
        self.registered = threading.Event()
        self._last_checkup = time.monotonic()
        self.has_data = threading.Event()
        self._pending_shard = None
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        dev_index = self.device.index if self.device.type == "cuda" else -1
        self.ring = core().IngestRing(4 << 20, 4, dev_index if dev_index is not None else 0)
        self.ring_lock = threading.Lock()  # one transfer through the ring at a time
        self.server: RpcServer | None = None
        self.ckpt_slot = 0
        if self.cfg.model == "simulate":
            # the reference's model: an empty vector of doubles, grown by gossip
            self.gossip = GossipState(torch.zeros(0, dtype=torch.float64), self.cfg.learn_rate,
                                      self.cfg.gossip_compat, growable=True)

    # ---- model -------------------------------------------------------------
    def _ensure_trainer(self):
        if self.trainer is not None or self.cfg.model == "simulate":
            return
        world = max(1, self.view["world"]) if self.cfg.sync == "allreduce" else 1
        kw = dict(batch=self.cfg.batch, lr=self.cfg.lr, momentum=self.cfg.momentum,
                  weight_decay=self.cfg.weight_decay, seed=self.cfg.seed, world_size=world)
        self.trainer = make_trainer(self.cfg.model, self.device, **kw)
        if self.cfg.sync in ("gossip", "ps"):
            self.gossip = GossipState(self._flat_view(), self.cfg.learn_rate, self.cfg.gossip_compat)

    def _flat_view(self) -> torch.Tensor:
        return self.trainer.params[:self.trainer.n_params]

    def _after_external_update(self):
        if self.trainer is not None:
            self.trainer.refresh_shadows()

    def _set_world(self, world: int):
        """Gradient scale follows the group size (mean over the global batch)."""
        if self.trainer is not None:
            self.trainer.set_world(world)

    # ---- RPC handlers --------------------------------------------------------
    def _receive_file(self, requests, context) -> bytes:
        md = metadata_dict(context)
        file_num = int(md.get(FILE_NUM_MD, "0"))
        size = int(md.get(FILE_SIZE_MD, "-1"))
        t0 = time.perf_counter()
        with self.ring_lock, trace.span("ingest", file_num=file_num):
            it = iter(requests)
            first = next(it, None)
            if first is None:
                return pb.ReceiveFileAck(ok=False).SerializeToString()
            head = bytes(chunk_payload(first)[:HEADER_SIZE])
            is_shard = head[:8] == SHARD_MAGIC
            try:
                if is_shard and size > 0 and self.device.type == "cuda":
                    buf = torch.empty(size, dtype=torch.uint8, device=self.device)
                    self.ring.begin(buf.data_ptr(), size, True)
                    self.ring.feed_chunk(first)
                    for msg in it:
                        self.ring.feed_chunk(msg)
                    got = self.ring.finish()
                elif size > 0:
                    arr = np.empty(size, dtype=np.uint8)
                    self.ring.begin(arr.ctypes.data, size, False)
                    self.ring.feed_chunk(first)
                    for msg in it:
                        self.ring.feed_chunk(msg)
                    got = self.ring.finish()
                    buf = arr
                else:  # a reference-style sender: no size metadata
                    parts = [bytes(chunk_payload(first))] + [bytes(chunk_payload(m)) for m in it]
                    buf = np.frombuffer(b"".join(parts), dtype=np.uint8)
                    got = buf.size
            except Exception as e:
                self.log.warn("ingest_failed", file_num=file_num, error=repr(e))
                return pb.ReceiveFileAck(ok=False).SerializeToString()
        if size > 0 and got != size:
            # a stream that ended early (sender died, deadline): the tail of the buffer is
            # uninitialised -- never train on it or ack it
            self.log.warn("ingest_short", file_num=file_num, announced=size, got=int(got))
            return pb.ReceiveFileAck(ok=False).SerializeToString()
        hdr = None
        if is_shard:
            try:
                hdr = decode_header(head)
                n, d = hdr["n"], hdr["height"] * hdr["width"] * hdr["channels"]
            except Exception as e:
                self.log.warn("ingest_bad_header", file_num=file_num, error=repr(e))
                return pb.ReceiveFileAck(ok=False).SerializeToString()
            if n <= 0 or d <= 0 or HEADER_SIZE + n * d + n > got:
                self.log.warn("ingest_bad_header", file_num=file_num, n=n, d=d, got=int(got))
                return pb.ReceiveFileAck(ok=False).SerializeToString()
        dt = time.perf_counter() - t0
        self.bytes_ingested += got
        self.files_received.append(file_num)
        kind = "data"
        if is_shard:
            if isinstance(buf, np.ndarray):
                buf = torch.from_numpy(buf)
            x = buf[HEADER_SIZE:HEADER_SIZE + n * d].view(n, d)
            y = buf[HEADER_SIZE + n * d:HEADER_SIZE + n * d + n]
            with self.train_lock:
                self._pending_shard = (x, y, file_num)
            self.has_data.set()
            kind = "shard"
        elif ckfmt.looks_like_checkpoint(buf[:8].tobytes() if isinstance(buf, np.ndarray) else b""):
            self._load_checkpoint(buf.tobytes())
            kind = "checkpoint"
        # else: opaque bytes (e.g. the reference dummy file) -- counted, then dropped, as worker.cc:54-56
        self.log.info("received_file", file_num=file_num, kind=kind, bytes=got, s=round(dt, 4),
                      mb_s=round(got / dt / 1e6, 1) if dt > 0 else 0, pinned=self.ring.pinned)
        return pb.ReceiveFileAck(ok=True).SerializeToString()

    def _check_up(self, request: bytes, context) -> bytes:
        pl = pb.PeerList.FromString(request)
        self._last_checkup = time.monotonic()
        with self.view_lock:
            self.view = {"epoch": pl.epoch, "peers": list(pl.peer_addrs), "rank": pl.rank,
                         "world": pl.world_size, "rendezvous": pl.rendezvous, "resume_file": pl.resume_file}
        ex = self.xgmi
        if ex is not None and pl.epoch > 0 and not set(self._group_peers) <= set(pl.peer_addrs):
            # a member of the live exchange was evicted (dead): release the queued consumers that
            # wait on it now -- the training thread is blocked on them, so it cannot do it itself
            # until the 10 s timeout (XgmiExchange.abort; the results since are void either way)
            ex.abort_once()
        gm = self.group_metrics
        fb = pb.FlowFeedback(step=self.step, samples_per_sec=self.rate,
                             loss=self.loss if self.loss == self.loss else 0.0,
                             bytes_ingested=self.bytes_ingested, epoch=self.group.epoch if self.group.epoch >= 0 else 0,
                             state=self.state, group_samples_per_sec=gm["samples_per_sec"],
                             group_loss=gm["loss"], group_accuracy=gm["accuracy"], group_world=gm["world"],
                             **self.phase_stats)
        return fb.SerializeToString()

    def _exchange_updates(self, request: bytes, context) -> bytes:
        delta = decode_update(request, "float64")
        with self.train_lock:
            if self.gossip is None:
                self._ensure_trainer()
            if self.gossip is None:  # allreduce/none worker asked to gossip: mix anyway
                self.gossip = GossipState(self._flat_view(), self.cfg.learn_rate, self.cfg.gossip_compat)
            with trace.span("gossip_serve", n=int(delta.size)):
                reply = self.gossip.serve(delta)
            self._after_external_update()
        return encode_update(reply)

    # ---- checkpoints -----------------------------------------------------------
    def _load_checkpoint(self, data: bytes) -> None:
        meta, params, mom, extra = ckfmt.decode_full(data)
        with self.train_lock:
            self._ensure_trainer()
            if self.trainer is None:
                return
            if meta.get("model", self.trainer.model_name) != self.trainer.model_name:
                self.log.warn("checkpoint_model_mismatch", ckpt=meta.get("model"), running=self.trainer.model_name)
                return
            if meta.get("step", 0) < self.step:
                self.log.info("checkpoint_skipped", ckpt_step=meta.get("step"), step=self.step)
                return
            self.trainer.set_flat(torch.from_numpy(params))
            if mom is not None and self.trainer.mom is not None:
                self.trainer.mom[:self.trainer.n_params].copy_(torch.from_numpy(mom))
            if extra and hasattr(self.trainer, "load_state_extra"):
                self.trainer.load_state_extra(extra)  # batch cursor, BN running statistics
            self.trainer.graph = None  # a captured graph holds the old state's launches
            self.step = int(meta.get("step", 0))
            self.resumed_step = self.step
            if self.gossip is not None:
                self.gossip.old.copy_(self._flat_view())
        self.log.info("checkpoint_loaded", step=self.step, epoch=meta.get("epoch"), extra=sorted(extra))

    def save_checkpoint(self) -> int:
        with self.train_lock:
            flat = self.trainer.get_flat().cpu().numpy()
            n = self.trainer.n_params
            mom = self.trainer.mom[:n].cpu().numpy() if self.trainer.mom is not None else None
            meta = {"model": self.trainer.model_name, "step": self.step, "epoch": self.group.epoch,
                    "layout": self.trainer.layout(),
                    "optimizer": {"lr": self.cfg.lr, "momentum": self.cfg.momentum}}
            extra = self.trainer.state_extra() if hasattr(self.trainer, "state_extra") else {}
        data = ckfmt.encode(flat, meta, mom, extra)
        file_num = ckfmt.CKPT_BASE + self.ckpt_slot
        self.ckpt_slot ^= 1  # two alternating slots: never overwrite one being served
        raw = self.channels.stream_unary(self.cfg.file_server_addr, "FileStore", "StoreFile", iter_chunks(data),
                                         timeout=max(10.0, self.cfg.rpc_timeout_s),
                                         metadata=((FILE_NUM_MD, str(file_num)),))
        if not pb.PushOutcome.FromString(raw).ok:
            raise RuntimeError("checkpoint upload rejected")
        self.channels.unary(self.cfg.master_addr, "MasterControl", "ReportCheckpoint",
                            pb.Push(recipient_addr=self.addr, file_num=file_num).SerializeToString())
        self.log.info("checkpoint_saved", step=self.step, file_num=file_num, bytes=len(data))
        return file_num

    # ---- loops -------------------------------------------------------------------
    def _register_once(self) -> bool:
        info = pb.WorkerBirthInfo(addr=self.addr, num_gpus=1 if self.device.type == "cuda" else 0,
                                  hostname=socket.gethostname(), incarnation=self.incarnation)
        raw = self.channels.unary(self.cfg.master_addr, "Master", "RegisterBirth", info.SerializeToString())
        return pb.RegisterBirthAck.FromString(raw).ok

    def _register_loop(self) -> None:
        """Register with retry/backoff, then keep watching the master's view of us.

        The reference registers once and never again (worker.cc:249-252).  Here a worker
        the master evicted (missed CheckUps during a network blip or a long stall) notices
        -- CheckUps stop for longer than the eviction window, or a PeerList arrives that no
        longer lists it -- and registers again (same incarnation: it is the same process,
        so the master treats it as a fresh join and bumps the epoch)."""
        delay = 0.1
        silence = max(2.0, self.cfg.max_misses * self.cfg.checkup_interval * 2.0 + self.cfg.rpc_timeout_s)
        while not self._stop.is_set():
            if not self.registered.is_set():
                try:
                    if self._register_once():
                        self._last_checkup = time.monotonic()
                        self.registered.set()
                        self.log.info("registered", master=self.cfg.master_addr)
                        delay = 0.1
                        continue
                except RpcFailure as e:
                    self.log.warn("register_retry", error=e.code.name if e.code else "", delay=delay)
                self._stop.wait(delay)
                delay = min(delay * 2, 5.0)
                continue
            self._stop.wait(min(1.0, silence / 4))
            with self.view_lock:
                dropped = self.view["epoch"] > 0 and self.view["rank"] < 0
            quiet = time.monotonic() - self._last_checkup > silence
            if dropped or quiet:
                self.log.warn("reregister", reason="not_in_peer_list" if dropped else "no_checkups",
                              silent_s=round(time.monotonic() - self._last_checkup, 2))
                with self.view_lock:
                    self.view = dict(self.view, epoch=0, rank=-1)
                self.registered.clear()

    def _ensure_resumed(self, resume_file: int) -> None:
        """Consume ``PeerList.resume_file``: a worker that has not trained yet (a fresh join,
        or a whole replacement group after every original member died) pulls the group's
        latest checkpoint from the file server before the group syncs state, so rank 0 never
        broadcasts untrained weights over a checkpoint the job already has.  The pull is the
        ordinary DoPush -> ReceiveFile path (the file server streams it into our ring and
        ``_load_checkpoint`` applies it); it does not depend on the master having pushed
        the checkpoint before the data."""
        if (not resume_file or resume_file == self._resume_pulled or self.step > 0
                or self.resumed_step >= 0 or self.cfg.model == "simulate"):
            return
        self._resume_pulled = resume_file
        req = pb.Push(recipient_addr=self.addr, file_num=resume_file).SerializeToString()
        try:
            raw = self.channels.unary(self.cfg.file_server_addr, "FileServer", "DoPush", req,
                                      timeout=max(60.0, self.cfg.rpc_timeout_s))
            ok = pb.PushOutcome.FromString(raw).ok
        except RpcFailure as e:
            ok = False
            self.log.warn("resume_pull_failed", file_num=resume_file, error=str(e))
        self.log.info("resume_pulled", file_num=resume_file, ok=ok, step=self.step)

    def _needs_regroup(self, v: dict) -> bool:
        """A live lock-step group (world > 1) switches epochs only at a step boundary every
        member agreed on (``_agree``): members learn of a join from their CheckUps at
        different times, and one that left while the others still ran steps would stall
        theirs (the xGMI barrier, RCCL) until a timeout.  A broken group, or a worker
        with no group, re-forms as soon as its view changes."""
        if v["epoch"] == 0 or v["rank"] < 0:
            return False
        if self.group.broken:
            if v["epoch"] == self.group.epoch and self.group.world > 1:
                # a collective failed but the view has not changed yet: most likely a member
                # died and the master will evict it within its miss window -- re-forming the
                # same membership now would only wait out the rendezvous timeout on the dead
                # peer.  Re-form the same epoch only once that window has passed.
                if self._broken_since is None:
                    self._broken_since = time.monotonic()
                window = (self.cfg.max_misses + 1) * self.cfg.checkup_interval + self.cfg.rpc_timeout_s
                return time.monotonic() - self._broken_since > window
            return True
        if v["epoch"] == self.group.epoch:
            return False
        if self.group.active and self.group.world > 1:
            return self._agreed_epoch > self.group.epoch and v["epoch"] >= self._agreed_epoch
        return True

    def _agree(self, have_data: bool | None = None):
        """One MAX all-reduce over the live group of [view epoch, -have_data]: returns
        (newest epoch any member sees, every member has data).  Posted asynchronously
        right after a step chunk is queued, so it overlaps the GPU work."""
        with self.view_lock:
            ep = float(self.view["epoch"])
        flags = [ep, -1.0 if (have_data is None or have_data) else 0.0]
        if self.group.backend != "nccl":
            t = torch.tensor(flags, dtype=torch.float64)
            work = self.group.allreduce_async(t, torch.distributed.ReduceOp.MAX)
        else:
            # RCCL: on a side stream of its own, so the collective does not queue behind the
            # step chunk just enqueued on the compute stream (it would then only complete when
            # the GPU has drained, and the next chunk could not be queued behind the current one)
            if self._agree_stream is None:
                self._agree_stream = torch.cuda.Stream(device=self.device)
            with torch.cuda.stream(self._agree_stream):
                t = torch.tensor(flags, dtype=torch.float64, device=self.device)
                work = self.group.allreduce_async(t, torch.distributed.ReduceOp.MAX)

        def result():
            if self.group.backend == "nccl":
                with torch.cuda.stream(self._agree_stream):  # the side stream waits for RCCL, then we read
                    self.group.wait(work)
                    v = t.cpu()
            else:
                self.group.wait(work)
                v = t
            return int(v[0]), bool(v[1] < -0.5)
        return result

    def _maybe_regroup(self) -> None:
        with self.view_lock:
            v = dict(self.view)
        if not self._needs_regroup(v):
            return
        self.state = "regrouping"
        self._broken_since = None
        self._drop_xgmi(healthy=not self.group.broken)
        self._ensure_resumed(v.get("resume_file", 0))
        with trace.span("regroup", epoch=v["epoch"], world=v["world"]):
            self._drop_graphs()  # a captured step may embed the old communicator
            # the drains above can take up to the exchange's peer timeout: form the view that is
            # current NOW, not the one read before them (a stale epoch's rendezvous waits out its
            # whole timeout for members that already moved on)
            with self.view_lock:
                now = dict(self.view)
            if now["epoch"] != v["epoch"]:
                v = now  # (same epoch: same membership; re-asking would restart the broken-group window)
                if not self._needs_regroup(v):
                    return
            epoch = v["epoch"]
            self._group_peers = list(v["peers"])
            ok = self.group.reform(v["epoch"], v["rank"], v["world"], v["rendezvous"],
                                   cancelled=lambda: self.view["epoch"] != epoch or self._stop.is_set())
            if not ok:
                self._stop.wait(0.2)
                return
            if self.group.active:
                # Every member must take part in the state broadcast, so a member whose
                # first shard has not arrived yet builds its (untrained) trainer now;
                # the shard is loaded into it later.
                with self.train_lock:
                    self._ensure_trainer()
                    self._set_world(max(1, v["world"]))
                    t = self.trainer
                    try:
                        bufs = t.buffers() if hasattr(t, "buffers") else []
                        self.group.sync_state([t.params, t.mom, *bufs])
                        step = torch.tensor([self.step], dtype=torch.int64, device=t.params.device)
                        self.group.broadcast_(step, 0)
                        self.step = int(step.item())
                    except GroupBroken as e:
                        self.log.warn("state_sync_failed", error=str(e))
                        return
                    self._after_external_update()
                    self._setup_xgmi()
            else:
                self._set_world(max(1, v["world"]))
        self._install_allreduce()
        self.state = "training"

    # ---- xGMI exchange (parallel/xgmi.py) -----------------------------------------
    def _xgmi_wanted(self) -> bool:
        """GPU MLP groups aggregate over xGMI.  RCCL groups always may; a gloo group of GPU
        workers (ranks sharing one GPU: the elastic rehearsal) only when ``SL_XGMI_GLOO=1``,
        as ``bench.py`` rehearses it."""
        from ..parallel import xgmi

        t = self.trainer
        if not (self.cfg.xgmi and t is not None and hasattr(t, "enable_xgmi") and self.device.type == "cuda"
                and 2 <= self.group.world <= xgmi.MAX_WORLD and xgmi.enabled()):
            return False
        return self.group.backend == "nccl" or os.environ.get("SL_XGMI_GLOO", "0") == "1"

    def _setup_xgmi(self) -> None:
        """MLP on a GPU group: aggregate through IPC-mapped exchange buffers over xGMI
        instead of an RCCL all-reduce per step.  Collective over the group; any rank that
        cannot map its peers makes every rank keep the process group's all-reduce."""
        from ..parallel import xgmi

        if not self._xgmi_wanted():
            return
        t = self.trainer
        hsize = int(xgmi.N.lib().sl_ipc_handle_size())
        gather = lambda b: self.group.allgather_fixed(b, hsize)  # noqa: E731
        try:
            bad = xgmi.probe(self.group.rank, self.group.world, self.device, gather, self.group.all_true)
            if bad:
                raise RuntimeError("exchange probe failed: " + bad)
            ex = xgmi.XgmiExchange(t.n_pad, self.group.rank, self.group.world, self.device,
                                   gather, self.group.all_true, two_shot=xgmi.default_two_shot(self.group.world))
        except (RuntimeError, GroupBroken) as e:
            self.log.warn("xgmi_unavailable", error=str(e))
            return
        self.xgmi = ex
        t.enable_xgmi(ex)
        self.log.info("xgmi_enabled", epoch=self.group.epoch, world=self.group.world, two_shot=ex.two_shot)

    def _drop_xgmi(self, healthy: bool = False) -> None:
        """Leave the exchange.  A peer may still have queued steps that read this rank's
        buffer or signal into it, so on a healthy group every member first drains its GPU
        and meets the others at a group barrier before unmapping; on a broken group (a peer
        died: its barrier timed out, later ones skip their wait) the local drain is all that
        can be done -- the survivors' queued steps finish within microseconds, and a dead
        peer's mapping keeps the freed memory alive until its process is gone."""
        ex, self.xgmi = self.xgmi, None
        if ex is None:
            return
        if not healthy:
            ex.abort_once()  # queued consumers stop waiting on the dead peer (else up to 10 s each drain)
        with self.train_lock:
            if self.trainer is not None and hasattr(self.trainer, "enable_xgmi"):
                self.trainer.enable_xgmi(None)
        torch.cuda.synchronize(self.device)
        closed_with_barrier = False
        if healthy and self.group.active:
            try:
                closed_with_barrier = self.group.all_true(not ex.error())
            except GroupBroken:
                pass
        ex.close(sync=False)
        self.log.info("xgmi_closed", epoch=self.group.epoch, barrier=closed_with_barrier)

    def _install_allreduce(self) -> None:
        """Gradient aggregation follows the group: set whenever a >1 group is live, cleared
        otherwise.  Called after every re-form and before every step chunk, so a trainer
        created after the group formed (first shard arriving late) still reduces its
        gradients.  With the xGMI exchange live the update kernel aggregates by itself: no
        hook.  Trainers with bucket hooks (the ResNet engine) launch one async all-reduce
        per bucket during backward instead of one blocking all-reduce after it."""
        t = self.trainer
        if t is None:
            return
        live = self.group.active and self.group.world > 1 and self.xgmi is None
        bucketed = hasattr(t, "bucket_hook")
        want = self.group.allreduce_ if live and not bucketed else None
        want_hook = self._bucket_hook if live and bucketed else None
        changed = t.allreduce != want or (bucketed and t.bucket_hook != want_hook)
        if changed:
            t.allreduce = want
            if bucketed:
                t.bucket_hook = want_hook
                t.bucket_wait = self._bucket_wait if want_hook else None
            if hasattr(t, "graph"):
                t.graph = None  # the captured step must be re-captured with (or without) the collective
                if hasattr(t, "graph_unrolled"):
                    t.graph_unrolled = None  # ... and so must the k-step graph
            self._set_world(max(1, self.group.world) if self.group.active and self.group.world > 1 else 1)

    def _drop_graphs(self) -> None:
        """Free the trainer's captured step graphs (the one-step and the k-step graph) after
        the device has drained them: they may hold the current communicator's kernels, so
        this runs before every re-form and teardown of the group.

        The drain must not wait on a collective whose peer is gone: the NCCL
        watchdog does not track collectives captured in a graph, and an eager all-reduce
        queued before a peer died only ends at the watchdog timeout.  So when the group is
        broken, or when the captured graphs hold collectives, the communicator is aborted
        FIRST (``ncclCommAbort`` releases the kernels waiting on the dead peer) and only then
        is the device drained; graphs of kernels only are drained directly."""
        t = self.trainer
        if t is None:
            return
        if self.group.active and (self.group.broken or self._graph_collectives):
            self.group.teardown()
        self._graph_collectives = False
        with self.train_lock:
            if hasattr(t, "drop_graphs"):
                t.drop_graphs()
            elif hasattr(t, "graph"):
                t.graph = None

    def _bucket_hook(self, view: torch.Tensor):
        return self.group.allreduce_async(view)

    def _bucket_wait(self, works) -> None:
        for w in works:
            if w is None:
                continue
            try:
                w.wait()
            except Exception as e:
                self.group.broken = True
                raise GroupBroken(repr(e)) from e

    # ---- training ------------------------------------------------------------------
    def _use_graph(self) -> bool:
        """hipGraph replay of whole steps: the fused GPU engines, with no host-side collective
        inside the step.  World 1 and the xGMI exchange have none; an RCCL group's all-reduce
        (the MLP hook, the ResNet bucket all-reduces and their stream waits) is device work
        ordered on the stream and is captured into the step graph with the kernels
        (tests/test_rccl_gpu.py).  A gloo group's collectives run on the host: eager steps.
        Capturing a multi-rank RCCL group's collectives is opt-in (``graph_collectives`` /
        ``SL_GRAPH_COLLECTIVES=1``): a peer failing inside a replayed graph does not reach
        ``_bucket_wait``'s GroupBroken path, so the elastic runtime steps eagerly by default.
        The captured graph embeds the communicator, so every re-form drops it
        (``_maybe_regroup`` -> ``_drop_graphs``)."""
        t = self.trainer
        if not (self.cfg.graph and self.device.type == "cuda" and hasattr(t, "capture")):
            return False
        host_hooks = t.allreduce is not None or getattr(t, "bucket_hook", None) is not None
        if not host_hooks:
            return True
        return self.group.active and self.group.backend == "nccl" and self.cfg.graph_collectives

    def _run_chunk(self, n: int) -> int:
        """Run exactly ``min(n, graph_steps)`` steps and return that count.

        The chunk length is a function of the step counter and the shared config only
        (``n`` comes from the log / checkpoint / hold boundaries), never of this rank's own
        graph state: every chunk posts one group collective (``_agree``), so members of a
        lock-step group must cut their chunks at the same steps even when a shard landing
        on one of them mid-run dropped only its graph.  Graph mode replays a
        captured k-step graph; a chunk that finds no graph runs one eager step (sizes the
        lazily-grown workspaces), captures, and replays the rest of the chunk.

        Eager steps take ``train_lock`` one step at a time, so ReceiveFile / ExchangeUpdates /
        gossip wait for at most one step, not a whole chunk.  A collective failing
        at step j of a chunk raises :class:`ChunkBroken` carrying the j steps that did complete,
        so the step counter stays equal to the trainer's real state.  That count is exact on
        the eager path.  On the graph path (opt-in RCCL-in-graph) a failure can only surface
        in the chunk's first eager step or its capture: ``done`` is then 0 or 1 while replays
        queued before the failure may still have advanced the device cursor and weights.  The
        regroup that follows re-synchronises both: rank 0 broadcasts the parameters, the
        momentum and its step counter (``_maybe_regroup``), so every member restarts from one
        consistent (step, state) pair."""
        t = self.trainer
        k = max(1, self.cfg.graph_steps)
        n = max(1, min(n, k))
        done = 0
        try:
            if self._probe_due and hasattr(t, "probe_step"):
                # once per log interval: the chunk's first step runs eagerly with its phase
                # boundaries recorded; resolved later, outside the lock (_poll_phases)
                self._probe_due = False
                with self.train_lock:
                    self._pending_phases = t.probe_step()
                done = 1
            if not self._use_graph():
                while done < n:
                    with self.train_lock:
                        t.step()
                    done += 1
                return n
            with self.train_lock:
                if t.graph is None:
                    if done == 0:
                        t.step()  # eager first: sizes lazily grown workspaces before the capture
                        done = 1
                    if hasattr(t, "steps"):
                        t.capture(warmup=0, unroll=k)
                    else:
                        t.capture(warmup=0)
                    # the replays now hold collectives iff the step has a host hook (RCCL in graph)
                    self._graph_collectives = (t.allreduce is not None
                                               or getattr(t, "bucket_hook", None) is not None)
                    self.log.info("graph_captured", steps=k, step=self.step + 1)
                if n > done:
                    if hasattr(t, "steps"):
                        t.steps(n - done)
                    else:
                        while done < n:
                            t.step()
                            done += 1
                    done = n
            self.graph_chunks += 1
            return n
        except GroupBroken as e:
            raise ChunkBroken(done, e) from e

    def _account_steps(self, prev: int, ran: int) -> None:
        self.step = prev + ran
        self.samples += ran * self.trainer.batch
        for s_i in range(prev + 1, self.step + 1):
            self.fault.on_step(s_i)

    def _group_metrics_update(self, dt: float, samples: int, st) -> None:
        """N3: all-reduce [loss_sum, correct_sum, samples] (SUM) and the interval (MAX) over
        the group every log_every steps: the job-level samples/s is total samples over the
        slowest rank's time.  Every member of a lock-step group calls this at the same step."""
        if not (self.group.active and self.group.world > 1):
            self.group_metrics = {"samples_per_sec": samples / max(dt, 1e-9), "loss": st.loss,
                                  "accuracy": st.accuracy, "world": 1}
            return
        dev = self.device if self.group.backend == "nccl" else torch.device("cpu")
        b = float(self.trainer.batch)
        v = torch.tensor([st.loss * b, st.accuracy * b, b, float(samples)], dtype=torch.float64, device=dev)
        m = torch.tensor([dt], dtype=torch.float64, device=dev)
        self.group.allreduce_(v)
        self.group.allreduce_(m, torch.distributed.ReduceOp.MAX)
        v, m = v.cpu(), float(m.item())
        self.group_metrics = {"samples_per_sec": float(v[3]) / max(m, 1e-9), "loss": float(v[0] / v[2]),
                              "accuracy": float(v[1] / v[2]), "world": self.group.world}

    def _train_loop(self) -> None:
        if self.cfg.model == "simulate":
            return self._simulate_loop()
        t_last, s_last = time.perf_counter(), 0
        ready_epoch = -1
        inflight = None  # event recorded after the previous chunk: at most two chunks queued
        while not self._stop.is_set():
            with self.train_lock:
                if self._pending_shard is not None:
                    self._ensure_trainer()
                    x, y, fnum = self._pending_shard
                    self._pending_shard = None
                    self.trainer.load_shard(x, y)
                    self.log.info("shard_loaded", file_num=fnum, records=int(x.shape[0]))
            have_data = self.trainer is not None and self.trainer.x is not None
            if self.cfg.sync == "allreduce":
                self._maybe_regroup()
                self._install_allreduce()
                if self.group.broken:
                    self.state = "regrouping"  # waiting for the master's next view (see _needs_regroup)
                    self._idle(0.05)
                    continue
                if self.group.active and self._agreed_epoch > self.group.epoch:
                    # the group agreed to move to a newer epoch that this worker's view has
                    # not reached yet: no more steps on the old group, wait for the CheckUp
                    self.state = "regrouping"
                    self._idle(0.05)
                    continue
                if self.view["world"] > 1:
                    if not self.group.active:
                        self._idle(0.05)
                        continue
                    if ready_epoch != self.group.epoch:
                        # every member must have data before the first lock-step collective;
                        # the same all-reduce agrees on the newest epoch any member has seen
                        try:
                            agreed, all_data = self._agree(have_data)()
                        except GroupBroken:
                            continue
                        self._agreed_epoch = max(self._agreed_epoch, agreed)
                        if agreed > self.group.epoch:
                            self._drop_xgmi(healthy=True)
                            continue
                        if all_data:
                            ready_epoch = self.group.epoch
                            t_last, s_last = time.perf_counter(), self.samples
                        else:
                            self.state = "waiting_for_data"
                            self._idle(0.1)
                            continue
            if not have_data:
                self.state = "idle"
                self._idle(0.2, self.has_data)
                self.has_data.clear()
                continue
            hold = self.hold_at
            if hold is not None and self.step >= hold:
                if self.held_step != self.step:
                    if self.device.type == "cuda":
                        torch.cuda.synchronize(self.device)
                    self.held_step = self.step  # every step up to here has finished on the device
                    self.state = "held"
                self._stop.wait(0.0002)
                continue
            want = self.cfg.max_steps - self.step if self.cfg.max_steps else 1 << 30
            if hold is not None:
                want = min(want, hold - self.step)
            # chunks end on log / checkpoint boundaries, so every member of a lock-step group
            # runs its group collectives (metrics) at the same step
            for every in (self.cfg.log_every, self.cfg.checkpoint_every):
                if every:
                    want = min(want, every - self.step % every)
            prev = self.step
            try:
                with trace.span("steps", step=self.step):
                    ran = self._run_chunk(want)
            except ChunkBroken as e:
                self._account_steps(prev, e.done)
                self.log.warn("collective_failed", error=str(e.cause), epoch=self.group.epoch, steps_done=e.done)
                continue
            self._account_steps(prev, ran)
            self._poll_phases()
            self.state = "training"
            lockstep = self.cfg.sync == "allreduce" and self.group.active and self.group.world > 1
            agreement = None
            if lockstep:
                try:
                    agreement = self._agree()
                except GroupBroken as e:
                    self.log.warn("collective_failed", error=str(e), epoch=self.group.epoch)
                    continue
            if self.device.type == "cuda":
                ev = torch.cuda.Event()
                ev.record()
                if inflight is not None:
                    inflight.synchronize()
                inflight = ev
            if agreement is not None:
                try:
                    agreed, _ = agreement()
                except GroupBroken as e:
                    self.log.warn("collective_failed", error=str(e), epoch=self.group.epoch)
                    continue
                if agreed > self.group.epoch:
                    # every member is at this same step boundary: leave the exchange together
                    self._agreed_epoch = max(self._agreed_epoch, agreed)
                    self._drop_xgmi(healthy=True)
            if self.xgmi is not None and self.xgmi.error():
                # a peer stopped answering the step barrier (checked at every chunk boundary,
                # i.e. every graph replay): results since are void -- re-form (the master's
                # next epoch) and resync from rank 0
                self.log.warn("xgmi_barrier_timeout", epoch=self.group.epoch, step=self.step)
                self.group.broken = True
                continue
            if self.cfg.log_every and self.step // self.cfg.log_every != prev // self.cfg.log_every:
                st = self.trainer.stats()
                now = time.perf_counter()
                dt = max(1e-9, now - t_last)
                self.rate = (self.samples - s_last) / dt
                try:
                    self._group_metrics_update(dt, self.samples - s_last, st)
                except GroupBroken as e:
                    self.log.warn("group_metrics_failed", error=str(e))
                steps_i = max(1, (self.samples - s_last) // max(1, self.trainer.batch))
                self.phase_stats["step_ms"] = dt * 1e3 / steps_i
                self.phase_stats["data_wait_ms"] = self._wait_s * 1e3 / steps_i
                self._wait_s = 0.0
                self._probe_due = True  # the next chunk times one step's phases
                t_last, s_last = time.perf_counter(), self.samples
                self.loss = st.loss
                gm = self.group_metrics
                extra = {}
                if self._log_param_sum:
                    # replica checksum for the elastic rehearsal (scripts/elastic_demo.py): a float64
                    # copy of every parameter and a device sync, so opt-in only
                    extra["param_sum"] = float(self.trainer.params.double().sum())
                self.log.info("train", step=self.step, loss=round(st.loss, 4), acc=round(st.accuracy, 4),
                              samples_per_sec=round(self.rate, 1), epoch=self.group.epoch,
                              group_samples_per_sec=round(gm["samples_per_sec"], 1), group_world=gm["world"],
                              group_loss=round(gm["loss"], 4), graph=self._use_graph(),
                              **{k: round(v, 4) for k, v in self.phase_stats.items()}, **extra)
            if (self.cfg.checkpoint_every and self.step // self.cfg.checkpoint_every != prev // self.cfg.checkpoint_every
                    and (self.group.rank <= 0)):
                try:
                    self.save_checkpoint()
                except Exception as e:
                    self.log.warn("checkpoint_failed", error=repr(e))
            if self.cfg.max_steps and self.step >= self.cfg.max_steps:
                self.state = "done"
                return

    def _idle(self, secs: float, event: threading.Event | None = None) -> None:
        """A wait of the training loop (no data, waiting for the group or a peer's data):
        counted into the next log interval's data-wait share (``phase_stats``)."""
        t0 = time.perf_counter()
        (event or self._stop).wait(secs)
        self._wait_s += time.perf_counter() - t0

    def _poll_phases(self) -> None:
        """Resolve the probed step once the device has finished it (a non-blocking event query:
        never a wait -- with a dead peer the step may stall until the exchange times out)."""
        pend = self._pending_phases
        if pend is not None and pend.ready():
            self._pending_phases = None
            self._record_phases(pend.result())

    def _record_phases(self, p: dict) -> None:
        """One probed step's phases (utils/phases.py) -> phase_stats / FlowFeedback."""
        ps = self.phase_stats
        ps["compute_ms"], ps["exchange_ms"], ps["update_ms"] = p["compute"], p["exchange"], p["update"]
        nbytes = p.get("exchange_bytes", 0)
        ps["exchange_gbps"] = nbytes / (p["exchange"] * 1e-3) / 1e9 if nbytes and p["exchange"] > 0 else 0.0

    def _simulate_loop(self) -> None:
        """The reference's training: every model element += 1 every 2 s (worker.cc:221-231)."""
        while not self._stop.wait(self.cfg.simulated_train_interval_ms / 1000.0):
            with self.gossip.lock:
                self.gossip.model += 1.0
            self.step += 1

    def _gossip_loop(self) -> None:
        while not self._stop.wait(self.cfg.gossip_interval):
            self.gossip_once()

    def gossip_once(self) -> bool:
        """One exchange with a random peer (or the master for sync=ps). False if nothing to do."""
        if self.gossip is None:
            return False
        if self.cfg.sync == "ps":
            target, service = self.cfg.master_addr, "Master"
            md = ((PS_CLIENT_MD, self.addr),)
        else:
            md = None
            with self.view_lock:
                peers = [p for p in self.view["peers"] if p != self.addr]
            if not peers:  # the reference computes rand() % 0 here (worker.cc:200)
                return False
            target, service = random.choice(peers), "Worker"
        with trace.span("gossip", peer=target):
            with self.train_lock:
                delta = self.gossip.make_delta()
            try:
                raw = self.channels.unary(target, service, "ExchangeUpdates", encode_update(delta), metadata=md)
            except RpcFailure as e:  # the reference applies the reply even on failure (worker.cc:153-165)
                self.log.warn("gossip_failed", peer=target, error=e.code.name if e.code else "")
                return False
            reply = decode_update(raw, "float64")
            with self.train_lock:
                self.gossip.absorb(reply, delta)
                self._after_external_update()
        return True

    def _stall_watch(self) -> None:
        """Diagnostics (``SL_STALL_DUMP_S`` seconds): dump every thread's stack to stderr when
        the interpreter makes no progress that long.  A thread re-arms faulthandler's C
        watchdog every quarter period; the watchdog fires only when this thread could not run
        (the GIL held by a blocking call: the stall that silenced CheckUp in r06_full7)."""
        import faulthandler

        period = float(os.environ["SL_STALL_DUMP_S"])
        while not self._stop.is_set():
            faulthandler.dump_traceback_later(period, repeat=False, file=sys.stderr)
            self._stop.wait(period / 4)
        faulthandler.cancel_dump_traceback_later()

    # ---- lifecycle ---------------------------------------------------------------
    def start(self) -> "Worker":
        self.server = RpcServer(self.addr_requested, max_workers=16, max_message_bytes=self.cfg.max_message_bytes,
                                metrics=self.metrics)
        handlers = {"ReceiveFile": self._receive_file, "CheckUp": self._check_up,
                    "ExchangeUpdates": self._exchange_updates}
        self.server.add_service("Worker", {k: self.fault.wrap(k, v) for k, v in handlers.items()})
        self.server.start()
        self.addr = self.server.addr
        self.log.addr = self.addr
        loops = [self._register_loop, self._train_loop]
        if self.cfg.sync in ("gossip", "ps") or self.cfg.model == "simulate":
            loops.append(self._gossip_loop)
        if float(os.environ.get("SL_STALL_DUMP_S", "0") or 0) > 0:
            loops.append(self._stall_watch)
        for fn in loops:
            t = threading.Thread(target=fn, daemon=True, name="sl-worker-" + fn.__name__)
            t.start()
            self._threads.append(t)
        if self.cfg.metrics_port > 0:
            self.metrics.serve(self.cfg.metrics_port)
        self.log.info("serving", device=str(self.device), sync=self.cfg.sync, model=self.cfg.model)
        return self

    def leave(self) -> None:
        """Graceful departure: deregister so the group re-forms immediately."""
        try:
            self.channels.unary(self.cfg.master_addr, "MasterControl", "Deregister",
                                pb.WorkerBirthInfo(addr=self.addr, incarnation=self.incarnation).SerializeToString())
        except RpcFailure:
            pass

    def stop(self, leave: bool = True) -> None:
        self.metrics.close()
        if leave:
            self.leave()
        self._stop.set()
        self.has_data.set()
        for t in self._threads:
            t.join(timeout=10)
        self._drop_xgmi(healthy=False)
        self._drop_graphs()
        self.group.teardown()
        if self.server:
            self.server.stop()
        self.channels.close()

    def wait(self) -> None:
        self.server.wait()
