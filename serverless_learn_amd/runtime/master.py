"""The master: membership, heartbeats/failure detection, push scheduling, PS.

Reference (/root/reference/src/master.cc, 310 LoC):
* ``RegisterBirth`` appends to a worker vector (:79-91) -- duplicates on
  re-register, entries never removed;
* ``periodically_do_checkups`` (:240-266) every 5 s CheckUps the file server and
  sends every worker the full ``PeerList`` over a brand-new channel, with no
  deadline; failures are only logged (:192-194);
* ``periodically_request_pushes`` (:220-237) every 5 s asks the file server,
  serially, to push file 0 to each worker;
* ``ExchangeUpdates`` (:95-114) is a parameter-server endpoint no client calls;
  ``periodically_send_updates`` (:268-293) is never started.

Here: a native membership registry (csrc/core/membership.cpp) with
incarnations, epochs, miss counting and eviction; heartbeats fan out in
parallel over cached channels with deadlines and carry the epoch, the
recipient's rank, the world size and the address of the collective
rendezvous store the master hosts (so workers can form an RCCL group without
any other coordinator); pushes are scheduled per rank (distinct shards,
concurrently, only when the assignment changes -- or every interval with
``push_policy="periodic"``, the reference's behaviour); newly joined workers
first receive the latest checkpoint; the PS endpoint is live and an optional
broadcast loop implements the dead ``periodically_send_updates``.
"""
from __future__ import annotations

import random
import threading
import time
from concurrent import futures

from .._core import core
from ..ckpt.format import CKPT_BASE
from ..config import Config
from ..parallel.ps import PS_CLIENT_MD, ParameterServer
from ..proto import messages as pb
from ..utils.log import Logger
from ..utils.metrics import Metrics
from ..wire.codec import decode_update, encode_update
from .transport import Channels, RpcFailure, RpcServer, metadata_dict

# FlowFeedback's step-time breakdown fields (proto fields 11-16)
PHASE_FIELDS = ("step_ms", "data_wait_ms", "compute_ms", "exchange_ms", "update_ms", "exchange_gbps")


def _free_port() -> int:
    from ..utils.ports import reserve_port

    return reserve_port()


class Master:
    def __init__(self, config: Config | None = None, addr: str | None = None, clock=time.monotonic):
        self.cfg = config or Config.from_env()
        self.addr_requested = addr or self.cfg.master_addr
        self.clock = clock
        self.metrics = Metrics("master")
        self.log = Logger("master", self.addr_requested, self.metrics)
        self.registry = core().Registry()
        self.ps = ParameterServer(self.cfg.learn_rate, per_client=not self.cfg.gossip_compat)
        self.ps_broadcasts = 0
        self.channels = Channels(self.cfg.max_message_bytes, self.cfg.rpc_timeout_s, metrics=self.metrics)
        self._lock = threading.Lock()
        self.incarnation: dict[str, int] = {}
        self.delivered: dict[str, tuple] = {}       # addr -> (incarnation, file_num)
        self.ckpt_delivered: dict[str, tuple] = {}  # addr -> (incarnation, ckpt file)
        self.latest_ckpt = 0
        self.feedback: dict[str, dict] = {}
        self._job_logged = 0.0
        self.file_server_ok = None
        self.rotation = 0
        self._wakes: list[threading.Event] = []
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self._pool = futures.ThreadPoolExecutor(max_workers=32, thread_name_prefix="sl-master")
        self.server: RpcServer | None = None
        self.store = None
        self.rendezvous = ""

    # ---- membership --------------------------------------------------------
    def peer_list(self, for_addr: str | None = None) -> "pb.PeerList":
        members = self.registry.members()
        rank = members.index(for_addr) if for_addr in members else -1
        return pb.PeerList(peer_addrs=members, epoch=self.registry.epoch(), rank=rank,
                           world_size=len(members), rendezvous=self.rendezvous,
                           resume_file=self.latest_ckpt)

    def _register(self, request: bytes, context) -> bytes:
        info = pb.WorkerBirthInfo.FromString(request)
        epoch, changed = self.registry.register_birth(info.addr, info.hostname, info.num_gpus,
                                                      info.incarnation, self.clock())
        with self._lock:
            self.incarnation[info.addr] = info.incarnation
        self.ps.client_joined(info.addr, info.incarnation)
        self.log.info("register_birth", worker=info.addr, epoch=epoch, changed=changed, gpus=info.num_gpus,
                      world=len(self.registry.members()))
        if changed:
            self._notify()  # disseminate the new view now, not in up to 5 s
        return pb.RegisterBirthAck(ok=True, epoch=epoch).SerializeToString()

    def _deregister(self, request: bytes, context) -> bytes:
        info = pb.WorkerBirthInfo.FromString(request)
        existed = self.registry.deregister(info.addr, info.incarnation)
        if existed:
            with self._lock:
                self.delivered.pop(info.addr, None)
                self.ckpt_delivered.pop(info.addr, None)
            self.ps.client_left(info.addr)
        self.log.info("deregister", worker=info.addr, existed=existed, epoch=self.registry.epoch(),
                      world=len(self.registry.members()))
        if existed:
            self._notify()
        return pb.RegisterBirthAck(ok=existed, epoch=self.registry.epoch()).SerializeToString()

    def _get_membership(self, request: bytes, context) -> bytes:
        return self.peer_list().SerializeToString()

    def _report_checkpoint(self, request: bytes, context) -> bytes:
        req = pb.Push.FromString(request)
        if req.file_num < CKPT_BASE:
            return pb.PushOutcome(ok=False, error="not a checkpoint file number").SerializeToString()
        with self._lock:
            self.latest_ckpt = req.file_num
        self.log.info("checkpoint_reported", file_num=req.file_num, by=req.recipient_addr)
        return pb.PushOutcome(ok=True).SerializeToString()

    # ---- parameter server ----------------------------------------------------
    def _exchange_updates(self, request: bytes, context) -> bytes:
        delta = decode_update(request, "float64")
        # Each client's exchanges are tracked separately (ParameterServer docstring); the
        # reference's Update carries no sender, so workers name themselves in metadata and a
        # reference-style client falls back to its connection's peer string.
        client = metadata_dict(context).get(PS_CLIENT_MD) or context.peer()
        reply = self.ps.exchange(delta, client)
        return encode_update(reply)

    def broadcast_once(self) -> bool:
        """What periodically_send_updates (master.cc:268-293) meant to do, without its % 0."""
        members = self.registry.members()
        if not members:
            return False
        target = random.choice(members)
        delta = self.ps.pending_delta(target)
        try:
            raw = self.channels.unary(target, "Worker", "ExchangeUpdates", encode_update(delta))
        except RpcFailure as e:
            self.log.warn("ps_broadcast_failed", to=target, error=str(e))
            return False
        self.ps.absorb_reply(decode_update(raw, "float64"), delta, target)
        self.ps_broadcasts += 1
        return True

    # ---- heartbeats / failure detection --------------------------------------
    def _checkup_worker(self, addr: str) -> None:
        pl = self.peer_list(addr)
        try:
            raw = self.channels.unary(addr, "Worker", "CheckUp", pl.SerializeToString(),
                                      timeout=self.cfg.rpc_timeout_s)
            fb = pb.FlowFeedback.FromString(raw)
            self.registry.heartbeat_ok(addr, self.clock())
            with self._lock:
                self.feedback[addr] = {"step": fb.step, "samples_per_sec": fb.samples_per_sec, "loss": fb.loss,
                                       "bytes_ingested": fb.bytes_ingested, "epoch": fb.epoch, "state": fb.state,
                                       "group_samples_per_sec": fb.group_samples_per_sec,
                                       "group_loss": fb.group_loss, "group_world": fb.group_world,
                                       **{k: getattr(fb, k) for k in PHASE_FIELDS}}
        except RpcFailure as e:
            evicted = self.registry.heartbeat_fail(addr, self.cfg.max_misses)
            self.log.warn("checkup_failed", worker=addr, evicted=evicted, error=e.code.name if e.code else "")
            if evicted:
                self.channels.forget(addr)
                with self._lock:
                    self.delivered.pop(addr, None)
                    self.ckpt_delivered.pop(addr, None)
                    self.feedback.pop(addr, None)
                self.ps.client_left(addr)
                self.log.info("evicted", worker=addr, epoch=self.registry.epoch(), world=len(self.registry.members()))
                self._notify()

    def checkup_once(self) -> None:
        try:
            raw = self.channels.unary(self.cfg.file_server_addr, "FileServer", "CheckUp",
                                      pb.Empty().SerializeToString(), timeout=self.cfg.rpc_timeout_s)
            lf = pb.LoadFeedback.FromString(raw)
            self.file_server_ok = {"active_pushes": lf.active_pushes, "bytes_sent": lf.bytes_sent, "files": lf.files}
        except RpcFailure as e:
            self.file_server_ok = None
            self.log.warn("file_server_checkup_failed", error=e.code.name if e.code else "")
        members = self.registry.members()
        list(self._pool.map(self._checkup_worker, members))
        job = self.job_metrics()
        now = time.monotonic()
        if job["workers"] and now - self._job_logged >= max(1.0, self.cfg.checkup_interval):
            self._job_logged = now
            self.log.info("job", **job)

    def job_metrics(self) -> dict:
        """Whole-job throughput from the workers' feedback (the metric the reference's empty
        FlowFeedback was reserved for, proto :73-75 / master.cc:155 TODO): a data-parallel
        group all-reduces its samples/s (N3) so every member reports the same group figure --
        counted once per group (by epoch); workers outside a group add their own rate."""
        with self._lock:
            fb = dict(self.feedback)
        groups: dict[int, float] = {}
        solo = 0.0
        for addr, f in fb.items():
            if f.get("state") not in ("training", "waiting_for_data", "regrouping"):
                continue
            if f.get("group_world", 0) > 1:
                groups[f["epoch"]] = max(groups.get(f["epoch"], 0.0), f.get("group_samples_per_sec", 0.0))
            else:
                solo += f.get("samples_per_sec", 0.0)
        # step-time breakdown over the training workers: mean per field, slowest step
        live = [f for f in fb.values() if f.get("state") == "training" and f.get("step_ms", 0.0) > 0]
        phases = {k: round(sum(f.get(k, 0.0) for f in live) / len(live), 4) for k in PHASE_FIELDS} if live else {}
        if live:
            phases["max_step_ms"] = round(max(f["step_ms"] for f in live), 4)
        return {"samples_per_sec": round(sum(groups.values()) + solo, 1), "groups": len(groups),
                "workers": len(fb), "phases": phases}

    # ---- push scheduling -------------------------------------------------------
    def _num_shards(self, n_members: int) -> int:
        return self.cfg.num_shards if self.cfg.num_shards > 0 else max(1, n_members)

    def _request_push(self, addr: str, file_num: int) -> bool:
        req = pb.Push(recipient_addr=addr, file_num=file_num).SerializeToString()
        try:
            raw = self.channels.unary(self.cfg.file_server_addr, "FileServer", "DoPush", req,
                                      timeout=max(60.0, self.cfg.rpc_timeout_s))
            out = pb.PushOutcome.FromString(raw)
        except RpcFailure as e:
            self.log.warn("push_request_failed", to=addr, file_num=file_num, error=str(e))
            return False
        if not out.ok:
            self.log.warn("push_failed", to=addr, file_num=file_num, error=out.error)
        return out.ok

    def _push_worker(self, addr: str, shard: int) -> None:
        with self._lock:
            inc = self.incarnation.get(addr, 0)
            ckpt = self.latest_ckpt
            need_ckpt = ckpt and self.ckpt_delivered.get(addr) != (inc, ckpt) and self.delivered.get(addr) is None
            need_data = (self.cfg.push_policy == "periodic") or self.delivered.get(addr) != (inc, shard)
        if need_ckpt:  # a fresh incarnation resumes from the newest checkpoint first
            if self._request_push(addr, ckpt):
                with self._lock:
                    self.ckpt_delivered[addr] = (inc, ckpt)
        if need_data and self._request_push(addr, shard):
            with self._lock:
                self.delivered[addr] = (inc, shard)

    def push_once(self) -> None:
        n = len(self.registry)
        assignment = self.registry.assignment(self._num_shards(n), self.rotation)
        list(self._pool.map(lambda a: self._push_worker(*a), assignment))

    # ---- loops -----------------------------------------------------------------
    def _notify(self) -> None:
        for ev in self._wakes:
            ev.set()

    def _loop(self, fn, interval: float, name: str, wake: threading.Event) -> None:
        while not self._stop.is_set():
            wake.clear()
            try:
                fn()
            except Exception as e:  # keep the control plane alive
                self.log.error(name + "_error", error=repr(e))
            wake.wait(interval)

    def _start_rendezvous(self) -> None:
        try:
            import datetime

            import torch.distributed as dist

            port = self.cfg.rendezvous_port or _free_port()
            host = self.addr.rsplit(":", 1)[0]
            host = "127.0.0.1" if host in ("localhost", "0.0.0.0", "[::]") else host
            self.store = dist.TCPStore(host, port, is_master=True, wait_for_workers=False,
                                       timeout=datetime.timedelta(seconds=60))
            self.rendezvous = f"{host}:{port}"
        except Exception as e:  # torch.distributed missing: gossip/PS still work
            self.log.warn("rendezvous_unavailable", error=repr(e))

    def start(self, loops: bool = True) -> "Master":
        self.server = RpcServer(self.addr_requested, max_workers=32, max_message_bytes=self.cfg.max_message_bytes,
                                metrics=self.metrics)
        self.server.add_service("Master", {"RegisterBirth": self._register, "ExchangeUpdates": self._exchange_updates})
        self.server.add_service("MasterControl", {"Deregister": self._deregister,
                                                  "GetMembership": self._get_membership,
                                                  "ReportCheckpoint": self._report_checkpoint})
        self.server.start()
        self.addr = self.server.addr
        self.log.addr = self.addr
        self._start_rendezvous()
        if self.cfg.metrics_port > 0:
            self.metrics.serve(self.cfg.metrics_port)
        self.log.info("serving", rendezvous=self.rendezvous)
        if loops:
            loops = [(self.checkup_once, self.cfg.checkup_interval, "checkup"),
                     (self.push_once, self.cfg.push_interval, "push")]
            if self.cfg.ps_broadcast_interval_ms > 0:  # the reference's unstarted periodically_send_updates
                loops.append((self.broadcast_once, self.cfg.ps_broadcast_interval, "ps_broadcast"))
            for fn, iv, name in loops:
                ev = threading.Event()
                self._wakes.append(ev)
                t = threading.Thread(target=self._loop, args=(fn, iv, name, ev), daemon=True, name=f"sl-master-{name}")
                t.start()
                self._threads.append(t)
        return self

    def stop(self) -> None:
        self.metrics.close()
        self._stop.set()
        self._notify()
        for t in self._threads:
            t.join(timeout=10)
        if self.server:
            self.server.stop()
        self._pool.shutdown(wait=False, cancel_futures=True)
        self.channels.close()

    def wait(self) -> None:
        self.server.wait()
