"""Synchronous data parallelism over RCCL (new).

The reference only mixes models by RPC gossip every 5 s.  Inside a node this
framework aggregates gradients every step with an all-reduce over xGMI:
``torch.distributed`` with backend ``"nccl"``, which on ROCm IS RCCL (one
process per GPU).  CPU workers use ``"gloo"`` with identical semantics, which
is how the multi-process logic is tested without a GPU.

:class:`ElasticGroup` forms and re-forms the group from the membership the
master disseminates in ``PeerList`` (epoch, rank, world size, rendezvous
address of the master-hosted TCPStore).  Every epoch uses its own key prefix
in the store, so only workers that agree on the epoch ever meet; a failed or
timed-out rendezvous/collective marks the group broken and the worker waits
for the next epoch (join/leave/eviction all bump it).  After a re-form, rank 0
-- the longest-lived member, ranks follow join order -- broadcasts the model
and optimizer state.

Bucketed, backward-overlapped all-reduce lives with the engine that produces the
gradients: the ResNet-18 engine launches one asynchronous all-reduce per flat
gradient bucket as its backward fills it (``FusedResNetTrainer.bucket_hook`` /
``bucket_wait``, wired to :meth:`ElasticGroup.allreduce_async` by the worker).
"""
from __future__ import annotations

import datetime
import threading
import time

import torch
import torch.distributed as dist

from ..utils.log import Logger


class GroupBroken(RuntimeError):
    pass


class GroupCancelled(RuntimeError):
    """A rendezvous abandoned because the membership it was for is no longer current."""


class ElasticGroup:
    """A re-formable process group object (not torch's global default group).

    Using the backend classes directly (``ProcessGroupNCCL`` = RCCL on ROCm,
    ``ProcessGroupGloo`` on CPU) lets a worker drop a broken communicator and
    build the next epoch's without touching global state -- and lets several
    in-process workers (tests) each own a group.
    """

    def __init__(self, backend: str | None = None, device: torch.device | None = None, timeout_s: float = 60.0):
        self.device = device or torch.device("cpu")
        self.backend = backend or ("nccl" if self.device.type == "cuda" else "gloo")
        self.timeout = datetime.timedelta(seconds=timeout_s)
        self.epoch = -1
        self.rank = -1
        self.world = 0
        self.pg = None
        self.broken = False
        self.lock = threading.Lock()
        self.log = Logger("dp")
        self._stores = {}
        self._rounds: dict[int, int] = {}
        self._retired: list = []

    @property
    def active(self) -> bool:
        return self.pg is not None

    def _store(self, rendezvous: str):
        st = self._stores.get(rendezvous)
        if st is None:
            host, port = rendezvous.rsplit(":", 1)
            st = dist.TCPStore(host, int(port), is_master=False, timeout=self.timeout)
            self._stores[rendezvous] = st
        return st

    RETIRED_KEEP = 8  # torn-down gloo groups kept alive (see teardown)

    def teardown(self) -> None:
        pg, self.pg = self.pg, None
        if pg is None:
            return
        if self.backend == "nccl":
            try:
                pg.abort()  # ncclCommAbort: never block on a dead peer
            except Exception as e:
                self.log.warn("abort_failed", error=repr(e))
            return
        # A gloo group's destructor waits for the collectives still queued on it, and one posted
        # to a dead peer ends only at the group timeout: a survivor's regroup sat 17 s in that
        # destructor (profiles/r06_elastic_abort, ResNet kill2).  Keep the group alive instead;
        # its threads fail those collectives on their own.  The oldest of RETIRED_KEEP is freed
        # once a newer one is retired, long after its timeout has passed.
        self._retired.append(pg)
        del self._retired[:-self.RETIRED_KEEP]

    def _open_round(self, ep_store, epoch: int, rank: int, world: int, cancelled=None) -> int:
        """Agree on a fresh rendezvous round for this epoch, with every rank checked in.

        Rank 0 opens round r+1 on every attempt; the other ranks check in to the newest
        round rank 0 has opened (``in<r>``) and wait for its go (``go<r>``), which rank 0
        posts once all ``world - 1`` of them are in.  Only then does anyone build the
        backend group, so a failed or half-formed attempt never leaves stale keys under the
        next attempt's prefix (gloo/RCCL would connect to dead endpoints).

        A rank that checked in to a round rank 0 has just given up on (its wait timed out as
        the rank arrived) moves to the next round as soon as rank 0 opens it.  Before the
        check-in, a late rank could join the abandoned round and wait out a whole timeout
        there while rank 0 waited in the next one (the r06_full7 elastic failure).
        ``cancelled()`` turning true (the worker's view moved past ``epoch``) ends the wait.
        """
        deadline = time.monotonic() + self.timeout.total_seconds()

        def tick(what: str) -> None:
            if cancelled is not None and cancelled():
                raise GroupCancelled(f"epoch {epoch} superseded while {what}")
            if time.monotonic() > deadline:
                raise TimeoutError(f"epoch {epoch}: timed out while {what}")
            time.sleep(0.02)

        if rank == 0:
            rnd = int(ep_store.add("round", 1))
            while int(ep_store.add(f"in{rnd}", 0)) < world - 1:
                tick(f"waiting for {world - 1} ranks to check in to round {rnd}")
            ep_store.add(f"go{rnd}", 1)
        else:
            need = self._rounds.get(epoch, 0) + 1
            rnd = 0
            while True:
                cur = int(ep_store.add("round", 0))
                if cur >= need and cur != rnd:
                    ep_store.add(f"in{cur}", 1)  # the newest round rank 0 opened
                    rnd = cur
                if rnd and int(ep_store.add(f"go{rnd}", 0)) > 0:
                    break
                tick(f"waiting for rank 0's go (round {rnd or '-'}, need >= {need})")
        self._rounds[epoch] = rnd
        return rnd

    def reform(self, epoch: int, rank: int, world: int, rendezvous: str, cancelled=None) -> bool:
        """Join the group for ``epoch``. Returns True when the group is usable.
        ``cancelled``: optional predicate polled during the rendezvous; True abandons it."""
        with self.lock:
            self.teardown()
            self.epoch, self.rank, self.world = epoch, rank, world
            self.broken = False
            if world <= 1 or rank < 0 or not rendezvous:
                return True  # single worker: nothing to reduce
            try:
                base = self._store(rendezvous)
                rnd = self._open_round(dist.PrefixStore(f"sl/e{epoch}", base), epoch, rank, world, cancelled)
                store = dist.PrefixStore(f"sl/e{epoch}/r{rnd}", base)
                if self.backend == "nccl":
                    opts = dist.ProcessGroupNCCL.Options()
                    opts._timeout = self.timeout
                    pg = dist.ProcessGroupNCCL(store, rank, world, opts)
                    pg.eager_connect_single_device(self.device)
                else:
                    pg = dist.ProcessGroupGloo(store, rank, world, self.timeout)
                self.pg = pg
                self.log.info("group_formed", epoch=epoch, round=rnd, rank=rank, world=world, backend=self.backend)
                return True
            except Exception as e:
                self.broken = True
                event = "group_form_cancelled" if isinstance(e, GroupCancelled) else "group_form_failed"
                self.log.warn(event, epoch=epoch, rank=rank, world=world, error=repr(e))
                self.teardown()
                return False

    # ---- collectives -----------------------------------------------------
    def _run(self, work) -> None:
        try:
            work.wait()
        except Exception as e:
            self.broken = True
            raise GroupBroken(repr(e)) from e

    def allreduce_(self, t: torch.Tensor, op=None) -> None:
        if self.pg is None:
            return
        try:
            if op is None:
                work = self.pg.allreduce([t])
            else:
                o = dist.AllreduceOptions()
                o.reduceOp = op
                work = self.pg.allreduce([t], o)
        except Exception as e:
            self.broken = True
            raise GroupBroken(repr(e)) from e
        self._run(work)

    def allreduce_async(self, t: torch.Tensor, op=None):
        if self.pg is None:
            return None
        try:
            if op is None:
                return self.pg.allreduce([t])
            o = dist.AllreduceOptions()
            o.reduceOp = op
            return self.pg.allreduce([t], o)
        except Exception as e:
            self.broken = True
            raise GroupBroken(repr(e)) from e

    def wait(self, work) -> None:
        if work is not None:
            self._run(work)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> None:
        if self.pg is None:
            return
        o = dist.BroadcastOptions()
        o.rootRank = src
        try:
            work = self.pg.broadcast([t], o)
        except Exception as e:
            self.broken = True
            raise GroupBroken(repr(e)) from e
        self._run(work)

    def allgather_fixed(self, data: bytes, size: int) -> list[bytes]:
        """All-gather one ``size``-byte record per rank (``b""`` = this rank has none)."""
        if self.pg is None:
            return [data]
        buf = torch.zeros(size + 1, dtype=torch.uint8)
        if data:
            if len(data) != size:
                raise ValueError(f"record of {len(data)} bytes, expected {size}")
            buf[0] = 1
            buf[1:] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        if self.backend == "nccl":
            buf = buf.to(self.device)
        outs = [torch.empty_like(buf) for _ in range(self.world)]
        try:
            work = self.pg.allgather([outs], [buf])
        except Exception as e:
            self.broken = True
            raise GroupBroken(repr(e)) from e
        self._run(work)
        return [bytes(o[1:].cpu().numpy().tobytes()) if int(o[0]) else b"" for o in outs]

    def all_true(self, ok: bool) -> bool:
        t = torch.tensor([1.0 if ok else 0.0])
        if self.backend == "nccl":
            t = t.to(self.device)
        self.allreduce_(t, dist.ReduceOp.MIN)
        return bool(t.item() > 0.5)

    def sync_state(self, tensors: list[torch.Tensor]) -> None:
        """Rank 0 broadcasts model/optimizer state to every member (N2)."""
        for t in tensors:
            if t is not None:
                self.broadcast_(t, 0)
