"""One-shot / two-shot all-reduce over xGMI through IPC-mapped peer buffers.

Inside a node the 8 MI355X are fully connected by xGMI (7 links per GPU).  For
the MLP's 1.08 MB gradient a ring all-reduce pays 2(W-1) latency-bound hops per
step; here each rank instead *reads every peer's gradient directly* (W-1
concurrent reads, one per link) and sums in rank order inside a kernel --
protocol and memory-ordering argument in ``csrc/kernels/xgmi.h``.  The exchange
needs no host synchronisation, so the whole multi-GPU step (forward, backward,
all-reduce, optimizer) is captured in one hipGraph like the 1-GPU step.

Synchronisation is inline (``SL_XGMI_BARRIER=1`` restores the one-wave barrier kernel): the
consumer kernel's workgroup 0 signals every peer in its prologue (the producer before it has
completed) and all its workgroups wait for the peers' signals there; the step id advances once
per step in the MLP rows kernel -- no barrier launch and no last-workgroup fan-in per step
(``profiles/r06_xchg``).  Whether ranks share a GPU (the rehearsals)
is detected at setup from the devices' PCI addresses; the consumer grid is then bounded so a
waiting rank never holds every CU its peer needs.

``two_shot=True`` switches to reduce-scatter + all-gather through the same buffers: each
rank sums only its 1/W chunk of the W payloads, and consumers read every chunk from its
owner -- 2(W-1)/W of a payload crosses each GPU's links instead of W-1 payloads, for one
more barrier.  Which one wins depends on W and the links (``bench.py`` times both).

Setup is collective: every rank allocates one uncached exchange buffer, exports
it with ``hipIpcGetMemHandle``, the 64-byte handles are all-gathered over the
existing process group (RCCL or gloo), and each rank maps every peer's buffer.
If any rank fails to map any peer, *all* ranks fall back to the process group's
all-reduce (decided by one all-reduce of an ok flag), so a group never mixes
the two paths.

The reference has no collective at all -- only 5-second RPC gossip
(/root/reference/src/worker.cc:194-219); this is the intra-node replacement.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Callable

import torch

from ..ops import _native as N

N.register("sl_xgmi_header_bytes", [])
N.register("sl_xgmi_alloc", [N.L, ctypes.POINTER(ctypes.c_void_p)])
N.register("sl_xgmi_free", [N.P])
N.register("sl_ipc_get_handle", [N.P, N.P])
N.register("sl_ipc_handle_size", [])
N.register("sl_ipc_open", [N.P, ctypes.POINTER(ctypes.c_void_p)])
N.register("sl_ipc_close", [N.P])
N.register("sl_xgmi_buffer_bytes", [N.L], restype=ctypes.c_long)
N.register("sl_xgmi_copyin", [N.P, N.P, N.L, N.I, N.I, N.L, N.P, N.L, N.P])
N.register("sl_xgmi_barrier", [N.P, N.P, N.L, N.I, N.I, N.L, N.I, N.P])
N.register("sl_xgmi_rs", [N.P, N.P, N.L, N.I, N.I, N.L, N.L, N.I, N.P])
N.register("sl_xgmi_abort", [N.P, N.P])
N.register("sl_xgmi_sum", [N.P, N.P, N.L, N.I, N.I, N.L, N.P, N.L, N.F, N.P])
N.register("sl_xgmi_peek", [N.P, N.P, N.L, N.I, N.I, N.L, N.I, N.I, N.I, N.P, N.L, N.P])

MAX_WORLD = 16


def enabled() -> bool:
    """``SL_XGMI=0`` forces the process-group (RCCL) all-reduce everywhere."""
    return os.environ.get("SL_XGMI", "1") != "0"


def two_shot_chunk4(slot_bytes: int, world: int) -> int:
    """float4 elements each rank reduces in two-shot mode: the W chunks cover the slot, and
    each is whole waves (64 float4), so a consumer wave reads from one owner's buffer."""
    per_rank = -(-(slot_bytes // 16) // world)
    return -(-per_rank // 64) * 64


def inline_sync_enabled() -> bool:
    """``SL_XGMI_BARRIER=1``: step barrier as its own one-wave kernel (the round-5 protocol)."""
    return os.environ.get("SL_XGMI_BARRIER", "0") != "1"


def device_key(device) -> bytes:
    """PCI address of the GPU (ranks that share one map to the same key)."""
    p = torch.cuda.get_device_properties(torch.device(device))
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}".encode()


def default_two_shot(world: int) -> bool:
    """Protocol for a group that cannot time both (the worker runtime): ``SL_XGMI_TWO_SHOT``
    = 1 / 0 forces it; by default two-shot from 4 ranks.  Bytes into each GPU for an n-byte
    payload: one-shot (W-1) n, spread over W-1 links (n per link); two-shot 2 (W-1) n / W
    (2 n / W per link) plus a second barrier -- at W = 8 and the MLP's 1.08 MB that is
    1.08 MB against 0.27 MB per link, while at W = 2 both move one payload over one link
    and the extra barrier only costs."""
    v = os.environ.get("SL_XGMI_TWO_SHOT", "")
    if v in ("0", "1"):
        return v == "1"
    return world >= 4


class XgmiExchange:
    """IPC-mapped exchange buffers of a whole group (one per rank) + step counter.

    ``allgather(bytes) -> list[bytes]`` and ``all_ok(bool) -> bool`` are the group's
    collectives (used only here, at setup)."""

    def __init__(self, payload_floats: int, rank: int, world: int, device: torch.device,
                 allgather: Callable[[bytes], list], all_ok: Callable[[bool], bool], two_shot: bool = False):
        if not (1 <= world <= MAX_WORLD) or not (0 <= rank < world):
            raise ValueError(f"xgmi exchange needs 1 <= world <= {MAX_WORLD}, got rank {rank} of {world}")
        lib = N.lib()
        self.rank, self.world, self.device = rank, world, device
        self.payload_floats = int(payload_floats)
        self.slot_bytes = (self.payload_floats * 4 + 255) // 256 * 256
        self.hdr = int(lib.sl_xgmi_header_bytes())
        self.chunk4 = two_shot_chunk4(self.slot_bytes, world)
        self.two_shot = bool(two_shot)
        # ranks sharing a GPU (rehearsals): bounded consumer grids under inline synchronisation
        keys = allgather(device_key(device).ljust(int(lib.sl_ipc_handle_size()), b"\0"))  # handle-sized record
        self.shared_gpu = len(set(keys)) < len(keys)
        self.inline_sync = (2 if self.shared_gpu else 1) if inline_sync_enabled() else 0
        self._own = ctypes.c_void_p()
        self._opened: list[int] = []
        self.table = None
        self._abort_stream = None
        self._abort_lock = threading.Lock()
        self._aborted = False
        ok = True
        err = ""
        with torch.cuda.device(device):
            rc = lib.sl_xgmi_alloc(int(lib.sl_xgmi_buffer_bytes(self.slot_bytes)), ctypes.byref(self._own))
            if rc != 0:
                raise RuntimeError(f"xgmi exchange allocation failed ({rc})")
            hsize = int(lib.sl_ipc_handle_size())
            handle = (ctypes.c_char * hsize)()
            rc = lib.sl_ipc_get_handle(self._own, handle)
            mine = bytes(handle) if rc == 0 else b""
            handles = allgather(mine)
            bases = []
            for q, h in enumerate(handles):
                if q == rank:
                    bases.append(self._own.value)
                    continue
                p = ctypes.c_void_p()
                if len(h) != hsize:
                    ok, err = False, f"rank {q} exported no IPC handle"
                    break
                buf = ctypes.create_string_buffer(h, hsize)
                rc = lib.sl_ipc_open(buf, ctypes.byref(p))
                if rc != 0:
                    ok, err = False, f"hipIpcOpenMemHandle(rank {q}) failed ({rc})"
                    break
                self._opened.append(p.value)
                bases.append(p.value)
            ok = all_ok(ok)
            if not ok:
                self.close(sync=False)
                raise RuntimeError("xgmi exchange unavailable: " + (err or "a peer failed to map its buffers"))
            self.table = torch.tensor(bases, dtype=torch.int64, device=device)
            # [0] completed steps (barrier mode) / step in flight (inline mode: advanced by the
            # MLP rows kernel), [1] finished-block counter, [2] error
            self.ctl = torch.zeros(4, dtype=torch.int32, device=device)

    # ---- pointers --------------------------------------------------------------
    @property
    def own(self) -> int:
        return self._own.value

    def slot_ptr(self, parity: int) -> int:
        return self.own + self.hdr + (parity & 1) * self.slot_bytes

    def args(self):
        """(table, ctl, slot_bytes, rank, world, chunk4) -- the launcher's XgArgs fields
        (chunk4 = 0 selects one-shot)."""
        return (self.table.data_ptr(), self.ctl.data_ptr(), self.slot_bytes, self.rank, self.world,
                self.chunk4 if self.two_shot else 0)

    def exchange_launches(self, n: int, inline: bool | None = None) -> list:
        """Launch specs run between "payload written" and "consumer": [(fn, extra args)].
        Inline synchronisation (the producer published the step): nothing for one-shot, the
        reduce-scatter (which waits and publishes by itself) for two-shot."""
        inl = self.inline_sync if inline is None else (self.inline_sync if inline else 0)
        if inl:
            return [("sl_xgmi_rs", (n, inl))] if self.two_shot else []
        if not self.two_shot:
            return [("sl_xgmi_barrier", (0,))]
        return [("sl_xgmi_barrier", (0,)), ("sl_xgmi_rs", (n, 0)), ("sl_xgmi_barrier", (1,))]

    # ---- generic all-reduce ----------------------------------------------------
    def allreduce_(self, t: torch.Tensor, scale: float = 1.0) -> None:
        """Sum ``t`` over the group in place (fp32, contiguous, numel % 4 == 0)."""
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() % 4:
            raise ValueError("xgmi allreduce_ needs a contiguous fp32 tensor with numel % 4 == 0")
        if t.numel() > self.payload_floats:
            raise ValueError("tensor larger than the exchange slot")
        s = N.stream_ptr()
        N.call("sl_xgmi_copyin", *self.args(), t.data_ptr(), t.numel(), s)
        for fn, extra in self.exchange_launches(t.numel(), inline=False):  # copyin does not publish
            N.call(fn, *self.args(), *extra, s)
        N.call("sl_xgmi_sum", *self.args(), t.data_ptr(), t.numel(), float(scale), s)

    def peek(self, q: int, parity: int, n: int, system: bool = True) -> torch.Tensor:
        """Copy of rank ``q``'s slot ``parity`` (diagnostics/tests)."""
        out = torch.empty((n + 3) // 4 * 4, dtype=torch.float32, device=self.device)
        N.call("sl_xgmi_peek", *self.args(), q, parity, 1 if system else 0, out.data_ptr(), out.numel(),
               N.stream_ptr())
        return out[:n]

    def steps_done(self) -> int:
        return int(self.ctl[0].item())

    def error(self) -> bool:
        """True if a barrier gave up waiting for a peer (the results since are invalid)."""
        return int(self.ctl[2].item()) != 0

    def abort(self) -> None:
        """The group is broken (a peer died): set the error word from a stream of its own, so
        a consumer spinning on the dead peer stops now instead of at the 10 s timeout, and the
        steps still queued skip their waits.  Their results are void, as after a timeout; the
        runtime re-forms the group and re-syncs the state from rank 0.

        Best effort: the abort kernel runs at once only if its (high-priority) stream does not
        share a hardware queue with the spinning consumer.  A process capped to 1-2 queues
        (several ranks on one GPU, utils/gpu_share.py) may have it queued behind the consumer
        until the timeout; that is harmless, just not faster."""
        with torch.cuda.device(self.device):  # callable from any thread (the runtime's CheckUp handler)
            if self._abort_stream is None:
                self._abort_stream = torch.cuda.Stream(device=self.device, priority=-1)
            N.call("sl_xgmi_abort", self.ctl.data_ptr(), N.stream_ptr(self._abort_stream))

    def abort_once(self) -> None:
        """:meth:`abort` unless already requested (the runtime may ask from its CheckUp thread
        and again from the training thread)."""
        with self._abort_lock:
            if self._aborted or not self._own.value:
                return
            self._aborted = True
        self.abort()

    def close(self, sync: bool = True) -> None:
        """Unmap peers and free the buffer.  ``sync``: the caller has already made sure
        (e.g. with a group barrier) that no peer still reads this rank's buffer."""
        if sync:
            torch.cuda.synchronize(self.device)
        lib = N.lib()
        for p in self._opened:
            lib.sl_ipc_close(ctypes.c_void_p(p))
        self._opened = []
        if self._own.value:
            lib.sl_xgmi_free(self._own)
            self._own = ctypes.c_void_p()


def probe(rank: int, world: int, device: torch.device, allgather: Callable[[bytes], list],
          all_ok: Callable[[bool], bool], n: int = 1 << 16) -> str:
    """Setup-time functional check of the exchange between THESE devices, before a trainer
    depends on it: a small one-shot and a small two-shot exchange each sum two payloads of
    small integers (exact in fp32, both slot parities) and compare with the closed form.  The
    verdict is agreed over the group.  Returns "" when every rank passed, otherwise the first
    failure seen here (or "a peer failed"), so the caller keeps the process group's all-reduce
    instead of finding out from a barrier timeout in every step.

    The protocol has been exercised only by ranks sharing one GPU on this pool; on a real
    multi-GPU node this is the first thing that crosses the xGMI links."""
    err = ""
    idx = torch.arange(n, device=device, dtype=torch.int64)
    for two in (False, True):
        ex = None
        try:
            ex = XgmiExchange(n, rank, world, device, allgather, all_ok, two_shot=two)
            for call in range(2):
                t = ((idx * (call + 3)) % 7 + rank + 1).to(torch.float32)
                ex.allreduce_(t)
                want = ((idx * (call + 3)) % 7 * world + world * (world + 1) // 2).to(torch.float32)
                torch.cuda.synchronize(device)
                if ex.error():
                    err = err or f"{'two' if two else 'one'}-shot probe: barrier timed out"
                elif not torch.equal(t, want):
                    bad = int((t != want).sum())
                    err = err or f"{'two' if two else 'one'}-shot probe call {call}: {bad} of {n} sums wrong"
        except RuntimeError as e:
            err = err or f"{'two' if two else 'one'}-shot probe: {e}"
            ex = None  # the constructor agreed on its own failure and freed what it had
        ok = all_ok(not err)  # every rank leaves this exchange together before anyone unmaps
        if ex is not None:
            ex.close()
        if not ok:
            return err or "a peer failed the exchange probe"
    return ""


def dist_collectives(group=None):
    """(allgather, all_ok) over a torch.distributed process group (default group)."""
    import torch.distributed as dist

    def allgather(b: bytes) -> list:
        out = [None] * dist.get_world_size(group)
        dist.all_gather_object(out, b, group=group)
        return out

    def all_ok(ok: bool) -> bool:
        out = [None] * dist.get_world_size(group)
        dist.all_gather_object(out, bool(ok), group=group)
        return all(out)

    return allgather, all_ok
