"""Step-phase breakdown ("per-worker metrics struct: samples/s, step time
breakdown, allreduce GB/s").  The reference has no step at all -- ``simulate_training`` adds 1
to every element every 2 s (/root/reference/src/worker.cc:221-231) -- and its feedback
messages are reserved and empty (/root/reference/src/protos/serverless_learn.proto:73-79,
``// TODO`` at /root/reference/src/master.cc:155).

A :class:`PhaseProbe` records device events at the phase boundaries of ONE eager training step
when armed (the runtime arms it once per log interval; captured graph replays are never
probed, so the hot path pays nothing).  Nothing here waits for the device: the probed step
hands back a :class:`PendingPhases` that the runtime resolves once the step has finished
(``ready()`` is a non-blocking event query) -- a wait inside the training lock would stall the
RPC handlers that need that lock for as long as the step runs.  Engines call :meth:`mark` at the END of each phase:

* ``compute``  -- forward + backward (plus the optimizer when it is fused into the backward's
  last launch: the world-1 MLP step);
* ``exchange`` -- gradient aggregation not hidden behind compute (RCCL / gloo all-reduce, the
  xGMI reduce + step barrier, the ResNet bucket waits);
* ``update``   -- the optimizer launches after the exchange.
"""
from __future__ import annotations

import time

import torch


class PhaseProbe:
    PHASES = ("compute", "exchange", "update")

    def __init__(self, device):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.armed = False
        self._marks: list = []

    def arm(self) -> None:
        self.armed = True
        self._marks = []
        self.mark("start")

    def mark(self, name: str) -> None:
        if not self.armed:
            return
        if self.cuda:
            if torch.cuda.is_current_stream_capturing():
                return
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._marks.append((name, ev))
        else:
            self._marks.append((name, time.perf_counter()))

    def finish(self) -> "PendingPhases":
        """Disarm and hand back the marks recorded since :meth:`arm`, unresolved: the device
        may still be running the step (never synchronise here -- callers hold locks)."""
        self.armed = False
        marks, self._marks = self._marks, []
        return PendingPhases(marks, self.cuda)


class PendingPhases:
    """The marks of one probed step; :meth:`ready` / :meth:`result` once the device is done."""

    def __init__(self, marks: list, cuda: bool, exchange_bytes: int = 0):
        self.marks, self.cuda, self.exchange_bytes = marks, cuda, exchange_bytes

    def ready(self) -> bool:
        """Non-blocking: has the probed step's last phase finished on the device?"""
        return not (self.cuda and self.marks) or self.marks[-1][1].query()

    def result(self) -> dict:
        """{phase: ms} (missing phases 0; a phase marked twice accumulates) and the gradient
        bytes the step exchanged; waits for the device if the step is still running."""
        out = {p: 0.0 for p in PhaseProbe.PHASES}
        out["exchange_bytes"] = self.exchange_bytes
        marks = self.marks
        if len(marks) < 2:
            return out
        if self.cuda:
            marks[-1][1].synchronize()
        for (_, a), (name, b) in zip(marks, marks[1:]):
            ms = a.elapsed_time(b) if self.cuda else (b - a) * 1e3
            out[name] = out.get(name, 0.0) + float(ms)
        return out
