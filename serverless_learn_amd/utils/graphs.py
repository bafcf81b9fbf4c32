"""Captured-graph lifetime for the fused trainers: a replaced graph is retired, not destroyed.

Destroying a hipGraphExec waits for its launches to finish, and the destructor runs when the
last Python reference goes -- with the GIL held.  A trainer used to drop its graph on any state
change (``self.graph = None`` in ``load_shard``, ``enable_xgmi``, the runtime's checkpoint
load).  When a replay was still spinning on a dead xGMI peer (the update kernel's 10 s
timeout), that assignment blocked the whole process for up to 10 s: the gRPC threads could not
answer the master's CheckUp, and the master evicted two healthy survivors (the
``test_gpu_workers_kill_one_respawn_with_xgmi`` failure in ``profiles/r06_elastic``).

So ``graph`` / ``graph_unrolled`` are slots whose setter keeps the replaced graph in a retired
list.  :meth:`GraphSlots.reap_graphs` frees that list after ``torch.cuda.synchronize``, which
waits with the GIL released.  Trainers call it where they sync anyway: ``capture()`` and
``drop_graphs()``.  Nothing is destroyed while a launch may still be in flight.
"""
from __future__ import annotations

import torch


def _slot(name: str) -> property:
    key = "_slot_" + name

    def get(self):
        return self.__dict__.get(key)

    def put(self, g) -> None:
        old = self.__dict__.get(key)
        if old is not None and old is not g:
            self.__dict__.setdefault("_retired_graphs", []).append(old)
        self.__dict__[key] = g

    return property(get, put)


class GraphSlots:
    """Mixin: ``graph`` and ``graph_unrolled`` retire what they replace (see module doc)."""

    graph = _slot("graph")
    graph_unrolled = _slot("graph_unrolled")

    @property
    def retired_graphs(self) -> int:
        return len(self.__dict__.get("_retired_graphs", ()))

    def reap_graphs(self, sync: bool = True) -> None:
        """Free the retired graphs.  ``sync`` first waits for the device (GIL released), so
        their destructors find nothing in flight; pass False only when the caller has just
        synchronized."""
        retired = self.__dict__.get("_retired_graphs")
        if not retired:
            return
        if sync and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        retired.clear()
