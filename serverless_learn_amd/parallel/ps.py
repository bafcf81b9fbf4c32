"""Parameter-server exchange on the master.

Reference: ``MasterImpl::ExchangeUpdates`` (/root/reference/src/master.cc:95-114)
holds ``model_state``/``old_state`` (:58-59) and applies the same rule as the
worker-side gossip server: grow to the incoming length, ``m += LEARN_RATE*d``,
reply ``m - o``, ``o = m``.  In the reference no client ever calls it and the
master-side broadcast loop ``periodically_send_updates`` (:268-293) is never
started.  Here it is reachable: workers running ``--sync ps`` call it every
gossip interval, and the master can optionally broadcast its own progress to a
random worker (``broadcast_once``), which is what the dead loop intended.
The model lives in float64 (the wire type) and is guarded by a lock (the
reference mutates it from handler threads unlocked).
"""
from __future__ import annotations

import threading

import numpy as np


class ParameterServer:
    def __init__(self, alpha: float = 0.5):
        self.alpha = float(alpha)
        self.model = np.zeros(0, np.float64)
        self.old = np.zeros(0, np.float64)
        self.lock = threading.Lock()
        self.exchanges = 0

    def _grow(self, n: int) -> None:
        k = self.model.size
        if n > k:
            self.model = np.concatenate([self.model, np.zeros(n - k)])
            self.old = np.concatenate([self.old, np.zeros(n - k)])

    def exchange(self, delta: np.ndarray) -> np.ndarray:
        with self.lock:
            d = np.asarray(delta, np.float64)
            self._grow(d.size)
            self.model[:d.size] += self.alpha * d
            reply = self.model - self.old
            self.old = self.model.copy()
            self.exchanges += 1
            return reply

    def pending_delta(self) -> np.ndarray:
        """m - o: what the master would send in a broadcast (master.cc:276-282)."""
        with self.lock:
            return self.model - self.old

    def absorb_reply(self, reply: np.ndarray) -> None:
        """Client-side mixing of a worker's reply to a master broadcast; then o = m."""
        with self.lock:
            r = np.asarray(reply, np.float64)
            self._grow(r.size)
            self.model[:r.size] += self.alpha * r
            self.old = self.model.copy()

    def set_model(self, flat: np.ndarray) -> None:
        with self.lock:
            self.model = np.asarray(flat, np.float64).copy()
            self.old = self.model.copy()
