"""Parameter-server exchange on the master.

Reference: ``MasterImpl::ExchangeUpdates`` (/root/reference/src/master.cc:95-114)
holds ``model_state``/``old_state`` (:58-59) and applies the same rule as the
worker-side gossip server: grow to the incoming length, ``m += LEARN_RATE*d``,
reply ``m - o``, ``o = m``.  In the reference no client ever calls it and the
master-side broadcast loop ``periodically_send_updates`` (:268-293) is never
started.  Here it is reachable: workers running ``--sync ps`` call it every
gossip interval, and the master can optionally broadcast its own progress to a
random worker (``broadcast_once``), which is what the dead loop intended.

One shared ``old`` (the reference's rule, ``per_client=False``) makes every
reply exactly ``alpha*d`` -- the caller's own delta echoed back, because ``o``
was set to ``m`` by whichever exchange came last.  An echo-free client removes
that echo and is left with nothing, so no model ever learns from another.
The default therefore keeps one ``old`` *per client*: the reply is everything
the PS model gained since that client's previous exchange (the other clients'
``alpha``-scaled deltas plus its own ``alpha*d``), which the echo-free client
turns into ``alpha * (others' progress)``.  Without concurrent clients and with
a single client the two rules are identical.

The model lives in float64 (the wire type) and is guarded by a lock (the
reference mutates it from handler threads unlocked).
"""
from __future__ import annotations

import threading

import numpy as np

# gRPC metadata key a worker sets to name itself on Master.ExchangeUpdates
PS_CLIENT_MD = "sl-client"


def _grown(v: np.ndarray, n: int) -> np.ndarray:
    return v if v.size >= n else np.concatenate([v, np.zeros(n - v.size)])


class ParameterServer:
    def __init__(self, alpha: float = 0.5, per_client: bool = True):
        self.alpha = float(alpha)
        self.per_client = per_client
        self.model = np.zeros(0, np.float64)
        self.old = np.zeros(0, np.float64)          # the reference's single old_state
        self.olds: dict[str, np.ndarray] = {}       # per-client: PS model at that client's last exchange
        self.base = np.zeros(0, np.float64)         # what a client that never exchanged has seen
        self.lock = threading.Lock()
        self.exchanges = 0
        self.incarnations: dict[str, int] = {}      # client addr -> incarnation its ``old`` belongs to
        self.max_anonymous = 64                     # bound on per-connection entries (peer() strings)

    def _grow(self, n: int) -> None:
        self.model = _grown(self.model, n)
        self.old = _grown(self.old, n)

    def _old_for(self, client: str | None) -> np.ndarray:
        if not self.per_client or client is None:
            return self.old
        o = self.olds.get(client)
        # a new client has seen nothing yet: everything the PS holds is news to it
        if o is None and client not in self.incarnations:
            self._evict_anonymous()
        o = _grown(self.base.copy() if o is None else o, self.model.size)
        self.olds[client] = o
        return o

    def _evict_anonymous(self) -> None:
        """Reference-style clients are keyed by their connection (``context.peer()``), a new
        key per connection: keep at most ``max_anonymous`` of them (oldest dropped first)."""
        anon = [k for k in self.olds if k not in self.incarnations]
        for k in anon[:max(0, len(anon) - self.max_anonymous + 1)]:
            del self.olds[k]

    def client_joined(self, client: str, incarnation: int = 0) -> None:
        """A worker (re-)registered.  A new incarnation at a known address is a different
        process: it has seen none of the PS model, so its ``old`` restarts from ``base``
        instead of inheriting its predecessor's (which would hide everything the PS had
        accumulated before the restart from the echo-free client)."""
        with self.lock:
            if self.incarnations.get(client) != incarnation:
                self.olds.pop(client, None)
            self.incarnations[client] = incarnation

    def client_left(self, client: str) -> None:
        with self.lock:
            self.olds.pop(client, None)
            self.incarnations.pop(client, None)

    def _set_old(self, client: str | None) -> None:
        if not self.per_client or client is None:
            self.old = self.model.copy()
        else:
            self.olds[client] = self.model.copy()

    def exchange(self, delta: np.ndarray, client: str | None = None) -> np.ndarray:
        """m += alpha*d; reply m - o[client]; o[client] = m (master.cc:95-114)."""
        with self.lock:
            d = np.asarray(delta, np.float64)
            self._grow(d.size)
            self.model[:d.size] += self.alpha * d
            reply = self.model - self._old_for(client)
            self._set_old(client)
            self.exchanges += 1
            return reply

    def pending_delta(self, client: str | None = None) -> np.ndarray:
        """m - o: what the master would send in a broadcast (master.cc:276-282)."""
        with self.lock:
            return self.model - self._old_for(client)

    def absorb_reply(self, reply: np.ndarray, sent: np.ndarray | None = None, client: str | None = None) -> None:
        """Master-side mixing of a worker's reply to a broadcast.

        With ``sent`` given (echo-free), the echo ``alpha*sent`` is removed first, as the
        worker-side client does (parallel/gossip.py).  ``o[client]`` then advances by exactly
        what was shared with that client -- ``sent`` plus what its reply brought in -- not to
        the whole model: another client's exchange that landed while the broadcast RPC was in
        flight was never sent to ``client`` and must stay pending for it (the in-flight race
        ``GossipState.absorb`` handles on the worker side).  The single shared ``old`` of the
        reference rule keeps ``o = m``."""
        with self.lock:
            r = np.asarray(reply, np.float64)
            self._grow(r.size)
            if sent is not None and self.per_client:
                s = np.asarray(sent, np.float64)
                r = r.copy()
                r[:s.size] -= self.alpha * s
            self.model[:r.size] += self.alpha * r
            if not self.per_client or client is None or sent is None:
                self._set_old(client)
                return
            o = self._old_for(client)
            o[:s.size] += s
            o[:r.size] += self.alpha * r

    def set_model(self, flat: np.ndarray) -> None:
        with self.lock:
            self.model = np.asarray(flat, np.float64).copy()
            self.old = self.model.copy()
            self.base = self.model.copy()
            self.olds.clear()
