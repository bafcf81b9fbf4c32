"""Asynchronous gossip model averaging.

Reference behaviour (broken as written, intent reconstructed in SURVEY.md §3.4):

* client (/root/reference/src/worker.cc:194-219 + :145-172): every
  GOSSIP_INTERVAL pick a random peer, send ``d = m - o``, receive ``r``,
  ``m += alpha * r``, then ``o = m``;
* server (/root/reference/src/worker.cc:81-100): grow ``m``/``o`` with zeros
  to ``len(d)``, ``m += alpha * d``, reply ``r = m - o``, ``o = m``.

With dA = mA - oA and dB = mB - oB that gives
``mB' = mB + a*dA``, ``r = dB + a*dA``, ``mA' = mA + a*dB + a^2*dA`` -- the
initiator re-absorbs a^2 of its own delta (the "echo").  ``compat=True``
reproduces that bit-exactly; the default echo-free client applies
``a*(r - a*d) = a*dB``.

The state lives wherever the model lives: a torch tensor on the GPU (the
delta-apply is then one fused HIP kernel, ``ops.gossip.delta_apply``: f64
wire values in, f64 reply out, f32 model) or a float64/float32 CPU tensor.
Callers serialize access with the training step (the reference mutated the
vectors from three threads unlocked).
"""
from __future__ import annotations

import threading

import numpy as np
import torch


class GossipState:
    def __init__(self, model: torch.Tensor, alpha: float = 0.5, compat: bool = False,
                 growable: bool = False):
        """``model`` is the live flat parameter tensor (mutated in place).

        ``growable`` models (the reference-style simulated vector, CPU only)
        are re-allocated with zeros to the length of a longer incoming update,
        as worker.cc:85-89 does; a trainer-owned model has a fixed size.
        """
        self.model = model
        self.growable = growable
        self.old = model.detach().clone()
        self.alpha = float(alpha)
        self.compat = compat
        self.lock = threading.RLock()
        self.exchanges = 0
        self.serves = 0  # server-side exchanges (each sets o = m)
        self._serves_at_send = 0

    # -- helpers -------------------------------------------------------------
    def _grow(self, n: int) -> None:
        """Reference semantics: both vectors grow with zeros to the incoming length."""
        if n <= self.model.numel():
            return
        if not self.growable:
            raise ValueError(f"incoming update has {n} elements, model has {self.model.numel()}")
        k = self.model.numel()
        m = torch.zeros(n, dtype=self.model.dtype, device=self.model.device)
        o = torch.zeros_like(m)
        m[:k] = self.model
        o[:k] = self.old
        self.model, self.old = m, o

    def _use_kernel(self) -> bool:
        return self.model.is_cuda

    # -- client side -----------------------------------------------------------
    def make_delta(self) -> np.ndarray:
        """d = m - o (float64, as it goes on the wire).

        Remembers how many server-side exchanges had happened, so ``absorb`` can
        tell whether ``o`` moved while the RPC was in flight."""
        with self.lock:
            self._serves_at_send = self.serves
            return (self.model.double() - self.old.double()).cpu().numpy()

    def absorb(self, reply: np.ndarray, sent: np.ndarray) -> None:
        """Apply the peer's reply (worker.cc:155-164) and advance ``o``.

        The reference then sets ``o = m`` (:215).  Training keeps stepping while the
        RPC is in flight, so ``m`` already holds progress that was never sent; copying
        it into ``o`` would drop it from every later exchange.  ``o`` instead advances
        by exactly what was shared: ``o += sent + a*r``.  If this worker served an
        exchange in the meantime, that serve already set ``o = m`` (its reply carried
        everything, ``sent`` included), so only ``a*r`` is added.  With no concurrent
        steps both rules give ``o = m``, so the exchange math of SURVEY.md §3.4 is
        unchanged.

        ``compat`` keeps the reference's ``o = m`` (worker.cc:215) exactly, so progress made
        while the RPC was in flight is dropped from later exchanges there too -- compat mode
        reproduces the reference, including that loss."""
        with self.lock:
            r = torch.from_numpy(np.asarray(reply, dtype=np.float64))
            self._grow(r.numel())
            a = self.alpha
            s = torch.from_numpy(np.asarray(sent, dtype=np.float64))
            if not self.compat and s.numel() == r.numel():
                r = r - a * s  # remove the echo of our own delta: a*(r - a*d) = a*dB
            if self.serves != self._serves_at_send or s.numel() > self.model.numel():
                s = None  # o was reset by a serve in between: `sent` is already accounted for
            if self._use_kernel():
                from ..ops import gossip as gk

                gk.absorb(self.model, self.old, r.to(self.model.device), a,
                          None if s is None else s.to(self.model.device))
            else:
                n = r.numel()
                m = self.model[:n]
                m.copy_((m.double() + a * r).to(m.dtype))
                o = self.old.double()
                if s is not None:
                    o[:s.numel()] += s
                o[:n] += a * r
                self.old.copy_(o.to(self.old.dtype))
            if self.compat:
                self.old.copy_(self.model)  # worker.cc:215, o = m
            self.exchanges += 1

    # -- server side -----------------------------------------------------------
    def serve(self, delta: np.ndarray) -> np.ndarray:
        """m += a*d; reply r = m - o; o = m (worker.cc:81-100)."""
        with self.lock:
            d = torch.from_numpy(np.asarray(delta, dtype=np.float64))
            self._grow(d.numel())
            a = self.alpha
            if self._use_kernel():
                from ..ops import gossip as gk

                out = torch.empty(self.model.numel(), dtype=torch.float64, device=self.model.device)
                gk.delta_apply(self.model, self.old, d.to(self.model.device), a, out)
                reply = out.cpu().numpy()
            else:
                n = d.numel()
                m = self.model
                m[:n].copy_((m[:n].double() + a * d).to(m.dtype))
                reply = (m.double() - self.old.double()).numpy()
                self.old.copy_(m)
            self.serves += 1
            self.exchanges += 1
            return reply


def exact_exchange(mA, oA, mB, oB, alpha=0.5, compat=True):
    """Closed form of one exchange A->B, for tests."""
    dA, dB = mA - oA, mB - oB
    mB2 = mB + alpha * dA
    r = dB + alpha * dA
    mA2 = mA + alpha * r if compat else mA + alpha * dB
    return mA2, mA2.copy(), mB2, mB2.copy(), r
