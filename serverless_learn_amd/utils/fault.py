"""Fault injection (the reference has none).

``SL_FAULT`` holds ``;``-separated rules:

* ``kill:step=N``            -- the worker process exits (code 137) after step N
* ``kill:after_s=T``         -- ... after T seconds of training
* ``drop:<Method>:p=P``      -- an incoming RPC <Method> fails with UNAVAILABLE with probability P
* ``delay:<Method>:ms=M``    -- an incoming RPC <Method> is delayed by M ms
* ``hang:<Method>``          -- an incoming RPC <Method> never answers (deadline tests)

Rules are evaluated by the worker; tests also build :class:`FaultInjector`
directly.
"""
from __future__ import annotations

import os
import random
import threading
import time

import grpc


class FaultInjector:
    def __init__(self, spec: str = ""):
        self.kill_step = None
        self.kill_after = None
        self.drop: dict[str, float] = {}
        self.delay: dict[str, float] = {}
        self.hang: set[str] = set()
        self._t0 = time.monotonic()
        self._rng = random.Random(os.getpid())
        self._release = threading.Event()
        for rule in filter(None, (r.strip() for r in spec.split(";"))):
            parts = rule.split(":")
            kind = parts[0]
            kv = dict(p.split("=", 1) for p in parts[1:] if "=" in p)
            names = [p for p in parts[1:] if "=" not in p]
            if kind == "kill":
                if "step" in kv:
                    self.kill_step = int(kv["step"])
                if "after_s" in kv:
                    self.kill_after = float(kv["after_s"])
            elif kind == "drop":
                self.drop[names[0]] = float(kv.get("p", "1"))
            elif kind == "delay":
                self.delay[names[0]] = float(kv.get("ms", "100")) / 1000.0
            elif kind == "hang":
                self.hang.add(names[0])
            else:
                raise ValueError(f"unknown fault rule {rule!r}")

    @classmethod
    def from_env(cls) -> "FaultInjector":
        return cls(os.environ.get("SL_FAULT", ""))

    @property
    def active(self) -> bool:
        return bool(self.kill_step is not None or self.kill_after is not None or self.drop or self.delay or self.hang)

    def on_step(self, step: int) -> None:
        if self.kill_step is not None and step >= self.kill_step:
            os._exit(137)
        if self.kill_after is not None and time.monotonic() - self._t0 >= self.kill_after:
            os._exit(137)

    def release(self) -> None:
        """Unblock every handler parked by a ``hang`` rule (test teardown)."""
        self._release.set()

    def wrap(self, method: str, fn):
        """Wrap an RPC handler with this injector's drop/delay/hang rules."""
        if method not in self.drop and method not in self.delay and method not in self.hang:
            return fn

        def wrapped(request, context):
            if method in self.hang:
                self._release.wait(120)
            if method in self.delay:
                time.sleep(self.delay[method])
            if method in self.drop and self._rng.random() < self.drop[method]:
                context.abort(grpc.StatusCode.UNAVAILABLE, "fault injection: dropped")
            return fn(request, context)

        return wrapped
