"""Step-phase tracing to Chrome trace JSON (``SL_TRACE=<path>``).

The reference has no tracing.  Spans (data wait, step,
all-reduce, gossip, checkpoint, ingest, regroup) are recorded from the host with
``perf_counter_ns``; GPU phases are additionally bracketed with
``torch.cuda.synchronize`` when ``SL_TRACE_SYNC=1`` so their host span equals
their device time.  Open the file in chrome://tracing or Perfetto.  Kernel-level
timing comes from ``rocprofv3 --kernel-trace`` (see profiles/).
"""
from __future__ import annotations

import atexit
import json
import os
import threading
import time
from contextlib import contextmanager

_lock = threading.Lock()
_events: list = []
_path = os.environ.get("SL_TRACE", "")
_sync = os.environ.get("SL_TRACE_SYNC", "0") == "1"
_pid = os.getpid()


def enabled() -> bool:
    return bool(_path)


@contextmanager
def span(name: str, **args):
    if not _path:
        yield
        return
    if _sync:
        _maybe_sync()
    t0 = time.perf_counter_ns()
    try:
        yield
    finally:
        if _sync:
            _maybe_sync()
        t1 = time.perf_counter_ns()
        with _lock:
            _events.append({"name": name, "ph": "X", "ts": t0 / 1000.0, "dur": (t1 - t0) / 1000.0,
                            "pid": _pid, "tid": threading.get_ident() % 100000, "args": args})


def counter(name: str, **values):
    if not _path:
        return
    with _lock:
        _events.append({"name": name, "ph": "C", "ts": time.perf_counter_ns() / 1000.0, "pid": _pid, "args": values})


def _maybe_sync():
    try:
        import torch

        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
    except Exception:
        pass


def flush(path: str | None = None) -> None:
    p = path or _path
    if not p:
        return
    with _lock:
        evs = list(_events)
    with open(p, "w") as f:
        json.dump({"traceEvents": evs, "displayTimeUnit": "ms"}, f)


if _path:
    atexit.register(flush)
