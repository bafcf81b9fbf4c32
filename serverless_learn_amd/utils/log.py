"""Structured JSON-lines logging.

The reference logs free text with ``std::cout`` at every RPC entry/exit
(e.g. /root/reference/src/master.cc:81,89,139-143, worker.cc:51,59,
file_server.cc:61,80,83-84).  Here every event is one JSON object on stderr
(or ``SL_LOG_FILE``) with ``ts``, ``role``, ``addr``, ``event`` and free
fields, so a multi-process run can be merged and queried.  ``SL_LOG_LEVEL``
(debug|info|warn|error) filters.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time

_LEVELS = {"debug": 10, "info": 20, "warn": 30, "error": 40}
_lock = threading.Lock()
_sink = None


def _out():
    global _sink
    if _sink is None:
        path = os.environ.get("SL_LOG_FILE")
        _sink = open(path, "a", buffering=1) if path else sys.stderr
    return _sink


class Logger:
    def __init__(self, role: str, addr: str = "", metrics=None):
        self.role = role
        self.addr = addr
        self.metrics = metrics  # utils.metrics.Metrics fed with every event (any level)
        self.min_level = _LEVELS.get(os.environ.get("SL_LOG_LEVEL", "info"), 20)

    def _emit(self, level: str, event: str, **fields):
        if self.metrics is not None:
            self.metrics.observe(level, event, fields)
        if _LEVELS[level] < self.min_level:
            return
        rec = {"ts": round(time.time(), 6), "level": level, "role": self.role, "addr": self.addr, "event": event}
        rec.update(fields)
        line = json.dumps(rec, default=str)
        with _lock:
            _out().write(line + "\n")

    def debug(self, event, **f):
        self._emit("debug", event, **f)

    def info(self, event, **f):
        self._emit("info", event, **f)

    def warn(self, event, **f):
        self._emit("warn", event, **f)

    def error(self, event, **f):
        self._emit("error", event, **f)
