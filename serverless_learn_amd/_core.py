"""Loader for the native runtime module ``_slcore`` (csrc/core, pybind11)."""
from __future__ import annotations

import importlib.util
import os
import threading

from .build import CORE_SO, build_core

_lock = threading.Lock()
_mod = None


def core():
    """The ``_slcore`` extension (built in-tree on first use)."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is None:
            if not os.path.exists(CORE_SO):
                build_core()
            spec = importlib.util.spec_from_file_location("_slcore", CORE_SO)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            _mod = mod
    return _mod
