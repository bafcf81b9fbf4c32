"""ctypes binding of ``libslkernels.so`` (the gfx950 HIP kernels).

Every launcher takes raw device pointers plus the HIP stream and returns 0 on
success (non-zero = hipError_t or an argument error).  Launchers are cheap to
call and are captured into hipGraphs by ``torch.cuda.graph`` because they
launch on the caller's current stream.

There is deliberately NO silent fallback: on a machine with a GPU the ops
raise if the extension is missing or fails, so a test can never pass on an
eager PyTorch path while claiming to exercise the HIP kernels.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from ..build import KERNELS_DET_SO, KERNELS_SO

_lock = threading.Lock()
_lib = None

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float

# name -> argtypes (restype is always c_int unless listed in _RESTYPE)
_SIGS: dict[str, list] = {
    "sl_mlp_param_count": [],
    "sl_mlp_slab_stride": [],
    "sl_mlp_rows": [P, P, P, I, I, P, P, P, P, P, P, F, F, F, F, P, P, P, P, P, P, P, I, P, P, P],
    "sl_mlp_wgrad": [I, P, P, I, P, P, P, P, I, P, I, L, P],
    "sl_mlp_wgrad_slices": [I, I],
    "sl_mlp_set_rows_bm": [I],
    "sl_conv_set_halo": [I],
    "sl_conv_set_phase": [I],
    "sl_mlp_rows_bm": [I],
    "sl_mlp_set_stamps": [P],
    "sl_mlp_set_wg_stamps": [P],
    "sl_mlp_set_sgd_stamps": [P],
    "sl_mlp_sgd_wgs": [],
    "sl_mlp_sgd": [P, P, P, I, L, P, P, F, F, F, F, F, I, P, P, P, P, P, P, P, P],
    "sl_mlp_reduce_xgmi": [P, I, L, F, F, P, P, P, P, L, I, I, L, I, P],
    "sl_mlp_sgd_xgmi": [P, P, F, F, F, P, P, P, P, P, P, P, P, L, I, I, L, P, I, P],
    "sl_clock_probe": [P, P, I, P],
    "sl_comm_proxy": [P, P, L, I, P],
}
_RESTYPE = {"sl_mlp_param_count": ctypes.c_long, "sl_mlp_slab_stride": ctypes.c_long}


def register(name: str, argtypes: list, restype=ctypes.c_int) -> None:
    """Register a launcher signature (used by the op modules at import)."""
    _SIGS[name] = argtypes
    if restype is not ctypes.c_int:
        _RESTYPE[name] = restype
    if _lib is not None:
        _bind(_lib, name)


def _bind(lib, name):
    fn = getattr(lib, name)
    fn.argtypes = _SIGS[name]
    fn.restype = _RESTYPE.get(name, ctypes.c_int)


def available() -> bool:
    return os.path.exists(KERNELS_SO)


def lib():
    """Load (building first if needed) the kernel library."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            det = os.environ.get("SL_DETERMINISTIC", "0") == "1"  # bit-reproducible kernel build
            path = os.environ.get("SL_KERNELS_SO") or (KERNELS_DET_SO if det else KERNELS_SO)  # override: A/B builds
            if not os.path.exists(path):
                from ..build import build_kernels

                build_kernels(deterministic=det)
            handle = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            for name in _SIGS:
                if path not in (KERNELS_SO, KERNELS_DET_SO) and not hasattr(handle, name):
                    continue  # an A/B build of older kernels: only what it exports
                _bind(handle, name)
            _lib = handle
    return _lib


def stream_ptr(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def ptr(t) -> int | None:
    """Device pointer of a tensor (None passes a NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def call(name: str, *args) -> None:
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc}")


class Launch:
    """A kernel launch with its arguments converted to ctypes ONCE.

    Engines with static buffers (the fused MLP/CNN steps) build these at setup
    and call them every step: the per-launch host cost drops to one ctypes
    call plus the current-stream lookup, which matters for the eager (non
    hipGraph) multi-GPU path where the host must stay ahead of ~30 us steps.
    """

    __slots__ = ("name", "fn", "args")

    def __init__(self, name: str, *args):
        self.name = name
        fn = getattr(lib(), name)
        self.fn = fn
        conv = []
        for a, t in zip(args, _SIGS[name]):
            conv.append(a if a is None else t(a))
        self.args = tuple(conv)

    def __call__(self, stream=None) -> None:
        rc = self.fn(*self.args, ctypes.c_void_p(stream_ptr(stream)))
        if rc != 0:
            raise RuntimeError(f"{self.name} failed with code {rc}")
