"""Wire codec facade: hot messages through the C++ codec (csrc/core/wire.cpp).

``Update`` (``repeated double delta = 1``, packed) and ``Chunk``
(``bytes data = 1``) are the two messages whose size scales with the model or
the data; everything else goes through the
descriptor-built protobuf classes in :mod:`serverless_learn_amd.proto.messages`.
"""
from __future__ import annotations

import numpy as np

from .._core import core

CHUNK_SIZE = 1_000_000  # /root/reference/src/file_server.cc:46


def encode_update(values) -> bytes:
    """float32/float64 array -> serialized Update (f64 on the wire)."""
    arr = np.ascontiguousarray(values)
    if arr.dtype not in (np.float32, np.float64):
        arr = arr.astype(np.float64)
    return core().encode_update(arr)


def decode_update(msg: bytes, dtype: str = "float64") -> np.ndarray:
    return core().decode_update(msg, dtype)


def encode_chunk(data) -> bytes:
    return core().encode_chunk(data)


def chunk_payload(msg: bytes) -> memoryview:
    off, n = core().chunk_payload(msg)
    return memoryview(msg)[off:off + n]


def iter_chunks(buf, chunk_size: int = CHUNK_SIZE):
    """Serialized ``Chunk`` messages covering ``buf`` (zero-copy slicing, one copy into each message)."""
    mv = memoryview(buf).cast("B")
    for pos in range(0, len(mv), chunk_size):
        yield encode_chunk(mv[pos:pos + chunk_size])
