"""Checkpoint format -- wire-compatible with the reference's only state message.

The reference has no checkpointing at all: state lives in RAM
(/root/reference/src/master.cc:58-59) and the only model serialization is
``Update{repeated double delta}`` (/root/reference/src/protos/serverless_learn.proto:81-83).
A checkpoint here is therefore a *file* on the file server made of sections
that reuse that message:

    offset 0   8s  magic   b"SLCKPT01"
           8   u32 version (1)
           12  u32 meta_len
           16  u8[meta_len]  JSON metadata: model, n_params, step, epoch,
                              layout [[name, shape, offset]], optimizer
           ..  u64 len + Update  ABSOLUTE parameters (a delta against zero)
           ..  u64 len + Update  momentum buffer (len 0 when absent)
    version 2 appends the trainer's extra state (everything an exact resume needs
    beyond the flat vectors: the batch cursor, BatchNorm running statistics):
           ..  u32 count, then per entry: u32 name_len + name + u64 len + Update

so any peer that can parse ``Update`` can read the weights.  Checkpoints live
under reserved file numbers (>= CKPT_BASE) and move with the ordinary
``Chunk``/``ReceiveFile`` machinery; uploads use the additive
``FileStore.StoreFile`` RPC.
"""
from __future__ import annotations

import json
import struct

import numpy as np

from ..wire.codec import decode_update, encode_update

MAGIC = b"SLCKPT01"
CKPT_BASE = 1 << 31
_HDR = struct.Struct("<8sII")
_LEN = struct.Struct("<Q")


def is_checkpoint_file(file_num: int) -> bool:
    return file_num >= CKPT_BASE


_U32 = struct.Struct("<I")


def encode(params: np.ndarray, meta: dict, momentum: np.ndarray | None = None,
           extra: dict | None = None) -> bytes:
    """``extra``: name -> array (written as float64 ``Update`` sections, so integer state such
    as the batch cursor is exact up to 2**53)."""
    meta = dict(meta)
    meta.setdefault("n_params", int(np.asarray(params).size))
    extra = extra or {}
    meta["extra"] = sorted(extra)
    mj = json.dumps(meta, sort_keys=True).encode()
    body = encode_update(np.asarray(params))
    mom = encode_update(np.asarray(momentum)) if momentum is not None else b""
    parts = [_HDR.pack(MAGIC, 2, len(mj)), mj, _LEN.pack(len(body)), body, _LEN.pack(len(mom)), mom,
             _U32.pack(len(extra))]
    for name in sorted(extra):
        nb = name.encode()
        u = encode_update(np.asarray(extra[name], dtype=np.float64).reshape(-1))
        parts += [_U32.pack(len(nb)), nb, _LEN.pack(len(u)), u]
    return b"".join(parts)


def decode_extra(buf) -> dict:
    """The version-2 extra-state sections (name -> float64 array); {} for version 1."""
    return _decode(buf, "float32")[3]


def decode(buf, dtype: str = "float32") -> tuple[dict, np.ndarray, np.ndarray | None]:
    meta, params, mom, _ = _decode(buf, dtype)
    return meta, params, mom


def decode_full(buf, dtype: str = "float32") -> tuple[dict, np.ndarray, np.ndarray | None, dict]:
    return _decode(buf, dtype)


def _decode(buf, dtype):
    mv = memoryview(buf)
    magic, ver, mlen = _HDR.unpack(bytes(mv[:_HDR.size]))
    if magic != MAGIC:
        raise ValueError("not a checkpoint")
    if ver not in (1, 2):
        raise ValueError(f"unsupported checkpoint version {ver}")
    pos = _HDR.size
    meta = json.loads(bytes(mv[pos:pos + mlen]))
    pos += mlen
    (n,) = _LEN.unpack(bytes(mv[pos:pos + 8]))
    pos += 8
    params = decode_update(bytes(mv[pos:pos + n]), dtype)
    pos += n
    (m,) = _LEN.unpack(bytes(mv[pos:pos + 8]))
    pos += 8
    mom = decode_update(bytes(mv[pos:pos + m]), dtype) if m else None
    pos += m
    if params.size != meta.get("n_params", params.size):
        raise ValueError("checkpoint parameter count mismatch")
    extra = {}
    if ver >= 2:
        (cnt,) = _U32.unpack(bytes(mv[pos:pos + 4]))
        pos += 4
        for _ in range(cnt):
            (nl,) = _U32.unpack(bytes(mv[pos:pos + 4]))
            name = bytes(mv[pos + 4:pos + 4 + nl]).decode()
            pos += 4 + nl
            (ul,) = _LEN.unpack(bytes(mv[pos:pos + 8]))
            pos += 8
            extra[name] = decode_update(bytes(mv[pos:pos + ul]), "float64")
            pos += ul
    return meta, params, mom, extra


def looks_like_checkpoint(buf) -> bool:
    return bytes(memoryview(buf)[:8]) == MAGIC
