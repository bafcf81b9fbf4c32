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


def encode(params: np.ndarray, meta: dict, momentum: np.ndarray | None = None) -> bytes:
    meta = dict(meta)
    meta.setdefault("n_params", int(np.asarray(params).size))
    mj = json.dumps(meta, sort_keys=True).encode()
    body = encode_update(np.asarray(params))
    mom = encode_update(np.asarray(momentum)) if momentum is not None else b""
    return b"".join([_HDR.pack(MAGIC, 1, len(mj)), mj, _LEN.pack(len(body)), body, _LEN.pack(len(mom)), mom])


def decode(buf, dtype: str = "float32") -> tuple[dict, np.ndarray, np.ndarray | None]:
    mv = memoryview(buf)
    magic, ver, mlen = _HDR.unpack(bytes(mv[:_HDR.size]))
    if magic != MAGIC:
        raise ValueError("not a checkpoint")
    if ver != 1:
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
    if params.size != meta.get("n_params", params.size):
        raise ValueError("checkpoint parameter count mismatch")
    return meta, params, mom


def looks_like_checkpoint(buf) -> bool:
    return bytes(memoryview(buf)[:8]) == MAGIC
