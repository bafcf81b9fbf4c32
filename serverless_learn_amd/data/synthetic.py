"""Seeded synthetic MNIST-shaped data and the shard record format.

The reference's file server serves one "dummy file": 100,000,000 bytes from a
default-seeded ``std::independent_bits_engine`` (/root/reference/src/file_server.cc:40,151-156),
which workers read and discard (/root/reference/src/worker.cc:54-56).  Here a
file is a *shard* of labelled MNIST-shaped records that a worker actually
trains on.  Records are learnable (10 smooth class prototypes + noise), so the
loss falls during a run and accuracy is meaningful, yet no dataset download is
needed (there is no network).

Shard wire/file layout (little-endian, all offsets from the file start):

    0   8s   magic  b"SLSHARD1"
    8   u32  version (1)
    12  u32  kind    (1 = u8 images + u8 labels)
    16  u64  n       number of records
    24  u32  height  (28)
    28  u32  width   (28)
    32  u32  classes (10)
    36  u32  shard_index
    40  u32  num_shards
    44  u32  channels (0 or 1 = grey [n][h*w]; 3 = colour NHWC [n][h][w][3])
    48  u64  seed
    56  u64  reserved
    64  u8[n*height*width*channels]  images, row-major (HWC), record-contiguous
    ..  u8[n]               labels

A 100,000,000-byte shard (the reference's file size) holds 127,388 records.
"""
from __future__ import annotations

import struct

import numpy as np

MAGIC = b"SLSHARD1"
HEADER = struct.Struct("<8sIIQIIIIII QQ")
HEADER_SIZE = 64
assert HEADER.size == HEADER_SIZE
RECORD_BYTES = 28 * 28 + 1
REFERENCE_FILE_BYTES = 100_000_000  # /root/reference/src/file_server.cc:40


def records_for_bytes(nbytes: int = REFERENCE_FILE_BYTES) -> int:
    return (nbytes - HEADER_SIZE) // RECORD_BYTES


def _prototypes(classes: int, h: int, w: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed ^ 0x5EED)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    protos = np.zeros((classes, h, w), np.float32)
    for c in range(classes):
        for _ in range(3):
            cy, cx = rng.uniform(5, h - 5), rng.uniform(5, w - 5)
            sy, sx = rng.uniform(1.5, 4.0), rng.uniform(1.5, 4.0)
            protos[c] += np.exp(-((yy - cy) ** 2 / (2 * sy * sy) + (xx - cx) ** 2 / (2 * sx * sx)))
    protos /= protos.max(axis=(1, 2), keepdims=True)
    return protos.reshape(classes, h * w)


def make_mnist_like(n: int, seed: int = 0, classes: int = 10, h: int = 28, w: int = 28,
                    noise: float = 1.0) -> tuple[np.ndarray, np.ndarray]:
    """(images u8 [n, h*w], labels u8 [n]) -- deterministic in (n, seed)."""
    rng = np.random.default_rng(seed)
    protos = _prototypes(classes, h, w, 1234)  # shared by every shard: same task
    labels = rng.integers(0, classes, size=n, dtype=np.uint8)
    out = np.empty((n, h * w), np.uint8)
    chunk = 16384
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        amp = rng.uniform(0.6, 1.0, size=(e - s, 1)).astype(np.float32)
        img = protos[labels[s:e]] * amp + rng.standard_normal((e - s, h * w), dtype=np.float32) * noise
        np.clip(img * 255.0, 0, 255, out=img)
        out[s:e] = img.astype(np.uint8)
    return out, labels


def make_cifar_like(n: int, seed: int = 0, classes: int = 10, hw: int = 32,
                    noise: float = 0.6) -> tuple[np.ndarray, np.ndarray]:
    """(images u8 [n, hw, hw, 3] NHWC, labels u8 [n]) -- CIFAR-shaped, learnable, deterministic.

    Each class is a colour-tinted sum of Gaussian blobs (shared prototypes, so
    every shard is the same task); records add amplitude jitter, a random
    circular shift of up to 3 pixels and Gaussian noise.
    """
    rng = np.random.default_rng(seed)
    base = _prototypes(classes, hw, hw, 4321).reshape(classes, hw, hw)
    tint = np.random.default_rng(99).uniform(0.3, 1.0, size=(classes, 3)).astype(np.float32)
    protos = base[..., None] * tint[:, None, None, :]  # [classes, hw, hw, 3]
    labels = rng.integers(0, classes, size=n, dtype=np.uint8)
    out = np.empty((n, hw, hw, 3), np.uint8)
    chunk = 4096
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        m = e - s
        amp = rng.uniform(0.6, 1.0, size=(m, 1, 1, 1)).astype(np.float32)
        img = protos[labels[s:e]] * amp
        dy, dx = rng.integers(-3, 4, size=2)
        img = np.roll(img, (int(dy), int(dx)), axis=(1, 2))
        img += rng.standard_normal(img.shape, dtype=np.float32) * (noise * 0.5)
        np.clip(img * 200.0 + 28.0, 0, 255, out=img)
        out[s:e] = img.astype(np.uint8)
    return out, labels


def encode_shard(images: np.ndarray, labels: np.ndarray, shard_index: int = 0, num_shards: int = 1,
                 seed: int = 0, h: int = 28, w: int = 28, classes: int = 10, channels: int = 1) -> bytes:
    n = images.shape[0]
    kind = 1 if channels <= 1 else 2
    hdr = HEADER.pack(MAGIC, 1, kind, n, h, w, classes, shard_index, num_shards, channels if channels > 1 else 0,
                      seed, 0)
    return hdr + np.ascontiguousarray(images, np.uint8).tobytes() + np.ascontiguousarray(labels, np.uint8).tobytes()


def decode_header(buf) -> dict:
    mv = memoryview(buf)
    if len(mv) < HEADER_SIZE:
        raise ValueError("shard too short")
    magic, ver, kind, n, h, w, classes, si, ns, ch, seed, _r2 = HEADER.unpack(bytes(mv[:HEADER_SIZE]))
    if magic != MAGIC:
        raise ValueError("bad shard magic")
    return dict(version=ver, kind=kind, n=n, height=h, width=w, classes=classes,
                shard_index=si, num_shards=ns, seed=seed, channels=max(1, ch))


def decode_shard(buf) -> tuple[dict, np.ndarray, np.ndarray]:
    """Zero-copy views (images [n, h*w*channels], labels [n]) into ``buf``."""
    hdr = decode_header(buf)
    n, d = hdr["n"], hdr["height"] * hdr["width"] * hdr["channels"]
    arr = np.frombuffer(buf, dtype=np.uint8)
    need = HEADER_SIZE + n * d + n
    if arr.size < need:
        raise ValueError(f"shard truncated: {arr.size} < {need}")
    images = arr[HEADER_SIZE:HEADER_SIZE + n * d].reshape(n, d)
    labels = arr[HEADER_SIZE + n * d:need]
    return hdr, images, labels


def make_shard_philox(n: int, shard_index: int = 0, num_shards: int = 1, seed: int = 0,
                      dataset: str = "synthetic-mnist", threads: int | None = None) -> bytes:
    """Shard ``shard_index`` = records [shard_index * n, (shard_index + 1) * n) of the Philox
    dataset keyed by ``seed``: the same records the on-device generator K8 produces
    (data/device_synth.py), synthesised by the native core on ``threads`` CPU threads straight
    into the encoded shard buffer (no intermediate arrays)."""
    import os

    from .._core import core
    from .device_synth import KINDS, prototypes

    kind = "cifar" if dataset == "synthetic-cifar" else "mnist"
    h, w, c, noise, scale, offset = KINDS[kind]
    pixels = h * w * c
    buf = bytearray(HEADER_SIZE + n * pixels + n)
    buf[:HEADER_SIZE] = HEADER.pack(MAGIC, 1, 1 if c == 1 else 2, n, h, w, 10, shard_index, num_shards,
                                    c if c > 1 else 0, seed, 0)
    arr = np.frombuffer(buf, dtype=np.uint8)
    images = arr[HEADER_SIZE:HEADER_SIZE + n * pixels]
    labels = arr[HEADER_SIZE + n * pixels:]
    threads = threads or max(1, min(16, (os.cpu_count() or 4)))
    core().synth_images(images, labels, n, pixels, prototypes(kind), 10, noise, scale, offset,
                        seed & ((1 << 64) - 1), shard_index * n, threads)
    return bytes(buf)


def make_shard(n: int, shard_index: int = 0, num_shards: int = 1, seed: int = 0, dataset: str = "synthetic-mnist",
               generator: str = "philox") -> bytes:
    """Shard ``shard_index`` of a seeded synthetic dataset (``synthetic-mnist`` or ``synthetic-cifar``).

    ``generator="philox"`` (default): the native multithreaded Philox generator (the K8
    records); ``"numpy"``: the original numpy generator (kept for comparisons and tests)."""
    if generator == "philox":
        return make_shard_philox(n, shard_index, num_shards, seed, dataset)
    if dataset == "synthetic-cifar":
        images, labels = make_cifar_like(n, seed=seed * 1000003 + shard_index)
        return encode_shard(images.reshape(n, -1), labels, shard_index, num_shards, seed, h=32, w=32, channels=3)
    images, labels = make_mnist_like(n, seed=seed * 1000003 + shard_index)
    return encode_shard(images, labels, shard_index, num_shards, seed)
