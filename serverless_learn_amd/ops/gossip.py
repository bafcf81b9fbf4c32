"""K7: fused gossip delta-apply on a device-resident model (csrc/kernels/elementwise.hip)."""
from __future__ import annotations

import ctypes

import torch

from . import _native as N

N.register("sl_gossip_apply", [N.P, N.P, N.P, N.L, ctypes.c_double, N.P, N.L, N.P])
N.register("sl_gossip_absorb", [N.P, N.P, N.P, N.L, ctypes.c_double, N.P, N.L, N.L, N.P])


def delta_apply(model: torch.Tensor, old: torch.Tensor, din: torch.Tensor | None, alpha: float,
                dout: torch.Tensor | None) -> None:
    """m += alpha*din (f64, may be shorter than m); dout = m - o (f64); o = m."""
    assert model.is_cuda and model.dtype == torch.float32 and old.dtype == torch.float32
    assert model.is_contiguous() and old.is_contiguous() and old.numel() == model.numel()
    n = model.numel()
    kin = 0
    if din is not None:
        din = din.to(torch.float64).contiguous()
        kin = din.numel()
        if kin > n:
            raise ValueError("incoming delta longer than the model")
    if dout is not None:
        assert dout.dtype == torch.float64 and dout.numel() >= n and dout.is_contiguous()
    N.call("sl_gossip_apply", N.ptr(model), N.ptr(old), N.ptr(din), kin, float(alpha), N.ptr(dout), n,
           N.stream_ptr())


def absorb(model: torch.Tensor, old: torch.Tensor, r: torch.Tensor, alpha: float,
           sent: torch.Tensor | None) -> None:
    """m += alpha*r; o += sent + alpha*r (sent omitted: o += alpha*r). r, sent: f64, may be short."""
    assert model.is_cuda and model.dtype == torch.float32 and old.dtype == torch.float32
    assert model.is_contiguous() and old.is_contiguous() and old.numel() == model.numel()
    n = model.numel()
    r = r.to(torch.float64).contiguous()
    if sent is not None:
        sent = sent.to(torch.float64).contiguous()
    kr, ks = r.numel(), (0 if sent is None else sent.numel())
    if kr > n or ks > n:
        raise ValueError("reply or sent delta longer than the model")
    N.call("sl_gossip_absorb", N.ptr(model), N.ptr(old), N.ptr(r), kr, float(alpha), N.ptr(sent), ks, n,
           N.stream_ptr())
