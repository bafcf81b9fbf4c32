"""K5: flat fused SGD (one launch for a whole model's parameter vector)."""
from __future__ import annotations

import torch

from . import _native as N

N.register("sl_sgd_flat", [N.P, N.P, N.P, N.P, N.L, N.F, N.F, N.F, N.F, N.P])
N.register("sl_to_bf16", [N.P, N.P, N.L, N.P])


def sgd_flat(w: torch.Tensor, g: torch.Tensor, mom: torch.Tensor | None, lr: float, momentum: float = 0.0,
             weight_decay: float = 0.0, shadow: torch.Tensor | None = None, grad_scale: float = 1.0) -> None:
    assert w.is_cuda and w.dtype == torch.float32 and g.dtype == torch.float32
    assert w.is_contiguous() and g.is_contiguous() and g.numel() == w.numel()
    if shadow is not None:
        assert shadow.dtype == torch.bfloat16 and shadow.numel() == w.numel()
    N.call("sl_sgd_flat", N.ptr(w), N.ptr(g), N.ptr(mom), N.ptr(shadow), w.numel(), float(lr), float(momentum),
           float(weight_decay), float(grad_scale), N.stream_ptr())


def to_bf16(src: torch.Tensor, dst: torch.Tensor) -> None:
    assert src.dtype == torch.float32 and dst.dtype == torch.bfloat16 and src.numel() == dst.numel()
    N.call("sl_to_bf16", N.ptr(src), N.ptr(dst), src.numel(), N.stream_ptr())
