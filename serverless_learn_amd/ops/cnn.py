"""ctypes bindings of the CNN kernels (csrc/kernels/conv.hip, cnn_aux.hip).

Thin, shape-checked wrappers: every function takes torch tensors (NHWC bf16
activations, fp32 statistics/gradients) and launches on the current stream,
so the CNN engine's whole step can be captured in a hipGraph.  No fallback:
on a GPU box a missing or failing kernel raises.
"""
from __future__ import annotations

import ctypes

import os

import torch

from . import _native as N

P, I, L, F = N.P, N.I, N.L, N.F

N.register("sl_conv_fwd", [P, I, I, I, I, P, I, I, I, I, I, I, I, P, I, P, P, P, P])
N.register("sl_conv_dgrad", [P, I, I, I, I, P, I, I, I, I, I, I, I, P, P, P])
N.register("sl_conv_dgrad_bnx", [P, I, I, I, I, P, I, I, I, I, I, I, I, P, P, P, P, P, P, P, P, I, P])
N.register("sl_conv_dgrad_s2_even", [P, I, I, I, I, P, I, I, I, P, P])
N.register("sl_conv_wgrad", [P, I, I, I, I, P, I, I, I, I, I, I, I, I, P, I, P, L, P])
N.register("sl_conv_wgrad_ws_need", [], ctypes.c_long)
N.register("sl_conv_wt", [P, I, L, P])
N.register("sl_conv_wt_desc_size", [])
N.register("sl_input_norm", [P, P, P, I, I, L, P, P, F, F, F, F, F, F, P])
N.register("sl_cursor_bump", [P, P])
N.register("sl_bn_finalize", [P, P, P, P, P, P, I, F, F, F, P])
N.register("sl_bn_apply", [P, P, P, P, P, L, I, I, I, P])
N.register("sl_bn_bwd_reduce", [P, P, P, P, P, P, P, P, P, L, I, P])
N.register("sl_bn_bwd_finalize", [P, P, P, P, P, I, F, P])
N.register("sl_bn_bwd_apply", [P, P, P, P, P, L, I, P])
N.register("sl_rsum_floats", [I], ctypes.c_long)
N.register("sl_rsum_result_offset", [I], ctypes.c_long)
N.register("sl_rsum_set_defer", [I])
N.register("sl_conv_set_s2", [I])
N.register("sl_bn_apply_stats", [P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, L, I, I, I, F, F, F, P])
N.register("sl_bn_bwd_apply_sums", [P, P, P, P, P, P, P, P, P, L, I, F, P])
N.register("sl_bn_bwd_apply_dual", [P, P, P, P, P, P, P, P, P, P, P, P, P, L, I, F, P])
N.register("sl_maxpool_fwd", [P, P, P, I, I, I, I, I, I, I, I, I, P])
N.register("sl_maxpool_bwd", [P, P, P, I, I, I, I, I, I, I, I, I, P])
N.register("sl_avgpool_fwd", [P, P, I, I, I, P])
N.register("sl_avgpool_bwd", [P, P, I, I, I, P])
N.register("sl_softmax_ce", [P, P, P, P, P, I, P, I, I, F, P])
N.register("sl_wgrad_side_begin", [P])
N.register("sl_wgrad_side_join", [P, I])
N.register("sl_conv3x3_c64_applicable", [I, I, I, I, I, I, I, I, I])
N.register("sl_conv3x3_bnin_fwd", [P, P, I, I, P, I, P, P, P, P, P, P, P, F, F, F, P])
N.register("sl_conv3x3_bnin_wgrad", [P, P, I, I, P, P, L, P, P, P, F, F, P])

p = N.ptr


def _bf16(t):
    assert t.dtype == torch.bfloat16 and t.is_contiguous(), (t.dtype, t.shape)
    return p(t)


def _f32(t):
    if t is None:
        return None
    assert t.dtype == torch.float32 and t.is_contiguous()
    return p(t)


def rsum_floats(n: int) -> int:
    """Size of a cross-workgroup sum buffer for n values (replicas | result | pad)."""
    return int(N.lib().sl_rsum_floats(n))


class rsum_deferred:
    """While active, the conv / BN-reduce launchers skip their separate BN-sum fold launch and
    the consuming kernels fold the replicas in their prologue (csrc/kernels/common.h,
    rsum_consume).  The ResNet engine wraps its forward and backward in it; standalone calls
    (tests) keep folded result rows right after each producer."""

    def __enter__(self):
        N.call("sl_rsum_set_defer", 1)
        return self

    def __exit__(self, *exc):
        N.call("sl_rsum_set_defer", 0)
        return False


def rsum_result(buf: torch.Tensor, n: int) -> torch.Tensor:
    """The folded result (n floats) inside an rsum buffer."""
    off = int(N.lib().sl_rsum_result_offset(n))
    return buf[off:off + n]


def out_size(h: int, k: int, s: int, pad: int) -> int:
    return (h + 2 * pad - k) // s + 1


def conv_fwd(x, w, cout: int, k: int, stride: int, pad: int, y=None, yf=None, bias=None, stats=None, ldy=None):
    """x [N,H,W,C] bf16, w [cout, k*k*C] bf16 -> y [N,OH,OW,ldy] bf16 and/or yf [N*OH*OW, cout] fp32."""
    n, h, wd, c = x.shape
    oh, ow = out_size(h, k, stride, pad), out_size(wd, k, stride, pad)
    assert w.numel() >= cout * k * k * c
    if y is not None:
        assert y.shape[:3] == (n, oh, ow), (y.shape, n, oh, ow)
        ldy = y.shape[3]
    N.call("sl_conv_fwd", _bf16(x), n, h, wd, c, _bf16(w), cout, k, k, stride, pad, oh, ow,
           _bf16(y) if y is not None else None, int(ldy or cout), _f32(yf), _f32(bias), _f32(stats), N.stream_ptr())
    return oh, ow


def conv_dgrad_s2_even(dy, wt, cin: int, dx):
    """Data gradient of a 1x1 / stride-2 / pad-0 convolution written to the (even, even) positions of
    dx [N,H,W,cin] only; the other positions are left as they are.  A downsample block passes dx
    on as ``add`` with ``add_even=True`` to its strided 3x3 conv1 data gradient, which writes every
    position and adds the shortcut's part at the even ones (csrc/kernels/conv.hip)."""
    n, oh, ow, cd = dy.shape
    _, h, wd, ci = dx.shape
    assert ci == cin and (h + 1) // 2 == oh and (wd + 1) // 2 == ow
    N.call("sl_conv_dgrad_s2_even", _bf16(dy), n, oh, ow, cd, _bf16(wt), cin, h, wd, _bf16(dx), N.stream_ptr())


def conv_dgrad(dy, wt, cin: int, k: int, stride: int, pad: int, dx, add=None, bn=None, add_even: bool = False):
    """dy [N,OH,OW,Cd] bf16 (Cd channels, zero beyond cout), wt [cin, k*k*Cd] -> dx [N,H,W,cin] (+ add).

    ``add_even`` (3x3 stride-2 only): ``add`` holds values at the (even, even) positions only and
    may be dx itself (see :func:`conv_dgrad_s2_even`).

    ``bn``: dx is the gradient at the input of ``relu(bn(x))`` (or of a block output
    ``relu(bn(x) + shortcut)``): a dict with ``x`` (the BN input, dx's shape), ``sums``
    (its zeroed rsum buffer) and the ReLU mask as ``mask_coef`` or ``y_mask`` -- the keys
    of :func:`bn_bwd_reduce`, optionally with ``x2``/``sums2``.  dx is then stored masked
    and the BN-backward sums are accumulated by the conv epilogue, replacing a
    :func:`bn_bwd_reduce` pass (csrc/kernels/bn_bwd_epi.h)."""
    n, oh, ow, cd = dy.shape
    _, h, wd, ci = dx.shape
    assert ci == cin
    if add is not None:
        assert add.shape == dx.shape and add.dtype == torch.bfloat16
    assert not add_even or (add is not None and k == 3 and stride == 2 and pad == 1)
    if bn is None:
        if add_even:
            N.call("sl_conv_dgrad_bnx", _bf16(dy), n, oh, ow, cd, _bf16(wt), cin, k, k, stride, pad, h, wd,
                   _bf16(dx), _bf16(add), None, None, None, None, None, None, 1, N.stream_ptr())
            return
        N.call("sl_conv_dgrad", _bf16(dy), n, oh, ow, cd, _bf16(wt), cin, k, k, stride, pad, h, wd, _bf16(dx),
               _bf16(add) if add is not None else None, N.stream_ptr())
        return
    x, ym, mc, x2 = bn["x"], bn.get("y_mask"), bn.get("mask_coef"), bn.get("x2")
    assert x.shape == dx.shape and dx.is_contiguous() and (ym is None or mc is None)
    if ym is not None:
        assert ym.dtype == torch.uint8 and ym.numel() * 8 == x.numel() and ym.is_contiguous()
    assert (x2 is None) == (bn.get("sums2") is None) and (x2 is None or x2.shape == x.shape)
    N.call("sl_conv_dgrad_bnx", _bf16(dy), n, oh, ow, cd, _bf16(wt), cin, k, k, stride, pad, h, wd, _bf16(dx),
           _bf16(add) if add is not None else None, _bf16(x), p(ym) if ym is not None else None,
           _f32(mc) if mc is not None else None, _f32(bn["sums"]), _bf16(x2) if x2 is not None else None,
           _f32(bn["sums2"]) if x2 is not None else None, 1 if add_even else 0, N.stream_ptr())


# split-K target for the implicit-GEMM weight gradient (workgroups per launch);
# SL_WGRAD_WGS overrides it for A/B runs
_WGRAD_WGS = int(os.environ.get("SL_WGRAD_WGS", "384"))  # re-swept on round-5 kernels: profiles/r05_sweep


NEED_WS = 7  # csrc/kernels/common.h SL_NEED_WS


def deterministic() -> bool:
    """True when the loaded kernel library is the deterministic build (fixed-point
    cross-workgroup sums, no split-K atomics: bit-identical runs)."""
    fn = getattr(N.lib(), "sl_deterministic", None)
    return bool(fn and fn())


class WgradWorkspace:
    """Slab for the weight gradient's split-K partials (plain stores + one ordered reduce
    launch instead of fp32 atomics into dw).  Sized by the launcher's own request: a call
    that finds it too small falls back to atomics and records the size it wanted, and
    :meth:`grow` (outside graph capture) makes the next call fit.  ``alternate``: two slabs
    handed out in turn (:meth:`take`), so a reduce running on a side stream
    (:func:`wgrad_side_begin`) does not block the next weight gradient's slab."""

    def __init__(self, device, floats: int = 0, alternate: bool = False):
        self.device = torch.device(device)
        self.bufs = [torch.empty(max(4, floats), dtype=torch.float32, device=device)
                     for _ in range(2 if alternate else 1)]
        self.i = 0

    @property
    def buf(self):
        return self.bufs[self.i]

    def take(self):
        b = self.bufs[self.i]
        self.i = (self.i + 1) % len(self.bufs)
        return b

    def untake(self) -> None:
        """Hand the slab of the last :meth:`take` out again (a call retried after :meth:`grow`
        keeps the alternation parity it would have had)."""
        self.i = (self.i - 1) % len(self.bufs)

    def grow(self) -> bool:
        need = int(N.lib().sl_conv_wgrad_ws_need())
        if need > self.bufs[0].numel():
            # a side-stream reduce (wgrad_side_begin) may still read the old slabs: let every
            # queued use finish before the caching allocator may hand their memory out again
            # (grow runs eagerly, outside graph capture, and rarely)
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self.bufs = [torch.empty(need, dtype=torch.float32, device=self.device) for _ in self.bufs]
            return True
        return False


def wgrad_side_begin(side_stream) -> None:
    """Route the slab reduces of the following weight gradients to ``side_stream`` (forked from
    the current stream per reduce, so it works inside a hipGraph capture); end with
    :func:`wgrad_side_join`."""
    N.call("sl_wgrad_side_begin", ctypes.c_void_p(side_stream.cuda_stream))


def wgrad_side_join(end: bool = True) -> None:
    """The current stream waits for every reduce issued so far; ``end`` stops the routing."""
    N.call("sl_wgrad_side_join", N.stream_ptr(), 1 if end else 0)


def conv_wgrad(x, dy, cout: int, k: int, stride: int, pad: int, dw, target_wgs: int = 0, ws=None):
    """dw [cout, k*k*C] fp32 += sum over pixels dy^T im2col(x).  ``ws``: WgradWorkspace."""
    n, h, wd, c = x.shape
    _, oh, ow, ldy = dy.shape
    assert dw.dtype == torch.float32 and dw.numel() >= cout * k * k * c
    for attempt in range(2):
        buf = ws.take() if ws is not None else None
        rc = N.lib().sl_conv_wgrad(_bf16(x), n, h, wd, c, _bf16(dy), ldy, cout, k, k, stride, pad, oh, ow, p(dw),
                                   int(target_wgs or _WGRAD_WGS), p(buf), int(buf.numel()) if buf is not None else 0,
                                   N.stream_ptr())
        # deterministic kernel build: no atomic split-K fallback, the workspace must fit (grown
        # here, eagerly: a first step runs before any graph capture)
        if rc == NEED_WS and ws is not None and attempt == 0 and not torch.cuda.is_current_stream_capturing():
            ws.grow()
            ws.untake()
            continue
        if rc != 0:
            raise RuntimeError(f"sl_conv_wgrad failed with code {rc}")
        return


def conv3x3_bnin_applicable(x_shape, cout: int, k: int, stride: int, pad: int) -> bool:
    """Whether :func:`conv3x3_bnin_fwd` / :func:`conv3x3_bnin_wgrad` serve this convolution of a
    BN output: the direct 3x3 kernel's 64 -> 64 / stride-1 / 32-wide case (csrc/kernels/conv3x3_halo.hip)."""
    n, h, w, c = x_shape
    return (c == 64 and cout == 64 and k == 3 and stride == 1 and pad == 1
            and bool(N.lib().sl_conv3x3_c64_applicable(h, w, c, cout, 3, 3, 1, 1, c)))


def conv3x3_bnin_fwd(x, w, bn, count: int, y, stats=None, eps: float = 1e-5, momentum: float = 0.1):
    """y = conv3x3(relu(bn(x))) with the BatchNorm applied to each input chunk between its load and
    the LDS store: bn_apply_stats's output is never written or read back.  ``bn`` exposes stats
    (folded sums), gamma, beta, coef, run_mean, run_var; the kernel publishes coef and the running
    statistics as :func:`bn_apply_stats` would.  ``stats``: the output BN's rsum buffer (folded here)."""
    n, h, wd, c = x.shape
    assert y.shape[:3] == (n, h, wd) and y.is_contiguous()
    N.call("sl_conv3x3_bnin_fwd", _bf16(x), _bf16(w), n, h, _bf16(y), int(y.shape[3]), _f32(stats), _f32(bn.stats),
           _f32(bn.gamma), _f32(bn.beta), _f32(bn.coef), _f32(bn.run_mean), _f32(bn.run_var), float(count),
           float(eps), float(momentum), N.stream_ptr())


def conv3x3_bnin_wgrad(x, dy, bn, count: int, dw, ws=None, eps: float = 1e-5):
    """dw += weight gradient of the convolution fed by :func:`conv3x3_bnin_fwd`: the operand
    relu(bn(x)) is rebuilt on load from the BN input ``x`` (same bf16 values as the forward)."""
    n, h, wd, c = x.shape
    assert dy.shape == (n, h, wd, 64) and dw.dtype == torch.float32 and dw.numel() >= 64 * 9 * 64
    for attempt in range(2):
        buf = ws.take() if ws is not None else None
        rc = N.lib().sl_conv3x3_bnin_wgrad(_bf16(x), _bf16(dy), n, h, p(dw), p(buf),
                                           int(buf.numel()) if buf is not None else 0, _f32(bn.stats),
                                           _f32(bn.gamma), _f32(bn.beta), float(count), float(eps), N.stream_ptr())
        if rc == NEED_WS and ws is not None and attempt == 0 and not torch.cuda.is_current_stream_capturing():
            ws.grow()
            ws.untake()
            continue
        if rc != 0:
            raise RuntimeError(f"sl_conv3x3_bnin_wgrad failed with code {rc}")
        return


class WtDesc(ctypes.Structure):
    _fields_ = [("w", ctypes.c_void_p), ("wt", ctypes.c_void_p), ("cout", ctypes.c_int), ("taps", ctypes.c_int),
                ("cin", ctypes.c_int), ("ldt", ctypes.c_int), ("begin", ctypes.c_long)]


class WeightTransposer:
    """Multi-tensor Wt[ci][tap][co] = W[co][tap][ci] for every conv (one launch)."""

    def __init__(self, items, device):
        """items: [(w_bf16_view, wt_bf16_view, cout, taps, cin, ldt)]"""
        assert ctypes.sizeof(WtDesc) == N.lib().sl_conv_wt_desc_size()
        arr = (WtDesc * len(items))()
        total = 0
        for i, (w, wt, cout, taps, cin, ldt) in enumerate(items):
            assert wt.numel() == cin * taps * ldt and w.numel() >= cout * taps * cin
            arr[i] = WtDesc(p(w), p(wt), cout, taps, cin, ldt, total)
            total += taps * ((ldt + 63) // 64) * ((cin + 63) // 64)  # 64x64 tiles
        host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        self.desc = host.to(device)
        self.n = len(items)
        self.total = total

    def __call__(self):
        N.call("sl_conv_wt", p(self.desc), self.n, self.total, N.stream_ptr())


def input_norm(x_u8, labels, cursor, batch: int, y, lab_out, mean, std):
    """Batch ``cursor % n_batches`` of the shard x_u8 [n,H,W,3] -> y [batch,H,W,8] bf16 (+ labels)."""
    assert x_u8.dtype == torch.uint8 and x_u8.shape[-1] == 3 and y.shape[-1] == 8
    img = x_u8.shape[1] * x_u8.shape[2]
    n_batches = x_u8.shape[0] // batch
    assert n_batches >= 1 and y.shape[0] == batch
    N.call("sl_input_norm", p(x_u8), p(labels), p(cursor), n_batches, batch, img, _bf16(y), p(lab_out),
           *[float(v) for v in mean], *[float(v) for v in std], N.stream_ptr())


def cursor_bump(cursor):
    N.call("sl_cursor_bump", p(cursor), N.stream_ptr())


def bn_finalize(stats, gamma, beta, coef, run_mean, run_var, count, eps=1e-5, momentum=0.1):
    c = gamma.numel()
    N.call("sl_bn_finalize", _f32(stats), _f32(gamma), _f32(beta), _f32(coef), _f32(run_mean), _f32(run_var), c,
           float(count), float(eps), float(momentum), N.stream_ptr())


def bn_apply(x, coef, y, relu=True, res=None, rcoef=None):
    c = x.shape[-1]
    rows = x.numel() // c
    mode = 0 if res is None else (2 if rcoef is not None else 1)
    N.call("sl_bn_apply", _bf16(x), _f32(coef), _bf16(res) if res is not None else None, _f32(rcoef), _bf16(y),
           rows, c, 1 if relu else 0, mode, N.stream_ptr())


def bn_bwd_reduce(dy, y, x, sums, dz_out=None, mask_coef=None, y_mask=None, x2=None, sums2=None):
    """dz = dy * relu'(.) and the per-channel sums for the BN backward.  The ReLU
    mask comes from ``y`` (block outputs with a residual) or, for a plain
    ``y = relu(bn(x))``, from ``x`` and the layer's forward ``mask_coef``
    (scale/shift rows of ``coef``), so ``y`` is never read.  ``y_mask`` is the
    1-bit-per-channel ReLU mask written by :func:`bn_apply_stats` (``mask_out``)
    for block outputs with a residual: 1/16 of the bytes of ``y``.  ``x2``/``sums2``
    add the sums of a second BN fed by the same dz (the downsample shortcut's
    input ``cs``), so dz is not read back for it."""
    c = x.shape[-1]
    rows = x.numel() // c
    assert (y is not None) + (mask_coef is not None) + (y_mask is not None) <= 1
    assert (x2 is None) == (sums2 is None) and (x2 is None or x2.shape == x.shape)
    if y_mask is not None:
        assert y_mask.dtype == torch.uint8 and y_mask.numel() * 8 == x.numel() and y_mask.is_contiguous()
    N.call("sl_bn_bwd_reduce", _bf16(dy), _bf16(y) if y is not None else None, _bf16(x),
           _f32(mask_coef) if mask_coef is not None else None, p(y_mask) if y_mask is not None else None,
           _bf16(dz_out) if dz_out is not None else None, _f32(sums),
           _bf16(x2) if x2 is not None else None, _f32(sums2) if sums2 is not None else None, rows, c,
           N.stream_ptr())


def bn_bwd_finalize(sums, coef, dcoef, grad_gamma, grad_beta, count):
    c = grad_gamma.numel()
    N.call("sl_bn_bwd_finalize", _f32(sums), _f32(coef), _f32(dcoef), _f32(grad_gamma), _f32(grad_beta), c,
           float(count), N.stream_ptr())


def bn_bwd_apply(dy, y, x, dcoef, dx):
    c = x.shape[-1]
    rows = x.numel() // c
    N.call("sl_bn_bwd_apply", _bf16(dy), _bf16(y) if y is not None else None, _bf16(x), _f32(dcoef), _bf16(dx),
           rows, c, N.stream_ptr())


def bn_apply_stats(x, bn, y, count, relu=True, res=None, rbn=None, eps=1e-5, momentum=0.1, mask_out=None,
                   res_relu=False):
    """Fused finalize + apply; ``bn``/``rbn`` expose stats, gamma, beta, coef, run_mean, run_var.
    ``mask_out`` (u8, numel/8) receives bit j of byte q = ``y[8q+j] > 0``.  ``res_relu``: the
    residual is ``relu(rbn(res))`` (a BN-on-load block input, whose BN was published by the
    conv that consumed it; ``rbn``'s coef / running stats are not written here)."""
    if mask_out is not None:
        assert mask_out.dtype == torch.uint8 and mask_out.numel() * 8 == x.numel() and mask_out.is_contiguous()
    c = x.shape[-1]
    rows = x.numel() // c
    mode = 0 if res is None else ((3 if res_relu else 2) if rbn is not None else 1)
    assert not res_relu or rbn is not None
    r = rbn
    N.call("sl_bn_apply_stats", _bf16(x), _f32(bn.stats), _f32(bn.gamma), _f32(bn.beta), _f32(bn.coef),
           _f32(bn.run_mean), _f32(bn.run_var), _bf16(res) if res is not None else None,
           _f32(r.stats) if r else None, _f32(r.gamma) if r else None, _f32(r.beta) if r else None,
           _f32(r.coef) if r else None, _f32(r.run_mean) if r else None, _f32(r.run_var) if r else None,
           _bf16(y), p(mask_out) if mask_out is not None else None, rows, c, 1 if relu else 0, mode, float(count), float(eps), float(momentum), N.stream_ptr())


def bn_bwd_apply_sums(dy, y, x, sums, coef, grad_gamma, grad_beta, dx, mask_coef=None):
    """Fused backward finalize + apply: dx, and dgamma/dbeta accumulated into the flat gradient.
    ``mask_coef`` as in :func:`bn_bwd_reduce`."""
    c = x.shape[-1]
    rows = x.numel() // c
    assert y is None or mask_coef is None
    N.call("sl_bn_bwd_apply_sums", _bf16(dy), _bf16(y) if y is not None else None, _bf16(x),
           _f32(mask_coef) if mask_coef is not None else None, _f32(sums),
           _f32(coef), _f32(grad_gamma), _f32(grad_beta), _bf16(dx), rows, c, float(rows), N.stream_ptr())


def bn_bwd_apply_dual(dz, xa, sums_a, coef_a, gg_a, gb_a, dx_a, xb, sums_b, coef_b, gg_b, gb_b, dx_b):
    """:func:`bn_bwd_apply_sums` for two BNs fed by the same ``dz`` (a downsample
    block's bn2 and shortcut BN), reading ``dz`` once."""
    c = xa.shape[-1]
    rows = xa.numel() // c
    assert xb.shape == xa.shape == dz.shape == dx_a.shape == dx_b.shape
    N.call("sl_bn_bwd_apply_dual", _bf16(dz), _bf16(xa), _f32(sums_a), _f32(coef_a), _f32(gg_a), _f32(gb_a),
           _bf16(dx_a), _bf16(xb), _f32(sums_b), _f32(coef_b), _f32(gg_b), _f32(gb_b), _bf16(dx_b), rows, c,
           float(rows), N.stream_ptr())


def maxpool_fwd(x, y, arg, k=3, s=2, pad=1):
    n, h, w, c = x.shape
    _, oh, ow, _ = y.shape
    N.call("sl_maxpool_fwd", _bf16(x), _bf16(y), p(arg), n, h, w, c, oh, ow, k, s, pad, N.stream_ptr())


def maxpool_bwd(dy, arg, dx, k=3, s=2, pad=1):
    n, h, w, c = dx.shape
    _, oh, ow, _ = dy.shape
    N.call("sl_maxpool_bwd", _bf16(dy), p(arg), _bf16(dx), n, h, w, c, oh, ow, k, s, pad, N.stream_ptr())


def avgpool_fwd(x, y):
    n, h, w, c = x.shape
    N.call("sl_avgpool_fwd", _bf16(x), _bf16(y), n, h * w, c, N.stream_ptr())


def avgpool_bwd(dy, dx):
    n, h, w, c = dx.shape
    N.call("sl_avgpool_bwd", _bf16(dy), _bf16(dx), n, h * w, c, N.stream_ptr())


def softmax_ce(logits, labels, loss, correct, dlogits, dbias, grad_scale):
    n, ncls = logits.shape
    N.call("sl_softmax_ce", _f32(logits), p(labels), _f32(loss), _f32(correct), _bf16(dlogits), dlogits.shape[-1],
           _f32(dbias), n, ncls, float(grad_scale), N.stream_ptr())
