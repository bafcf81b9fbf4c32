"""The flagship model: a 3-layer MLP (784-256-256-10) on MNIST-shaped data.

The reference has no model at all -- its "model" is a ``std::vector<double>``
that ``simulate_training`` bumps by one every 2 s
(/root/reference/src/worker.cc:221-231) and that workers mix by gossip
(/root/reference/src/worker.cc:81-100).  This module provides the real model
that takes its place, in three forms:

* :func:`param_layout` / :func:`init_params` -- the flat fp32 parameter vector.
  A flat vector is what travels in the reference's ``Update{repeated double
  delta}`` message (proto :81-83), what the checkpoint format stores and what
  the data-parallel all-reduce moves in one bucket.
* :class:`MLP` -- a ``torch.nn.Module`` view of that vector, used on CPU
  workers (BASELINE config 1, "plumbing, no GPU") and as the fp32 reference
  in numerics tests.
* :class:`FusedMLPTrainer` -- the MI355X path: three hand-written HIP kernels
  per step (csrc/kernels/mlp_fused.hip) on bf16 MFMA with fp32 master
  weights, optionally wrapped in a hipGraph, with an RCCL all-reduce hook.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..utils.graphs import GraphSlots

D_IN = 784
D_IN_PAD = 832  # w1h row stride: layer-1 K in 13 chunks of 64 (mlp_fused.hip)
HIDDEN = 256
CLASSES = 10
MNIST_MEAN = 0.1307
MNIST_STD = 0.3081
BLOCK_ROWS = 64  # batch rows per workgroup of the fused row kernel
W3P_LD = 3088  # row stride of the rows kernel's partial rows: [dW3 | db3 | pad | db1 | db2]
R1_BLK = 25  # 32-column blocks per W1 row: fixed-point partial row sums of the fp16 shadow
R1_OVF_MIN = 1 << 51  # a partial row sum at or past this flags a W1 weight beyond fp16 (mlp_fused.hip)

LAYOUT = (
    ("fc1.weight", (HIDDEN, D_IN)),
    ("fc1.bias", (HIDDEN,)),
    ("fc2.weight", (HIDDEN, HIDDEN)),
    ("fc2.bias", (HIDDEN,)),
    ("fc3.weight", (CLASSES, HIDDEN)),
    ("fc3.bias", (CLASSES,)),
)


def param_layout():
    """[(name, shape, offset, numel)] of the flat parameter vector."""
    out, off = [], 0
    for name, shape in LAYOUT:
        n = math.prod(shape)
        out.append((name, shape, off, n))
        off += n
    return out


N_PARAMS = sum(math.prod(s) for _, s in LAYOUT)  # 269,322
N_PARAMS_B1 = HIDDEN * D_IN  # offset of fc1.bias in the flat vector


def norm_coeffs(mean: float = MNIST_MEAN, std: float = MNIST_STD) -> tuple[float, float]:
    """u8 pixel p -> (p/255 - mean)/std == p*a + b."""
    return 1.0 / (255.0 * std), -mean / std


def init_params(seed: int = 0, device="cpu") -> torch.Tensor:
    """nn.Linear default init (U(-1/sqrt(fan_in), 1/sqrt(fan_in))) into a flat fp32 vector."""
    g = torch.Generator().manual_seed(seed)
    flat = torch.empty(N_PARAMS, dtype=torch.float32)
    for name, shape, off, n in param_layout():
        fan_in = shape[1] if len(shape) == 2 else (D_IN if name.startswith("fc1") else HIDDEN)
        bound = 1.0 / math.sqrt(fan_in)
        flat[off:off + n] = (torch.rand(n, generator=g) * 2 - 1) * bound
    return flat.to(device)


def views(flat: torch.Tensor) -> dict:
    return {name: flat[off:off + n].view(shape) for name, shape, off, n in param_layout()}


def normalize(x_u8: torch.Tensor) -> torch.Tensor:
    a, b = norm_coeffs()
    return x_u8.float() * a + b


class MLP(nn.Module):
    """nn.Module over a flat parameter vector (CPU path and fp32 reference)."""

    def __init__(self, flat: torch.Tensor | None = None, seed: int = 0):
        super().__init__()
        if flat is None:
            flat = init_params(seed)
        self.flat = nn.Parameter(flat.clone().float())

    def forward(self, x_u8: torch.Tensor) -> torch.Tensor:
        v = views(self.flat)
        h = normalize(x_u8.reshape(-1, D_IN))
        h = F.relu(F.linear(h, v["fc1.weight"], v["fc1.bias"]))
        h = F.relu(F.linear(h, v["fc2.weight"], v["fc2.bias"]))
        return F.linear(h, v["fc3.weight"], v["fc3.bias"])


def reference_grads(flat: torch.Tensor, x_u8: torch.Tensor, y: torch.Tensor,
                    grad_scale: float | None = None):
    """fp32 autograd reference: (loss_sum, correct, grad_flat) with dZ scaled by grad_scale."""
    w = flat.detach().clone().float().requires_grad_(True)
    m = MLP.__new__(MLP)
    nn.Module.__init__(m)
    m.flat = w
    logits = m(x_u8)
    losses = F.cross_entropy(logits, y.long(), reduction="none")
    scale = grad_scale if grad_scale is not None else 1.0 / x_u8.shape[0]
    (losses.sum() * scale).backward()
    correct = (logits.argmax(1) == y.long()).float().sum()
    return losses.detach().sum(), correct.detach(), w.grad.detach()


def reference_grads_bf16(flat: torch.Tensor, x_u8: torch.Tensor, y: torch.Tensor, grad_scale: float):
    """fp32 math with bf16 rounding at exactly the points the fused kernels round.

    A tight check of csrc/kernels/mlp_fused.hip: any indexing/layout bug shows
    up as an O(1) error, while legitimate differences are fp32 summation order.
    Returns (loss_sum, correct, grad_flat).
    """
    r = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    v = {k: t.detach().float() for k, t in views(flat).items()}
    a, b = norm_coeffs()
    # layer 1: exact normalised pixels against the fp16 W1 shadow (the kernel multiplies the
    # exact pixels 1024 + u and removes the offset with W1's exact row sums)
    xe = x_u8.reshape(-1, D_IN).float() * a + b
    w1 = v["fc1.weight"].to(torch.float16).float()
    w2, w3 = r(v["fc2.weight"]), r(v["fc3.weight"])
    p1 = xe @ w1.t() + v["fc1.bias"]
    h1 = r(torch.relu(p1))
    p2 = h1 @ w2.t() + v["fc2.bias"]
    h2 = r(torch.relu(p2))
    z = h2 @ w3.t() + v["fc3.bias"]
    yl = y.reshape(-1).long()
    losses = torch.logsumexp(z, 1) - z.gather(1, yl[:, None])[:, 0]
    dz = r((torch.softmax(z, 1) - F.one_hot(yl, CLASSES).float()) * grad_scale)
    dh2 = r((dz @ w3) * (p2 > 0).float())
    dh1 = r((dh2 @ w2) * (p1 > 0).float())
    # dW1 uses the exact normalised input too: the weight-gradient kernel multiplies the raw
    # u8 pixels (exact in fp16) and applies the normalisation affinely afterwards
    g = torch.cat([(dh1.t() @ xe).reshape(-1), dh1.sum(0), (dh2.t() @ h1).reshape(-1), dh2.sum(0),
                   (dz.t() @ h2).reshape(-1), dz.sum(0)])
    correct = (z.argmax(1) == yl).float().sum()
    return losses.sum(), correct, g


def sgd_update(flat, mom, grad, lr, momentum, weight_decay):
    """torch.optim.SGD semantics (dampening 0, no nesterov), in place."""
    d = grad + weight_decay * flat
    if mom is not None:
        mom.mul_(momentum).add_(d)
        d = mom
    flat.sub_(lr * d)


@dataclass
class StepStats:
    loss: float
    accuracy: float
    samples: int


class CPUTrainer:
    """Plain-torch trainer with the same interface as FusedMLPTrainer (CPU workers)."""

    def __init__(self, batch: int, lr: float = 0.05, momentum: float = 0.9,
                 weight_decay: float = 0.0, seed: int = 0, world_size: int = 1,
                 flat: torch.Tensor | None = None):
        self.batch = batch
        self.lr, self.momentum, self.weight_decay = lr, momentum, weight_decay
        self.world_size = world_size
        self.params = (flat if flat is not None else init_params(seed)).clone().float()
        self.mom = torch.zeros_like(self.params) if momentum > 0 else None
        self.cursor = 0
        self.x = self.y = None
        self.allreduce = None  # callable(tensor) -> None (sum in place)
        self._last = None
        from ..utils.phases import PhaseProbe

        self.phases = PhaseProbe("cpu")

    n_params = N_PARAMS
    model_name = "mlp-784-256-256-10"

    def layout(self):
        return [[n, list(s), o] for n, s, o, _ in param_layout()]

    def set_world(self, world: int) -> None:
        self.world_size = world

    def refresh_shadows(self) -> None:
        pass

    def load_shard(self, x_u8: torch.Tensor, y_u8: torch.Tensor) -> None:
        assert x_u8.shape[0] >= self.batch
        self.x, self.y = x_u8.reshape(-1, D_IN), y_u8.reshape(-1)
        self.n_batches = self.x.shape[0] // self.batch

    def step(self) -> None:
        b = self.cursor % self.n_batches
        xs = self.x[b * self.batch:(b + 1) * self.batch]
        ys = self.y[b * self.batch:(b + 1) * self.batch]
        loss, correct, g = reference_grads(self.params, xs, ys, 1.0 / (self.batch * self.world_size))
        self.phases.mark("compute")
        if self.allreduce is not None:
            self.allreduce(g)
        self.phases.mark("exchange")
        sgd_update(self.params, self.mom, g, self.lr, self.momentum, self.weight_decay)
        self.cursor += 1
        self.phases.mark("update")
        self._last = (float(loss), float(correct))

    def probe_step(self):
        """One training step with its phases timed (utils/phases.py; wall clock on the CPU):
        a PendingPhases, ready at once."""
        self.phases.arm()
        self.step()
        pending = self.phases.finish()
        pending.exchange_bytes = 4 * int(self.params.numel()) if self.allreduce is not None else 0
        return pending

    def stats(self) -> StepStats:
        loss, correct = self._last
        return StepStats(loss / self.batch, correct / self.batch, self.batch)

    def get_flat(self) -> torch.Tensor:
        return self.params.clone()

    def set_flat(self, flat: torch.Tensor) -> None:
        self.params.copy_(flat.to(self.params))

    def state_extra(self) -> dict:
        return {"cursor": np.array([self.cursor], dtype=np.float64)}

    def load_state_extra(self, d: dict) -> None:
        if "cursor" in d:
            self.cursor = int(d["cursor"][0])

    def buffers(self) -> list:
        return []


def dh1_scale(grad_scale: float) -> float:
    """Power of two that brings grad_scale-sized dH1 values to O(1) before the rows kernel
    stores them as fp16 for the weight gradient (fp16 would flush them to subnormals)."""
    return 2.0 ** round(-math.log2(grad_scale))


def dw1_coeffs(xa: float, xb: float, scale: float) -> tuple:
    """(a, b) with dW1 = a * slab + b * db1.  The slab holds scale * dH1^T (X + 1024) (the fp16
    GEMM on raw pixels, u -> 1024 + u exactly), and dW1 of the normalised input xa X + xb is
    xa dH1^T X + xb db1 = (xa / scale) slab + (xb - 1024 xa) db1."""
    return xa / scale, xb - 1024.0 * xa


def default_slices(batch: int) -> int:
    """Split-K slices of the weight-gradient GEMM (the kernel's own choice: one workgroup per CU)."""
    from ..ops import _native

    return int(_native.lib().sl_mlp_wgrad_slices(batch, 0))


class FusedMLPTrainer(GraphSlots):
    """MI355X training engine for the MLP: 3 HIP launches per step.

    Buffers are allocated once for a fixed per-GPU batch; the data shard stays
    resident in HBM and a device-side cursor selects the batch, so a step has
    no host work and replays from a hipGraph (:meth:`capture`).
    """

    def __init__(self, batch: int, device="cuda", lr: float = 0.05, momentum: float = 0.9,
                 weight_decay: float = 0.0, seed: int = 0, world_size: int = 1,
                 slices: int | None = None, flat: torch.Tensor | None = None):
        from ..ops import _native

        if batch % BLOCK_ROWS != 0:
            raise ValueError(f"batch must be a multiple of {BLOCK_ROWS}")
        self._n = _native
        _native.lib()  # fail loudly if the HIP library cannot be loaded
        if os.environ.get("SL_MLP_ROWS_BM"):  # force the rows kernel's tile height (64 / 128)
            _native.call("sl_mlp_set_rows_bm", int(os.environ["SL_MLP_ROWS_BM"]))
        dev = torch.device(device)
        self.device = dev
        self.batch = batch
        self.lr, self.momentum, self.weight_decay = lr, momentum, weight_decay
        self.world_size = world_size
        self.grad_scale = 1.0 / (batch * world_size)
        s1 = slices or int(os.environ.get("SL_MLP_WG_SLICES", "0") or 0)  # split-K slices (0: library default)
        self.slices = int(_native.lib().sl_mlp_wgrad_slices(batch, s1))
        if self.slices <= 0:
            raise ValueError(f"batch {batch} not supported by the weight-gradient kernel")
        self.xa, self.xb = norm_coeffs()
        n = N_PARAMS
        self.n_pad = (n + 3) // 4 * 4
        self.params = torch.zeros(self.n_pad, dtype=torch.float32, device=dev)
        init = flat if flat is not None else init_params(seed)
        self.params[:n].copy_(init.to(dev))
        self.mom = torch.zeros_like(self.params) if momentum > 0 else None
        bf = torch.bfloat16
        # W1's shadow is fp16: layer 1 multiplies the exact pixels (fp16 1024 + u) and corrects the
        # offset with the W1 row sums, kept as 64-bit fixed-point partials (mlp_fused.hip, R1_BLK)
        self.w1h = torch.zeros(HIDDEN, D_IN_PAD, dtype=torch.float16, device=dev)
        self.r1p = torch.zeros(HIDDEN * R1_BLK, dtype=torch.int64, device=dev)
        self.w2h = torch.zeros(HIDDEN, HIDDEN, dtype=bf, device=dev)
        self.w2th = torch.zeros(HIDDEN, HIDDEN, dtype=bf, device=dev)
        self.w3h = torch.zeros(16, HIDDEN, dtype=bf, device=dev)
        self.w3th = torch.zeros(HIDDEN, 32, dtype=bf, device=dev)
        # row-major activations for the weight-gradient kernel ([batch][256], dZ [batch][16])
        self.h1t = torch.empty(batch, HIDDEN, dtype=bf, device=dev)
        self.dh1t = torch.empty(batch, HIDDEN, dtype=bf, device=dev)
        self.dh2t = torch.empty(batch, HIDDEN, dtype=bf, device=dev)
        # per-64-row partials of [dW3 | db3] from the rows kernel (H2 / dZ never reach HBM)
        self.w3p = torch.empty(batch // 64, W3P_LD, dtype=torch.float32, device=dev)
        self.loss = torch.zeros(batch, dtype=torch.float32, device=dev)
        self.correct = torch.zeros(batch, dtype=torch.float32, device=dev)
        # per-slice stride of the weight-gradient slab (the kernel library's layout: tiled in the
        # wgrad kernel's register order, larger than the parameter count)
        lib = _native.lib()
        # (older kernel builds, kept for A/B runs, have no tiled layout and no stride query)
        self.slab_stride = int(lib.sl_mlp_slab_stride()) if hasattr(lib, "sl_mlp_slab_stride") else self.n_pad
        self.slab = torch.empty(self.slices, self.slab_stride, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.n_pad, dtype=torch.float32, device=dev)
        self.cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        self.allreduce = None  # callable(grad_tensor) -> None, sums in place (RCCL)
        self.xgmi = None       # parallel.xgmi.XgmiExchange: all-reduce fused into the update (no RCCL)
        self.x = self.y = None
        self.n_batches = 1
        self.graph = None
        from ..utils.phases import PhaseProbe

        self.phases = PhaseProbe(dev)
        self.refresh_shadows()
        # torch loads its reduction kernel's code object on first use (~27 ms): take that here,
        # at construction, not in the first logged chunk of a training worker (profiles/r04_runtime)
        self.stats()

    n_params = N_PARAMS
    model_name = "mlp-784-256-256-10"

    def layout(self):
        return [[n, list(s), o] for n, s, o, _ in param_layout()]

    def set_world(self, world: int) -> None:
        """Gradient scale follows the group size (mean over the global batch)."""
        self.world_size = world
        self.grad_scale = 1.0 / (self.batch * world)
        self.graph = None

    # ---- data ----
    def load_shard(self, x_u8: torch.Tensor, y_u8: torch.Tensor) -> None:
        """Make a device-resident shard current ([N,784] u8 images, [N] u8 labels)."""
        x = x_u8.reshape(-1, D_IN)
        if x.shape[0] < self.batch:
            raise ValueError("shard smaller than one batch")
        self.x = x.to(self.device, non_blocking=True).contiguous()
        self.y = y_u8.reshape(-1).to(self.device, non_blocking=True).to(torch.uint8).contiguous()
        self.n_batches = self.x.shape[0] // self.batch
        self.graph = None

    # ---- kernels ----
    def refresh_shadows(self) -> None:
        n = self._n
        n.call("sl_mlp_sgd", n.ptr(self.params), None, None, 0, 0, None, None, 0.0, 0.0, 0.0, self.xa, self.xb, 0,
               n.ptr(self.w1h), n.ptr(self.w2h), n.ptr(self.w2th), n.ptr(self.w3h), n.ptr(self.w3th),
               None, n.ptr(self.r1p), n.stream_ptr())

    @property
    def dh1_scale(self) -> float:
        return dh1_scale(self.grad_scale)

    @property
    def dw1_coeffs(self) -> tuple:
        return dw1_coeffs(self.xa, self.xb, self.dh1_scale)

    def _launches(self):
        """Cached launches for the current buffers/hyper-parameters (rebuilt on change)."""
        key = (self.x.data_ptr() if self.x is not None else 0, self.n_batches, self.grad_scale, self.lr,
               self.momentum, self.weight_decay, id(self.xgmi), bool(self.xgmi and self.xgmi.two_shot),
               self.xgmi.inline_sync if self.xgmi is not None else None)
        if getattr(self, "_lkey", None) == key:
            return self._lc
        n, p = self._n, self._n.ptr
        ws = (p(self.w1h), p(self.w2h), p(self.w2th), p(self.w3h), p(self.w3th))
        lc = {
            "rows": n.Launch("sl_mlp_rows", p(self.x), p(self.y), p(self.cursor), self.n_batches, self.batch,
                             p(self.w1h), p(self.w2h), p(self.w3h), p(self.w2th), p(self.w3th),
                             p(self.params), self.xa, self.xb, self.grad_scale, self.dh1_scale,
                             p(self.h1t), p(self.w3p), p(self.dh2t), p(self.dh1t),
                             p(self.loss), p(self.correct), None, 1, p(self.r1p),
                             # xGMI inline synchronisation: this launch advances the exchange's step id
                             self.xgmi.ctl.data_ptr() if self.xgmi is not None and self.xgmi.inline_sync else None),
            "wgrad": n.Launch("sl_mlp_wgrad", self.batch, p(self.x), p(self.cursor), self.n_batches,
                              p(self.h1t), p(self.dh2t), p(self.dh1t), p(self.w3p), self.w3p.shape[0], p(self.slab),
                              self.slices, self.slab_stride),
        }
        for name, (mode, from_grad, grad_out, bump) in {"sgd": (2, False, False, True),
                                                        "reduce": (1, False, True, False),
                                                        "update": (2, True, False, True)}.items():
            lc[name] = n.Launch("sl_mlp_sgd", p(self.params), p(self.mom),
                                None if from_grad else p(self.slab), self.slices, self.slab_stride,
                                p(self.grad) if from_grad else None, p(self.grad) if grad_out else None,
                                self.lr, self.momentum, self.weight_decay, *self.dw1_coeffs, mode, *ws,
                                p(self.cursor) if bump else None, p(self.r1p))
        if self.xgmi is not None:
            xg = self.xgmi
            # inline synchronisation: the reduce publishes the step, the update waits per workgroup
            lc["xreduce"] = n.Launch("sl_mlp_reduce_xgmi", p(self.slab), self.slices, self.slab_stride, *self.dw1_coeffs,
                                     xg.slot_ptr(0), xg.slot_ptr(1), *xg.args(), xg.inline_sync)
            lc["xbarrier"] = [n.Launch(fn, *xg.args(), *extra) for fn, extra in xg.exchange_launches(self.n_pad)]
            lc["xupdate"] = n.Launch("sl_mlp_sgd_xgmi", p(self.params), p(self.mom), self.lr, self.momentum,
                                     self.weight_decay, *ws, p(self.cursor), *xg.args(), p(self.r1p), xg.inline_sync)
        self._lc, self._lkey = lc, key
        return lc

    def _rows(self, train: bool = True):
        if train:
            return self._launches()["rows"]()
        n = self._n
        n.call("sl_mlp_rows", n.ptr(self.x), n.ptr(self.y), n.ptr(self.cursor), self.n_batches, self.batch,
               n.ptr(self.w1h), n.ptr(self.w2h), n.ptr(self.w3h), n.ptr(self.w2th), n.ptr(self.w3th),
               n.ptr(self.params), self.xa, self.xb, self.grad_scale, self.dh1_scale,
               n.ptr(self.h1t), n.ptr(self.w3p), n.ptr(self.dh2t), n.ptr(self.dh1t),
               n.ptr(self.loss), n.ptr(self.correct), None, 0, n.ptr(self.r1p), None, n.stream_ptr())

    def _wgrad(self):
        self._launches()["wgrad"]()

    def _sgd(self, mode: int, from_grad: bool, grad_out: bool, bump: bool = True):
        name = {(2, False, False, True): "sgd", (1, False, True, False): "reduce",
                (2, True, False, True): "update"}[(mode, from_grad, grad_out, bump)]
        self._launches()[name]()

    def compute_grads(self) -> torch.Tensor:
        """Forward + backward only; returns the reduced (local) gradient (not with an xGMI
        exchange enabled: its rows launch advances the exchange's step id)."""
        self._rows(True)
        self._wgrad()
        self._sgd(1, from_grad=False, grad_out=True, bump=False)
        return self.grad[:N_PARAMS]

    def step(self) -> None:
        if self.graph is not None:
            self.graph.replay()
            return
        self._step_eager()

    def steps(self, n: int) -> None:
        """Run ``n`` full training steps.  With a multi-step graph captured
        (``capture(unroll=k)``) they replay k at a time: the ~8 us gap that every
        graph launch leaves between the previous step's SGD and the next rows
        kernel is paid once per k steps (every step still runs all three kernels
        on its own batch; the device cursor advances inside the graph)."""
        g, k = getattr(self, "graph_unrolled", None), getattr(self, "unroll", 1)
        if self.graph is not None and g is not None and k > 1:  # self.graph=None invalidates both
            while n >= k:
                g.replay()
                n -= k
        for _ in range(n):
            self.step()

    def enable_xgmi(self, exchange) -> None:
        """Aggregate gradients through an :class:`~serverless_learn_amd.parallel.xgmi.XgmiExchange`
        (the slab reduction lands in this rank's exchange slot; the update kernel sums every
        rank's slot over xGMI and applies SGD).  ``None`` switches back."""
        if exchange is not None and exchange.payload_floats < self.n_pad:
            raise ValueError("exchange slot smaller than the parameter vector")
        self.xgmi = exchange
        self.graph = None
        self._lkey = None

    def enable_clock_probe(self, cap: int = 16 * 2048) -> None:
        """Diagnostics (bench.py SL_CLOCK_PROBE=1): a 16-workgroup kernel stamps (XCC id,
        shader clock, 100 MHz wall clock) at the start of every step, inside the captured
        graphs too (csrc/kernels/diag.hip)."""
        self.probe_buf = torch.zeros(3 * cap, dtype=torch.int64, device=self.device)
        self.probe_cnt = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.probe = self._n.Launch("sl_clock_probe", self._n.ptr(self.probe_buf), self._n.ptr(self.probe_cnt), cap)
        self.graph = None

    def clock_probe_steps(self) -> list:
        """Per probed step boundary: (wall time in us of the 100 MHz clock, {xcc: shader ticks})."""
        n = min(int(self.probe_cnt.item()), self.probe_buf.numel() // 3)
        rec = self.probe_buf[:3 * n].view(n, 3).cpu().tolist()
        out = []
        for i in range(0, n - n % 16, 16):  # one launch = 16 consecutive records
            grp = rec[i:i + 16]
            wall = min(r[2] for r in grp)
            ticks = {}
            for x, t, w in grp:
                ticks.setdefault(x, (t, w))
            out.append((wall, ticks))
        return out

    def _step_eager(self) -> None:
        if getattr(self, "probe", None) is not None:
            self.probe()
        ph = self.phases
        self._rows(True)
        self._wgrad()
        ph.mark("compute")
        if self.xgmi is not None:
            lc = self._launches()
            lc["xreduce"]()
            for launch in lc["xbarrier"]:
                launch()
            ph.mark("exchange")  # slab reduction into the exchange slot + the step barrier(s)
            lc["xupdate"]()      # (the peers' slots are summed inside the update kernel)
        elif self.allreduce is None:
            self._sgd(2, from_grad=False, grad_out=False)
        else:
            self._sgd(1, from_grad=False, grad_out=True, bump=False)
            self.allreduce(self.grad)
            ph.mark("exchange")
            self._sgd(2, from_grad=True, grad_out=False)
        ph.mark("update")

    def probe_step(self):
        """One eager training step with its phase boundaries recorded (utils/phases.py): returns
        a PendingPhases (resolved by the caller once the device has finished the step) carrying
        the gradient payload aggregated per step (fp32 bytes, 0 at world 1)."""
        self.phases.arm()
        self._step_eager()
        pending = self.phases.finish()
        pending.exchange_bytes = 4 * N_PARAMS if (self.allreduce is not None or self.xgmi is not None) else 0
        return pending

    def drop_graphs(self) -> None:
        """Release every captured step graph after the device has finished with them.  A
        graph may hold a communicator's kernels: the runtime calls this before it re-forms or
        tears down the group, so no replay is in flight when the old
        communicator goes away and the k-step graph is not left alive holding it."""
        if self.graph is not None or self.retired_graphs:  # steps() ignores graph_unrolled once graph is None
            torch.cuda.synchronize(self.device)
        self.graph = None
        self.graph_unrolled = None
        self.reap_graphs(sync=False)

    def capture(self, warmup: int = 2, unroll: int = 1) -> None:
        """Capture one step into a hipGraph (kernels only, or kernels + RCCL);
        ``unroll > 1`` also captures a k-step graph used by :meth:`steps`.  Graphs replaced
        since the last capture are freed first, after a device sync (utils/graphs.py)."""
        self.reap_graphs()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._step_eager()
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._step_eager()
        self.graph = g
        self.graph_unrolled, self.unroll = None, max(1, int(unroll))
        if self.unroll > 1:
            gk = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gk):
                for _ in range(self.unroll):
                    self._step_eager()
            self.graph_unrolled = gk

    # ---- eval / state ----
    def w1_out_of_range(self) -> bool:
        """True when a W1 weight no longer fits the fp16 shadow layer 1 runs on (|w| >= 65488):
        the SGD kernel saturates that shadow entry and flags its row sum (mlp_fused.hip h_fix)."""
        return int(self.r1p.max()) >= R1_OVF_MIN

    def stats(self) -> StepStats:
        loss = float(self.loss.sum())
        acc = float(self.correct.sum())
        if self.w1_out_of_range():
            loss = float("nan")  # visible: never a number from a saturated layer 1
        return StepStats(loss / self.batch, acc / self.batch, self.batch)

    def evaluate(self, x_u8: torch.Tensor, y_u8: torch.Tensor) -> StepStats:
        n = self._n
        x = x_u8.reshape(-1, D_IN).to(self.device).contiguous()
        y = y_u8.reshape(-1).to(self.device).to(torch.uint8).contiguous()
        rows = x.shape[0] // BLOCK_ROWS * BLOCK_ROWS
        loss = torch.zeros(rows, device=self.device)
        corr = torch.zeros(rows, device=self.device)
        n.call("sl_mlp_rows", n.ptr(x), n.ptr(y), None, 1, rows,
               n.ptr(self.w1h), n.ptr(self.w2h), n.ptr(self.w3h), n.ptr(self.w2th), n.ptr(self.w3th),
               n.ptr(self.params), self.xa, self.xb, 1.0, 1.0, None, None, None, None,
               n.ptr(loss), n.ptr(corr), None, 0, n.ptr(self.r1p), None, n.stream_ptr())
        lv = float("nan") if self.w1_out_of_range() else float(loss.mean())
        return StepStats(lv, float(corr.mean()), rows)

    def logits(self, x_u8: torch.Tensor) -> torch.Tensor:
        n = self._n
        x = x_u8.reshape(-1, D_IN).to(self.device).contiguous()
        rows = x.shape[0]
        if rows % BLOCK_ROWS:
            raise ValueError(f"rows must be a multiple of {BLOCK_ROWS}")
        out = torch.empty(rows, CLASSES, device=self.device)
        n.call("sl_mlp_rows", n.ptr(x), None, None, 1, rows,
               n.ptr(self.w1h), n.ptr(self.w2h), n.ptr(self.w3h), n.ptr(self.w2th), n.ptr(self.w3th),
               n.ptr(self.params), self.xa, self.xb, 1.0, 1.0, None, None, None, None,
               None, None, n.ptr(out), 0, n.ptr(self.r1p), None, n.stream_ptr())
        if self.w1_out_of_range():
            out.fill_(float("nan"))
        return out

    def get_flat(self) -> torch.Tensor:
        return self.params[:N_PARAMS].clone()

    def set_flat(self, flat: torch.Tensor) -> None:
        self.params[:N_PARAMS].copy_(flat.to(self.params))
        self.refresh_shadows()

    # ---- exact-resume state beyond the flat vectors (ckpt format v2) ----
    def state_extra(self) -> dict:
        """The device batch cursor: a resumed run continues with the batch the saved run
        would have taken next, so save-at-k + resume + m steps equals k + m steps."""
        return {"cursor": self.cursor.double().cpu().numpy()}

    def load_state_extra(self, d: dict) -> None:
        if "cursor" in d:
            self.cursor.fill_(int(d["cursor"][0]))

    def buffers(self) -> list:
        return []
