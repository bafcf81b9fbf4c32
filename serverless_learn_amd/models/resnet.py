"""ResNet-18-shaped CNN (BASELINE config 4): spec, flat parameter layout,
fp32 torch reference and the CPU trainer.

The reference has no model (its "training" is ``model[i] += 1`` every 2 s,
/root/reference/src/worker.cc:221-231, on a ``std::vector<double>`` that the
``Update{repeated double delta}`` message carries, proto :81-83).  Like the
MLP, the CNN's parameters live in ONE flat fp32 vector, so the same wire
message, checkpoint format and single-bucket collectives apply unchanged.

Layout choices are made for the MI355X kernels (csrc/kernels/conv.hip):

* activations are NHWC; conv weights are stored ``[Cout][KH][KW][Cin]`` so
  the implicit-GEMM reduction index (kh, kw, ci) is contiguous;
* the 3-channel input is padded to 8 channels (16-byte gathers), so the stem
  weight is stored with Cin = 8; the 5 padding channels see zero input, get
  zero gradient and stay zero;
* every tensor starts at a 64-element boundary of the flat vector.

Two stems: ``cifar`` (3x3 s1 conv, 32x32 input, the usual CIFAR ResNet-18,
11.17 M parameters) and ``imagenet`` (7x7 s2 conv + 3x3 s2 max-pool).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

ALIGN = 64
CIFAR_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR_STD = (0.2470, 0.2435, 0.2616)
STAGES = ((64, 1), (128, 2), (256, 2), (512, 2))


@dataclass
class ConvSpec:
    name: str
    cin: int        # stored input channels (stem: 8)
    cin_real: int   # logical input channels (stem: 3)
    cout: int
    k: int
    stride: int
    pad: int
    off: int = 0

    @property
    def numel(self) -> int:
        return self.cout * self.k * self.k * self.cin

    @property
    def kdim(self) -> int:
        return self.k * self.k * self.cin


@dataclass
class BNSpec:
    name: str
    c: int
    g_off: int = 0
    b_off: int = 0


@dataclass
class BlockSpec:
    conv1: ConvSpec
    bn1: BNSpec
    conv2: ConvSpec
    bn2: BNSpec
    down: ConvSpec | None = None
    dbn: BNSpec | None = None


@dataclass
class ResNetSpec:
    stem: str
    in_hw: int
    classes: int
    stem_conv: ConvSpec
    stem_bn: BNSpec
    blocks: list = field(default_factory=list)
    fc_in: int = 512
    fc_w: int = 0
    fc_b: int = 0
    n_flat: int = 0
    n_logical: int = 0

    def convs(self):
        yield self.stem_conv
        for b in self.blocks:
            yield b.conv1
            yield b.conv2
            if b.down is not None:
                yield b.down

    def bns(self):
        yield self.stem_bn
        for b in self.blocks:
            yield b.bn1
            yield b.bn2
            if b.dbn is not None:
                yield b.dbn


def resnet18_spec(stem: str = "cifar", classes: int = 10, in_hw: int | None = None) -> ResNetSpec:
    if stem not in ("cifar", "imagenet"):
        raise ValueError(stem)
    in_hw = in_hw or (32 if stem == "cifar" else 224)
    off = 0
    n_logical = 0

    def take(n: int) -> int:
        nonlocal off
        o = off
        off += (n + ALIGN - 1) // ALIGN * ALIGN
        return o

    def conv(name, cin, cout, k, s, p, cin_real=None):
        nonlocal n_logical
        c = ConvSpec(name, cin, cin_real or cin, cout, k, s, p)
        c.off = take(c.numel)
        n_logical += c.cout * c.k * c.k * c.cin_real
        return c

    def bn(name, c):
        nonlocal n_logical
        b = BNSpec(name, c)
        b.g_off = take(c)
        b.b_off = take(c)
        n_logical += 2 * c
        return b

    if stem == "cifar":
        sc = conv("stem", 8, 64, 3, 1, 1, cin_real=3)
    else:
        sc = conv("stem", 8, 64, 7, 2, 3, cin_real=3)
    sb = bn("stem_bn", 64)
    spec = ResNetSpec(stem, in_hw, classes, sc, sb)
    cin = 64
    for si, (w, s) in enumerate(STAGES):
        for bi in range(2):
            stride = s if bi == 0 else 1
            pre = f"layer{si + 1}.{bi}"
            c1 = conv(pre + ".conv1", cin, w, 3, stride, 1)
            b1 = bn(pre + ".bn1", w)
            c2 = conv(pre + ".conv2", w, w, 3, 1, 1)
            b2 = bn(pre + ".bn2", w)
            blk = BlockSpec(c1, b1, c2, b2)
            if stride != 1 or cin != w:
                blk.down = conv(pre + ".down", cin, w, 1, stride, 0)
                blk.dbn = bn(pre + ".down_bn", w)
            spec.blocks.append(blk)
            cin = w
    spec.fc_w = take(classes * 512)
    spec.fc_b = take(classes)
    n_logical += classes * 512 + classes
    spec.n_flat = off
    spec.n_logical = n_logical
    return spec


def spec_layout(spec: ResNetSpec) -> list:
    """[name, shape, offset] of every tensor in the flat vector (checkpoint metadata)."""
    out = []
    for c in spec.convs():
        out.append([c.name + ".weight", [c.cout, c.k, c.k, c.cin], c.off])
    for b in spec.bns():
        out.append([b.name + ".weight", [b.c], b.g_off])
        out.append([b.name + ".bias", [b.c], b.b_off])
    out.append(["fc.weight", [spec.classes, 512], spec.fc_w])
    out.append(["fc.bias", [spec.classes], spec.fc_b])
    return sorted(out, key=lambda e: e[2])


def init_params(spec: ResNetSpec, seed: int = 0) -> torch.Tensor:
    """Kaiming-normal (fan_out, relu) convs, BN gamma=1/beta=0, nn.Linear-style FC."""
    g = torch.Generator().manual_seed(seed)
    flat = torch.zeros(spec.n_flat, dtype=torch.float32)
    for c in spec.convs():
        std = math.sqrt(2.0 / (c.cout * c.k * c.k))
        w = torch.randn(c.cout, c.k, c.k, c.cin, generator=g) * std
        w[..., c.cin_real:] = 0
        flat[c.off:c.off + c.numel] = w.reshape(-1)
    for b in spec.bns():
        flat[b.g_off:b.g_off + b.c] = 1.0
    bound = 1.0 / math.sqrt(512)
    flat[spec.fc_w:spec.fc_w + spec.classes * 512] = (torch.rand(spec.classes * 512, generator=g) * 2 - 1) * bound
    flat[spec.fc_b:spec.fc_b + spec.classes] = (torch.rand(spec.classes, generator=g) * 2 - 1) * bound
    return flat


def running_stats(spec: ResNetSpec, device="cpu") -> dict:
    return {b.name: (torch.zeros(b.c, device=device), torch.ones(b.c, device=device)) for b in spec.bns()}


def conv_weight_nchw(flat: torch.Tensor, c: ConvSpec) -> torch.Tensor:
    w = flat[c.off:c.off + c.numel].view(c.cout, c.k, c.k, c.cin)
    return w[..., :c.cin_real].permute(0, 3, 1, 2)


def normalize_input(x_u8: torch.Tensor) -> torch.Tensor:
    """[N,H,W,3] u8 -> [N,3,H,W] fp32 normalised."""
    x = x_u8.float().div(255.0)
    mean = torch.tensor(CIFAR_MEAN, device=x.device)
    std = torch.tensor(CIFAR_STD, device=x.device)
    return ((x - mean) / std).permute(0, 3, 1, 2)


def ref_forward(spec: ResNetSpec, flat: torch.Tensor, x_u8: torch.Tensor, training: bool = True,
                running: dict | None = None, momentum: float = 0.1, eps: float = 1e-5) -> torch.Tensor:
    """fp32 NCHW torch forward of exactly the network the HIP engine runs."""
    def bn(x, b: BNSpec):
        rm, rv = running[b.name] if running is not None else (None, None)
        return F.batch_norm(x, rm, rv, flat[b.g_off:b.g_off + b.c], flat[b.b_off:b.b_off + b.c],
                            training=training or rm is None, momentum=momentum, eps=eps)

    def conv(x, c: ConvSpec):
        return F.conv2d(x, conv_weight_nchw(flat, c), stride=c.stride, padding=c.pad)

    x = normalize_input(x_u8)
    x = F.relu(bn(conv(x, spec.stem_conv), spec.stem_bn))
    if spec.stem == "imagenet":
        x = F.max_pool2d(x, 3, 2, 1)
    for blk in spec.blocks:
        o = F.relu(bn(conv(x, blk.conv1), blk.bn1))
        o = bn(conv(o, blk.conv2), blk.bn2)
        sc = bn(conv(x, blk.down), blk.dbn) if blk.down is not None else x
        x = F.relu(o + sc)
    x = x.mean(dim=(2, 3))
    w = flat[spec.fc_w:spec.fc_w + spec.classes * 512].view(spec.classes, 512)
    return F.linear(x, w, flat[spec.fc_b:spec.fc_b + spec.classes])


def ref_grads(spec: ResNetSpec, flat: torch.Tensor, x_u8: torch.Tensor, y: torch.Tensor, grad_scale: float,
              running: dict | None = None):
    """(loss_sum, correct, grad_flat) with d(loss_i)/dlogits scaled by grad_scale."""
    w = flat.detach().clone().float().requires_grad_(True)
    logits = ref_forward(spec, w, x_u8, True, running)
    losses = F.cross_entropy(logits, y.long(), reduction="none")
    (losses.sum() * grad_scale).backward()
    correct = (logits.argmax(1) == y.long()).float().sum()
    return losses.detach().sum(), correct.detach(), w.grad.detach()


class CPUResNetTrainer:
    """Plain-torch trainer with FusedResNetTrainer's interface (CPU workers, tests)."""

    def __init__(self, batch: int, lr: float = 0.05, momentum: float = 0.9, weight_decay: float = 5e-4,
                 seed: int = 0, world_size: int = 1, stem: str = "cifar", flat: torch.Tensor | None = None,
                 in_hw: int | None = None):
        from .mlp import StepStats, sgd_update  # noqa: F401

        self.spec = resnet18_spec(stem, 10, in_hw)
        self.batch = batch
        self.lr, self.momentum, self.weight_decay = lr, momentum, weight_decay
        self.world_size = world_size
        self.params = (flat if flat is not None else init_params(self.spec, seed)).clone().float()
        self.mom = torch.zeros_like(self.params) if momentum > 0 else None
        self.running = running_stats(self.spec)
        self.x = self.y = None
        self.cursor = 0
        self.allreduce = None
        self._last = None
        from ..utils.phases import PhaseProbe

        self.phases = PhaseProbe("cpu")

    @property
    def n_params(self) -> int:
        return self.spec.n_flat

    @property
    def model_name(self) -> str:
        return f"resnet18-{self.spec.stem}"

    def layout(self):
        return spec_layout(self.spec)

    def set_world(self, world: int) -> None:
        self.world_size = world

    def refresh_shadows(self) -> None:
        pass

    def load_shard(self, x_u8: torch.Tensor, y_u8: torch.Tensor) -> None:
        hw = self.spec.in_hw
        self.x = x_u8.reshape(-1, hw, hw, 3)
        self.y = y_u8.reshape(-1)
        self.n_batches = self.x.shape[0] // self.batch

    def step(self) -> None:
        from .mlp import sgd_update

        b = self.cursor % self.n_batches
        xs = self.x[b * self.batch:(b + 1) * self.batch]
        ys = self.y[b * self.batch:(b + 1) * self.batch]
        loss, correct, g = ref_grads(self.spec, self.params, xs, ys, 1.0 / (self.batch * self.world_size),
                                     self.running)
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

    def stats(self):
        from .mlp import StepStats

        loss, correct = self._last
        return StepStats(loss / self.batch, correct / self.batch, self.batch)

    def get_flat(self) -> torch.Tensor:
        return self.params.clone()

    def set_flat(self, flat: torch.Tensor) -> None:
        self.params.copy_(flat.to(self.params))

    # ---- exact-resume state beyond the flat vectors (ckpt format v2) ----
    def state_extra(self) -> dict:
        d = {"cursor": np.array([self.cursor], dtype=np.float64)}
        for name, (rm, rv) in self.running.items():
            d[f"bn/{name}/mean"] = rm.double().numpy()
            d[f"bn/{name}/var"] = rv.double().numpy()
        return d

    def load_state_extra(self, d: dict) -> None:
        if "cursor" in d:
            self.cursor = int(d["cursor"][0])
        for name, (rm, rv) in self.running.items():
            if f"bn/{name}/mean" in d:
                rm.copy_(torch.from_numpy(np.asarray(d[f"bn/{name}/mean"])).to(rm.dtype))
                rv.copy_(torch.from_numpy(np.asarray(d[f"bn/{name}/var"])).to(rv.dtype))

    def buffers(self) -> list:
        """Non-parameter state every replica must agree on (broadcast after a regroup)."""
        return [t for pair in self.running.values() for t in pair]

    def evaluate(self, x_u8: torch.Tensor, y_u8: torch.Tensor):
        """Inference with the BatchNorm running statistics (eval mode)."""
        from .mlp import StepStats

        with torch.no_grad():
            logits = ref_forward(self.spec, self.params, x_u8.reshape(-1, self.spec.in_hw, self.spec.in_hw, 3),
                                 False, self.running)
            y = y_u8.reshape(-1).long()
            loss = F.cross_entropy(logits, y, reduction="mean")
            acc = (logits.argmax(1) == y).float().mean()
        return StepStats(float(loss), float(acc), int(y.numel()))


def block_backward_errors(tr, g: torch.Tensor) -> list:
    """Per residual block of a FusedResNetTrainer that just ran ``compute_grads`` (returned
    ``g``): the block's backward (BN x2-3, conv data / weight gradients, ReLU masks, skip)
    against fp32 autograd of that block run on the engine's OWN stored input, bf16 weights and
    incoming gradient.  Returns [(conv name, "dx" | "dW", relative L2 error)].  Used by the GPU
    numerics tests at B = 32 (tests/test_cnn_gpu.py) and at the bench batch
    (scripts/resnet_block_check.py)."""
    spec = tr.spec
    w32 = tr.shadow.float()
    f32 = lambda t: t.float().permute(0, 3, 1, 2).detach()  # noqa: E731
    nhwc = lambda t: t.permute(0, 2, 3, 1)  # noqa: E731

    def rel(a, b):
        a, b = a.detach().float(), b.detach().float()
        return float((a - b).norm() / (b.norm() + 1e-12))

    def bn(xx, b):
        return F.batch_norm(xx, None, None, tr.params[b.g_off:b.g_off + b.c], tr.params[b.b_off:b.b_off + b.c],
                            training=True)

    if tr.stem_onload:  # block 0's input a0 is rebuilt on load from c0, never stored: materialise it
        tr.K.bn_apply(tr.c0, tr.bn[spec.stem_bn.name].coef, tr.a0, relu=True)
        torch.cuda.synchronize()
    nb = len(tr.blocks)
    if tr.fuse_bn_bwd:
        # the data gradient of block i+1 lands in block i's dz, already ReLU-masked by block
        # i's output (the block input of i+1); block 0's in its own dx, masked by the stem's ReLU
        dys = [tr.blocks[i]["dz"] for i in range(nb - 1)] + [tr.dfeat_in]
        dxs = [tr.blocks[0]["dx"]] + [tr.blocks[i - 1]["dz"] for i in range(1, nb)]
    else:
        dys = [tr.blocks[i + 1]["dx"] for i in range(nb - 1)] + [tr.dfeat_in]
        dxs = [st["dx"] for st in tr.blocks]
    errs = []
    for st, blk, dy, dx in zip(tr.blocks, spec.blocks, dys, dxs):
        ws = {c.name: conv_weight_nchw(w32, c).clone().requires_grad_(True)
              for c in (blk.conv1, blk.conv2, blk.down) if c is not None}
        xin = f32(st["x"]).requires_grad_(True)
        conv = lambda t, c: F.conv2d(t, ws[c.name], stride=c.stride, padding=c.pad)  # noqa: E731
        o = F.relu(bn(conv(xin, blk.conv1), blk.bn1))
        o = bn(conv(o, blk.conv2), blk.bn2)
        sc = bn(conv(xin, blk.down), blk.dbn) if blk.down is not None else xin
        out = F.relu(o + sc)
        out.backward(f32(dy))
        # compared where the block input is positive: the fused path stores the input
        # gradient masked by the ReLU that produced the input
        keep = (st["x"] > 0).float()
        errs.append((blk.conv1.name, "dx", rel(dx.float() * keep, nhwc(xin.grad) * keep)))
        for c in (blk.conv1, blk.conv2, blk.down):
            if c is None:
                continue
            mine = g[c.off:c.off + c.numel].view(c.cout, c.k, c.k, c.cin).permute(0, 3, 1, 2)
            errs.append((c.name, "dW", rel(mine, ws[c.name].grad)))
        del ws, xin, o, sc, out, keep
    return errs
