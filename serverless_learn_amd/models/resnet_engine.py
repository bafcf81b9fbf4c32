"""MI355X training engine for the ResNet-18-shaped CNN (BASELINE config 4).

A static execution plan, not an autograd graph: every activation, gradient
and statistics buffer is allocated once for the fixed per-GPU batch, and a
step is a fixed sequence of hand-written HIP kernels (csrc/kernels/conv.hip,
cnn_aux.hip, elementwise.hip) -- so it can be captured whole in a hipGraph
and replayed with zero host work (the data batch is chosen by a device-side
cursor, like the MLP engine).

Per step:
  forward   input_norm -> [conv (+BN stats in the epilogue) -> bn_apply with
            the finalize folded in (+residual, ReLU)] x 20 -> avgpool -> fc ->
            softmax-CE (loss, dlogits, dbias); a 64-channel block's conv2 applies
            relu(bn1(.)) while loading c1 instead (BN-on-load, no a1 pass)
  backward  per block, in reverse: bn_bwd_apply (ReLU mask fused), conv wgrad
            (split-K partials in a slab + one ordered reduce into the flat
            gradient) and dgrad, whose epilogue adds the residual gradient,
            applies the next BN's ReLU mask and accumulates that BN's backward
            sums (csrc/kernels/bn_bwd_epi.h), so only the first BN after the
            average pool still needs a bn_bwd_reduce pass (SL_BNB_FUSE=0: one
            per BN, as before)
            (SL_WGRAD_SIDE=1: the split-K slab reduces run on a side stream, forked
            per reduce and joined before the optimizer and each gradient bucket)
  comms     optional: the flat gradient is laid out in forward order, so
            when a block's backward is done its whole parameter range is final
            -> a bucket hook can launch RCCL all-reduce of that range while
            backward continues
  update    one multi-tensor SGD launch over the flat vector (fp32 master,
            momentum, weight decay, bf16 shadow) + one launch that re-lays the
            bf16 conv weights out for dgrad.
"""
from __future__ import annotations

import os
import torch

from ..utils.graphs import GraphSlots
from .mlp import StepStats
from .resnet import CIFAR_MEAN, CIFAR_STD, BlockSpec, BNSpec, ConvSpec, init_params, resnet18_spec

LOGIT_LD = 16  # dlogits row stride (classes padded for 16-B gathers)


class _BN:
    """Per-BatchNorm buffers.  ``stats_buf``/``sums_buf`` are cross-workgroup sum
    buffers (replicas | result | ticket, csrc/kernels/common.h rsum_*) living in
    the per-step zeroed arena; ``stats``/``sums`` are their folded results."""

    def __init__(self, spec: BNSpec, params, grad, arena, off, dev, rs):
        from ..ops import cnn as K

        c = spec.c
        self.spec = spec
        self.gamma = params[spec.g_off:spec.g_off + c]
        self.beta = params[spec.b_off:spec.b_off + c]
        self.ggamma = grad[spec.g_off:spec.g_off + c]
        self.gbeta = grad[spec.b_off:spec.b_off + c]
        self.stats_buf = arena[off:off + rs]
        self.sums_buf = arena[off + rs:off + 2 * rs]
        self.stats = K.rsum_result(self.stats_buf, 2 * c)
        self.sums = K.rsum_result(self.sums_buf, 2 * c)
        self.coef = torch.zeros(4 * c, device=dev)
        self.dcoef = torch.zeros(3 * c, device=dev)
        self.run_mean = torch.zeros(c, device=dev)
        self.run_var = torch.ones(c, device=dev)


class _Conv:
    def __init__(self, spec: ConvSpec, params, shadow, grad, dev, ld_out=None):
        self.spec = spec
        self.w = shadow[spec.off:spec.off + spec.numel]
        self.g = grad[spec.off:spec.off + spec.numel]
        self.ldt = ld_out or spec.cout  # dgrad source channels
        self.wt = torch.zeros(spec.cin * spec.k * spec.k * self.ldt, dtype=torch.bfloat16, device=dev)


class FusedResNetTrainer(GraphSlots):
    def __init__(self, batch: int, device="cuda", lr: float = 0.05, momentum: float = 0.9,
                 weight_decay: float = 5e-4, seed: int = 0, world_size: int = 1, stem: str = "cifar",
                 classes: int = 10, flat: torch.Tensor | None = None, bn_momentum: float = 0.1,
                 in_hw: int | None = None):
        from ..ops import _native
        from ..ops import cnn as K
        from ..ops import optim as O

        _native.lib()
        self.K, self.O = K, O
        self.spec = spec = resnet18_spec(stem, classes, in_hw)
        dev = self.device = torch.device(device)
        self.batch = B = batch
        self.lr, self.momentum, self.weight_decay = lr, momentum, weight_decay
        self.world_size = world_size
        self.grad_scale = 1.0 / (batch * world_size)
        self.bn_momentum = bn_momentum
        self.shortcut_even_on = os.environ.get("SL_SHORTCUT_EVEN", "1") != "0"
        # BN-on-load: where the direct 3x3 kernel serves a block's conv2 (64 channels, 32 wide), it
        # reads relu(bn1(c1)) straight from c1 -- forward and weight gradient -- and a1 is never
        # written (SL_BN_ONLOAD=0: bn_apply_stats + a1, as before)
        self.bn_onload = os.environ.get("SL_BN_ONLOAD", "1") != "0"
        n = spec.n_flat
        self.params = torch.zeros(n, dtype=torch.float32, device=dev)
        self.params.copy_((flat if flat is not None else init_params(spec, seed)).to(dev))
        self.mom = torch.zeros_like(self.params) if momentum > 0 else None
        self.grad = torch.zeros_like(self.params)
        self.shadow = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        bns = list(spec.bns())
        rsz = {b.name: (K.rsum_floats(2 * b.c) + 3) // 4 * 4 for b in bns}  # 16-B aligned regions
        self.arena = torch.zeros(sum(2 * rsz[b.name] for b in bns), device=dev)
        off = 0
        self.bn = {}
        for b in bns:
            self.bn[b.name] = _BN(b, self.params, self.grad, self.arena, off, dev, rsz[b.name])
            off += 2 * rsz[b.name]
        self.conv = {c.name: _Conv(c, self.params, self.shadow, self.grad, dev) for c in spec.convs()}
        self.fc_w = self.shadow[spec.fc_w:spec.fc_w + classes * 512]
        self.fc_b = self.params[spec.fc_b:spec.fc_b + classes]
        self.fc_gw = self.grad[spec.fc_w:spec.fc_w + classes * 512]
        self.fc_gb = self.grad[spec.fc_b:spec.fc_b + classes]
        self.fc_wt = torch.zeros(512 * LOGIT_LD, dtype=torch.bfloat16, device=dev)

        bf = dict(dtype=torch.bfloat16, device=dev)
        hw = spec.in_hw
        self.x0 = torch.empty(B, hw, hw, 8, **bf)
        self.labels = torch.zeros(B, dtype=torch.uint8, device=dev)
        # ---- stem buffers ----
        sc = spec.stem_conv
        s_hw = K.out_size(hw, sc.k, sc.stride, sc.pad)
        self.c0 = torch.empty(B, s_hw, s_hw, 64, **bf)
        self.a0 = torch.empty_like(self.c0)
        self.dc0 = torch.empty_like(self.c0)
        self.da0 = torch.empty_like(self.c0)
        cur = self.a0
        if spec.stem == "imagenet":
            p_hw = K.out_size(s_hw, 3, 2, 1)
            self.p0 = torch.empty(B, p_hw, p_hw, 64, **bf)
            self.p0_arg = torch.empty(B, p_hw, p_hw, 64, dtype=torch.uint8, device=dev)
            self.dp0 = torch.empty_like(self.p0)
            cur = self.p0
        # ---- residual blocks ----
        self.blocks = []
        for blk in spec.blocks:
            st = {"spec": blk, "x": cur}
            h = cur.shape[1]
            oh = K.out_size(h, 3, blk.conv1.stride, 1)
            shp = (B, oh, oh, blk.conv1.cout)
            for name in ("c1", "a1", "c2", "y", "dz", "dc2", "da1", "dc1"):
                st[name] = torch.empty(shp, **bf)
            # 1-bit ReLU mask of y (bit j of byte q = y[8q+j] > 0) for the backward
            st["ym"] = torch.empty(B * oh * oh * blk.conv1.cout // 8, dtype=torch.uint8, device=dev)
            if blk.down is not None:
                st["cs"] = torch.empty(shp, **bf)
                st["dcs"] = torch.empty(shp, **bf)
                if not self._shortcut_even(blk):  # else the shortcut gradient goes straight into dx
                    st["dxs"] = torch.empty_like(cur)
            st["dx"] = torch.empty_like(cur)
            c2s = blk.conv2
            st["bnin"] = self.bn_onload and K.conv3x3_bnin_applicable(shp, c2s.cout, c2s.k, c2s.stride, c2s.pad)
            self.blocks.append(st)
            cur = st["y"]
        self.feat_in = cur
        # stem BN-on-load: with an identity first block, a0 = relu(bn0(c0)) feeds only block 0's
        # conv1 (forward, weight gradient) and its residual; both rebuild it from c0
        b0 = self.blocks[0]
        c1s = b0["spec"].conv1
        self.stem_onload = (self.bn_onload and spec.stem != "imagenet" and b0["spec"].down is None
                            and K.conv3x3_bnin_applicable(self.c0.shape, c1s.cout, c1s.k, c1s.stride, c1s.pad))
        self.feat = torch.empty(B, 1, 1, 512, **bf)
        self.dfeat = torch.empty_like(self.feat)
        self.dfeat_in = torch.empty_like(cur)
        self.logits = torch.empty(B, classes, device=dev)
        self.dlogits = torch.zeros(B, 1, 1, LOGIT_LD, **bf)
        self.loss = torch.zeros(B, device=dev)
        self.correct = torch.zeros(B, device=dev)
        self.cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        self.x = self.y = None
        self.graph = None
        self.bucket_hook = None   # callable(flat_view) -> handle, launched during backward
        self.bucket_wait = None   # callable(handles) -> None, before the optimizer
        from ..utils.phases import PhaseProbe

        self.phases = PhaseProbe(self.device)
        self.allreduce = None     # callable(grad) -> None (simple, non-overlapped)
        self.bucket_bytes = 16 << 20
        # SL_WGRAD_SIDE=1: the slab reduces run on a side stream beside the next data gradient.  Off by
        # default: starved by the one-workgroup-per-CU conv kernels, the reduces stretched from 13 to
        # 36 us and the step got 3.6 % slower (profiles/r03_side)
        self.wgrad_side = torch.cuda.Stream(dev) if os.environ.get("SL_WGRAD_SIDE", "0") == "1" else None
        # split-K slab(s) of the weight gradients, grown on the first step
        self.wgws = K.WgradWorkspace(dev, alternate=self.wgrad_side is not None)
        # BN-backward sums in the data-gradient epilogues instead of bn_bwd_reduce passes
        self.fuse_bn_bwd = os.environ.get("SL_BNB_FUSE", "1") != "0"

        items = [(c.w, c.wt, c.spec.cout, c.spec.k * c.spec.k, c.spec.cin, c.ldt)
                 for c in self.conv.values() if c.spec.name != "stem"]
        items.append((self.fc_w, self.fc_wt, classes, 1, 512, LOGIT_LD))
        self.wt = K.WeightTransposer(items, dev)
        self.refresh_shadows()
        self.stats()  # load torch's reduction kernel now, not inside the first logged chunk (as mlp.py)

    def _shortcut_even(self, blk) -> bool:
        """A 1x1 / stride-2 shortcut beside a 3x3 / stride-2 conv1 (every ResNet-18 downsample
        block): its data gradient is written straight into the (even, even) positions of the block's
        input gradient, and conv1's parity-class data gradient adds there (ops.cnn.conv_dgrad_s2_even).
        SL_SHORTCUT_EVEN=0 keeps the full-resolution shortcut gradient + add (A/B, tests)."""
        d, c1 = blk.down, blk.conv1
        return (self.shortcut_even_on and d is not None and d.k == 1 and d.stride == 2 and d.pad == 0
                and c1.k == 3 and c1.stride == 2 and c1.pad == 1 and d.cout % 64 == 0 and c1.cout % 64 == 0)

    @property
    def n_params(self) -> int:
        return self.spec.n_flat

    @property
    def model_name(self) -> str:
        return f"resnet18-{self.spec.stem}"

    def layout(self):
        from .resnet import spec_layout

        return spec_layout(self.spec)

    def set_world(self, world: int) -> None:
        self.world_size = world
        self.grad_scale = 1.0 / (self.batch * world)
        self.graph = None

    # ------------------------------------------------------------------
    def refresh_shadows(self) -> None:
        self.O.to_bf16(self.params, self.shadow)
        self.wt()

    def load_shard(self, x_u8: torch.Tensor, y_u8: torch.Tensor) -> None:
        hw = self.spec.in_hw
        x = x_u8.reshape(-1, hw, hw, 3)
        if x.shape[0] < self.batch:
            raise ValueError("shard smaller than one batch")
        self.x = x.to(self.device, non_blocking=True).contiguous()
        self.y = y_u8.reshape(-1).to(self.device, non_blocking=True).to(torch.uint8).contiguous()
        self.graph = None

    # ------------------------------------------------------------------
    def _conv_bn(self, x, conv: _Conv, bn: _BN, out):
        K = self.K
        c = conv.spec
        K.conv_fwd(x, conv.w, c.cout, c.k, c.stride, c.pad, y=out, stats=bn.stats_buf)

    def forward(self, train: bool = True):
        with self.K.rsum_deferred():  # BN-sum folds in the consuming kernels (ops/cnn.py)
            return self._forward(train)

    def _forward(self, train: bool = True):
        K, spec = self.K, self.spec
        self.arena.zero_()
        K.input_norm(self.x, self.y, self.cursor, self.batch, self.x0, self.labels, CIFAR_MEAN, CIFAR_STD)
        sbn = self.bn[spec.stem_bn.name]
        self._conv_bn(self.x0, self.conv["stem"], sbn, self.c0)
        cnt0 = self.c0.numel() // 64
        if not self.stem_onload:
            K.bn_apply_stats(self.c0, sbn, self.a0, cnt0, momentum=self.bn_momentum)
        if spec.stem == "imagenet":
            K.maxpool_fwd(self.a0, self.p0, self.p0_arg)
        for i, st in enumerate(self.blocks):
            blk: BlockSpec = st["spec"]
            b1, b2 = self.bn[blk.bn1.name], self.bn[blk.bn2.name]
            stem_in = i == 0 and self.stem_onload
            if stem_in:
                K.conv3x3_bnin_fwd(self.c0, self.conv[blk.conv1.name].w, sbn, cnt0, st["c1"], stats=b1.stats_buf,
                                   momentum=self.bn_momentum)
            else:
                self._conv_bn(st["x"], self.conv[blk.conv1.name], b1, st["c1"])
            cnt = st["c1"].numel() // blk.conv1.cout
            if st["bnin"]:
                K.conv3x3_bnin_fwd(st["c1"], self.conv[blk.conv2.name].w, b1, cnt, st["c2"], stats=b2.stats_buf,
                                   momentum=self.bn_momentum)
            else:
                K.bn_apply_stats(st["c1"], b1, st["a1"], cnt, momentum=self.bn_momentum)
                self._conv_bn(st["a1"], self.conv[blk.conv2.name], b2, st["c2"])
            if blk.down is not None:
                bd = self.bn[blk.dbn.name]
                self._conv_bn(st["x"], self.conv[blk.down.name], bd, st["cs"])
                K.bn_apply_stats(st["c2"], b2, st["y"], cnt, res=st["cs"], rbn=bd, momentum=self.bn_momentum,
                                 mask_out=st["ym"])
            elif stem_in:
                K.bn_apply_stats(st["c2"], b2, st["y"], cnt, res=self.c0, rbn=sbn, res_relu=True,
                                 momentum=self.bn_momentum, mask_out=st["ym"])
            else:
                K.bn_apply_stats(st["c2"], b2, st["y"], cnt, res=st["x"], momentum=self.bn_momentum,
                                 mask_out=st["ym"])
        K.avgpool_fwd(self.feat_in, self.feat)
        K.conv_fwd(self.feat, self.fc_w, spec.classes, 1, 1, 0, yf=self.logits, bias=self.fc_b)
        K.softmax_ce(self.logits, self.labels, self.loss, self.correct, self.dlogits.view(self.batch, LOGIT_LD),
                     self.fc_gb if train else None, self.grad_scale)

    def backward(self):
        with self.K.rsum_deferred():
            return self._backward()

    def _backward(self):
        K, spec = self.K, self.spec
        handles = []
        pending_from = spec.n_flat  # grad[pending_from:] is final and not yet reduced
        bucket_elems = self.bucket_bytes // 4

        side = self.wgrad_side
        if side is not None:
            K.wgrad_side_begin(side)

        def maybe_bucket(lo, force=False):
            nonlocal pending_from
            if self.bucket_hook is None:
                return
            if force or (pending_from - lo) >= bucket_elems:
                if side is not None:
                    K.wgrad_side_join(end=False)  # the bucket's reduces are in the gradient
                handles.append(self.bucket_hook(self.grad[lo:pending_from]))
                pending_from = lo

        K.conv_wgrad(self.feat, self.dlogits, spec.classes, 1, 1, 0, self.fc_gw, ws=self.wgws)
        K.conv_dgrad(self.dlogits, self.fc_wt, 512, 1, 1, 0, self.dfeat)
        K.avgpool_bwd(self.dfeat.view(self.batch, 512), self.dfeat_in)
        dy = self.dfeat_in
        fuse = self.fuse_bn_bwd
        sbn = self.bn[spec.stem_bn.name]
        rblocks = list(reversed(self.blocks))

        def block_out_bn(st):
            # BN backward of a block output y = relu(bn2(c2) + sc): the mask is the forward's
            # 1-bit image of y; a downsample shortcut's BN (input cs) is fed by the same dz
            blk = st["spec"]
            b2 = self.bn[blk.bn2.name]
            d = dict(x=st["c2"], sums=b2.sums_buf, y_mask=st["ym"])
            if blk.down is not None:
                d.update(x2=st["cs"], sums2=self.bn[blk.dbn.name].sums_buf)
            return d

        for i, st in enumerate(rblocks):
            blk: BlockSpec = st["spec"]
            c1, c2 = self.conv[blk.conv1.name], self.conv[blk.conv2.name]
            b1, b2 = self.bn[blk.bn1.name], self.bn[blk.bn2.name]
            # y = relu(bn2(c2) + sc): dz = dy * 1[y > 0] feeds bn2 and the shortcut.  Fused: the
            # previous conv1 data gradient (next block's) already stored dz and the sums.
            down = blk.down is not None
            bd = self.bn[blk.dbn.name] if down else None
            if not (fuse and i > 0):
                bo = block_out_bn(st)
                K.bn_bwd_reduce(dy, None, bo["x"], bo["sums"], dz_out=st["dz"], y_mask=bo["y_mask"],
                                x2=bo.get("x2"), sums2=bo.get("sums2"))
            # the input gradient is the previous block's output gradient (its dz, stored masked
            # with that block's BN sums) or, for the first block, the stem BN's
            nxt = None
            if fuse and i + 1 < len(rblocks):
                nxt = block_out_bn(rblocks[i + 1])
                dx = rblocks[i + 1]["dz"]
            elif fuse and spec.stem != "imagenet":
                nxt = dict(x=self.c0, sums=sbn.sums_buf, mask_coef=sbn.coef)
                dx = st["dx"]
            else:
                dx = st["dx"]
            add, add_even = st["dz"], False
            if down:
                cd = self.conv[blk.down.name]
                # dc2 and dcs from one read of dz
                K.bn_bwd_apply_dual(st["dz"], st["c2"], b2.sums, b2.coef, b2.ggamma, b2.gbeta, st["dc2"],
                                    st["cs"], bd.sums, bd.coef, bd.ggamma, bd.gbeta, st["dcs"])
                K.conv_wgrad(st["x"], st["dcs"], blk.down.cout, 1, blk.down.stride, 0, cd.g, ws=self.wgws)
                if self._shortcut_even(blk):
                    # 1x1/s2 shortcut: only the (even, even) positions of dx get a gradient; write
                    # them into dx now, and conv1's parity-class data gradient adds there
                    K.conv_dgrad_s2_even(st["dcs"], cd.wt, blk.down.cin, dx)
                    add, add_even = dx, True
                else:
                    K.conv_dgrad(st["dcs"], cd.wt, blk.down.cin, 1, blk.down.stride, 0, st["dxs"])
                    add = st["dxs"]
            else:
                K.bn_bwd_apply_sums(st["dz"], None, st["c2"], b2.sums, b2.coef, b2.ggamma, b2.gbeta, st["dc2"])
            if st["bnin"]:
                K.conv3x3_bnin_wgrad(st["c1"], st["dc2"], b1, st["c1"].numel() // blk.conv1.cout, c2.g, ws=self.wgws)
            else:
                K.conv_wgrad(st["a1"], st["dc2"], blk.conv2.cout, 3, 1, 1, c2.g, ws=self.wgws)
            # a1 = relu(bn1(c1)): the mask is re-derived from c1 and bn1's coefficients
            bn1 = dict(x=st["c1"], sums=b1.sums_buf, mask_coef=b1.coef)
            if fuse:
                K.conv_dgrad(st["dc2"], c2.wt, blk.conv2.cin, 3, 1, 1, st["da1"], bn=bn1)
            else:
                K.conv_dgrad(st["dc2"], c2.wt, blk.conv2.cin, 3, 1, 1, st["da1"])
                K.bn_bwd_reduce(st["da1"], None, st["c1"], b1.sums_buf, mask_coef=b1.coef)
            K.bn_bwd_apply_sums(st["da1"], None, st["c1"], b1.sums, b1.coef, b1.ggamma, b1.gbeta, st["dc1"],
                                mask_coef=b1.coef)
            if st is self.blocks[0] and self.stem_onload:
                K.conv3x3_bnin_wgrad(self.c0, st["dc1"], sbn, self.c0.numel() // 64, c1.g, ws=self.wgws)
            else:
                K.conv_wgrad(st["x"], st["dc1"], blk.conv1.cout, 3, blk.conv1.stride, 1, c1.g, ws=self.wgws)
            K.conv_dgrad(st["dc1"], c1.wt, blk.conv1.cin, 3, blk.conv1.stride, 1, dx, add=add, bn=nxt,
                         add_even=add_even)
            dy = dx
            maybe_bucket(blk.conv1.off)
        # stem
        if spec.stem == "imagenet":
            K.maxpool_bwd(dy, self.p0_arg, self.da0)
            dy = self.da0
        if not (fuse and spec.stem != "imagenet"):
            K.bn_bwd_reduce(dy, None, self.c0, sbn.sums_buf, mask_coef=sbn.coef)
        K.bn_bwd_apply_sums(dy, None, self.c0, sbn.sums, sbn.coef, sbn.ggamma, sbn.gbeta, self.dc0,
                            mask_coef=sbn.coef)
        sc = spec.stem_conv
        K.conv_wgrad(self.x0, self.dc0, 64, sc.k, sc.stride, sc.pad, self.conv["stem"].g, ws=self.wgws)
        maybe_bucket(0, force=True)
        if side is not None:
            K.wgrad_side_join(end=True)
        return handles

    def _step_eager(self) -> None:
        self.grad.zero_()
        if not torch.cuda.is_current_stream_capturing():
            self.wgws.grow()  # size the split-K slab before any capture (first call: atomics)
        self.forward(train=True)
        handles = self.backward()
        self.phases.mark("compute")
        if self.bucket_wait is not None:
            self.bucket_wait(handles)  # the bucket all-reduces ran during backward: the exposed part
        if self.allreduce is not None:
            self.allreduce(self.grad)
        self.phases.mark("exchange")
        self.O.sgd_flat(self.params, self.grad, self.mom, self.lr, self.momentum, self.weight_decay,
                        shadow=self.shadow)
        self.wt()
        self.K.cursor_bump(self.cursor)
        self.phases.mark("update")

    def step(self) -> None:
        if self.graph is not None:
            self.graph.replay()
            return
        self._step_eager()

    def probe_step(self):
        """One eager training step with its phase boundaries recorded (utils/phases.py): returns
        a PendingPhases, resolved by the caller once the device has finished the step."""
        self.phases.arm()
        self._step_eager()
        pending = self.phases.finish()
        hooked = self.allreduce is not None or self.bucket_hook is not None
        pending.exchange_bytes = 4 * int(self.grad.numel()) if hooked else 0
        return pending

    def drop_graphs(self) -> None:
        """Release the captured step graph once the device is done with it (called by the
        runtime before it re-forms or tears down a group whose collectives the graph holds)."""
        if self.graph is not None or self.retired_graphs:
            torch.cuda.synchronize(self.device)
        self.graph = None
        self.reap_graphs(sync=False)

    def capture(self, warmup: int = 2) -> None:
        self.reap_graphs()  # graphs replaced since the last capture, freed after a sync (utils/graphs.py)
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

    # ------------------------------------------------------------------
    def compute_grads(self) -> torch.Tensor:
        """Forward + backward on the current batch (no update, no cursor bump)."""
        self.grad.zero_()
        self.forward(train=True)
        self.backward()
        return self.grad

    def stats(self) -> StepStats:
        return StepStats(float(self.loss.sum()) / self.batch, float(self.correct.sum()) / self.batch, self.batch)

    def get_flat(self) -> torch.Tensor:
        return self.params.clone()

    def set_flat(self, flat: torch.Tensor) -> None:
        self.params.copy_(flat.to(self.params))
        self.refresh_shadows()

    def running_stats(self) -> dict:
        return {name: (b.run_mean, b.run_var) for name, b in self.bn.items()}

    # ---- exact-resume state beyond the flat vectors (ckpt format v2) ----
    def state_extra(self) -> dict:
        d = {"cursor": self.cursor.double().cpu().numpy()}
        for name, b in self.bn.items():
            d[f"bn/{name}/mean"] = b.run_mean.double().cpu().numpy()
            d[f"bn/{name}/var"] = b.run_var.double().cpu().numpy()
        return d

    def load_state_extra(self, d: dict) -> None:
        if "cursor" in d:
            self.cursor.fill_(int(d["cursor"][0]))
        for name, b in self.bn.items():
            if f"bn/{name}/mean" in d:
                b.run_mean.copy_(torch.as_tensor(d[f"bn/{name}/mean"], dtype=torch.float32))
                b.run_var.copy_(torch.as_tensor(d[f"bn/{name}/var"], dtype=torch.float32))

    def buffers(self) -> list:
        """BN running statistics: broadcast with the parameters after a regroup, so every
        replica evaluates identically (each rank's statistics come from its own batches)."""
        return [t for b in self.bn.values() for t in (b.run_mean, b.run_var)]

    # ---- inference with running statistics ----
    def _eval_coef(self, bn: _BN, eps: float = 1e-5) -> torch.Tensor:
        sc = bn.gamma * torch.rsqrt(bn.run_var + eps)
        return torch.cat([sc, bn.beta - bn.run_mean * sc, bn.run_mean, torch.rsqrt(bn.run_var + eps)])

    def forward_eval(self) -> None:
        """Eval-mode forward of the current batch: every BatchNorm normalises with its running
        statistics (no batch statistics are computed, none are updated), then loss / correct
        / logits.  Same kernels as training -- conv_fwd without the statistics epilogue and
        bn_apply with coefficients folded from (gamma, beta, running mean, running var)."""
        K, spec = self.K, self.spec
        co = {name: self._eval_coef(b) for name, b in self.bn.items()}
        K.input_norm(self.x, self.y, self.cursor, self.batch, self.x0, self.labels, CIFAR_MEAN, CIFAR_STD)
        sc = spec.stem_conv
        K.conv_fwd(self.x0, self.conv["stem"].w, sc.cout, sc.k, sc.stride, sc.pad, y=self.c0)
        K.bn_apply(self.c0, co[spec.stem_bn.name], self.a0, relu=True)
        if spec.stem == "imagenet":
            K.maxpool_fwd(self.a0, self.p0, self.p0_arg)
        for st in self.blocks:
            blk: BlockSpec = st["spec"]
            c1, c2 = blk.conv1, blk.conv2
            K.conv_fwd(st["x"], self.conv[c1.name].w, c1.cout, c1.k, c1.stride, c1.pad, y=st["c1"])
            K.bn_apply(st["c1"], co[blk.bn1.name], st["a1"], relu=True)
            K.conv_fwd(st["a1"], self.conv[c2.name].w, c2.cout, c2.k, c2.stride, c2.pad, y=st["c2"])
            if blk.down is not None:
                d = blk.down
                K.conv_fwd(st["x"], self.conv[d.name].w, d.cout, d.k, d.stride, d.pad, y=st["cs"])
                K.bn_apply(st["c2"], co[blk.bn2.name], st["y"], relu=True, res=st["cs"], rcoef=co[blk.dbn.name])
            else:
                K.bn_apply(st["c2"], co[blk.bn2.name], st["y"], relu=True, res=st["x"])
        K.avgpool_fwd(self.feat_in, self.feat)
        K.conv_fwd(self.feat, self.fc_w, spec.classes, 1, 1, 0, yf=self.logits, bias=self.fc_b)
        K.softmax_ce(self.logits, self.labels, self.loss, self.correct, self.dlogits.view(self.batch, LOGIT_LD),
                     None, self.grad_scale)

    def evaluate(self, x_u8: torch.Tensor, y_u8: torch.Tensor) -> StepStats:
        """Eval-mode loss / accuracy over every whole batch of (x, y) with the running
        statistics; the training shard, cursor and statistics are left untouched."""
        hw = self.spec.in_hw
        x = x_u8.reshape(-1, hw, hw, 3).to(self.device).contiguous()
        y = y_u8.reshape(-1).to(self.device).to(torch.uint8).contiguous()
        nb = x.shape[0] // self.batch
        if nb < 1:
            raise ValueError("evaluation set smaller than one batch")
        saved = (self.x, self.y, self.cursor)
        self.x, self.y, self.cursor = x, y, torch.zeros(1, dtype=torch.int32, device=self.device)
        loss = corr = 0.0
        try:
            for _ in range(nb):
                self.forward_eval()
                loss += float(self.loss.sum())
                corr += float(self.correct.sum())
                self.K.cursor_bump(self.cursor)
        finally:
            self.x, self.y, self.cursor = saved
        n = nb * self.batch
        return StepStats(loss / n, corr / n, n)
