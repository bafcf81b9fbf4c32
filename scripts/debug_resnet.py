"""Per-block forward/backward comparison of the HIP ResNet engine vs fp32 torch (debug aid)."""
import sys
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from serverless_learn_amd.data.synthetic import make_cifar_like
from serverless_learn_amd.models.resnet import conv_weight_nchw, normalize_input
from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer

DEV = "cuda"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
tr = FusedResNetTrainer(batch=B, device=DEV, momentum=0.0, weight_decay=0.0)
x, y = make_cifar_like(B, seed=3)
tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
g = tr.compute_grads().clone()
torch.cuda.synchronize()
spec = tr.spec
flat = tr.params.detach().clone().requires_grad_(True)


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def bn(xx, b):
    return F.batch_norm(xx, None, None, flat[b.g_off:b.g_off + b.c], flat[b.b_off:b.b_off + b.c], training=True)


def conv(xx, c):
    return F.conv2d(xx, conv_weight_nchw(flat, c), stride=c.stride, padding=c.pad)


nhwc = lambda t: t.permute(0, 2, 3, 1)  # noqa
xi = normalize_input(torch.from_numpy(x).to(DEV))
c0 = conv(xi, spec.stem_conv)
print("stem conv out", rel(tr.c0, nhwc(c0)))
a = F.relu(bn(c0, spec.stem_bn))
if tr.stem_onload:  # a0 is rebuilt on load from c0 by the engine, never stored: materialise it
    tr.K.bn_apply(tr.c0, tr.bn[spec.stem_bn.name].coef, tr.a0, relu=True)
print("stem act", rel(tr.a0, nhwc(a)))
outs = []
for i, (st, blk) in enumerate(zip(tr.blocks, spec.blocks)):
    a.retain_grad()
    outs.append(a)
    c1 = conv(a, blk.conv1)
    o = F.relu(bn(c1, blk.bn1))
    c2 = conv(o, blk.conv2)
    o2 = bn(c2, blk.bn2)
    sc = bn(conv(a, blk.down), blk.dbn) if blk.down is not None else a
    a = F.relu(o2 + sc)
    print(f"block {i} fwd: c1 {rel(st['c1'], nhwc(c1)):.4f} a1 {rel(st['a1'], nhwc(o)):.4f} "
          f"c2 {rel(st['c2'], nhwc(c2)):.4f} y {rel(st['y'], nhwc(a)):.4f}")
a.retain_grad()
feat = a.mean((2, 3))
wf = flat[spec.fc_w:spec.fc_w + spec.classes * 512].view(spec.classes, 512)
logits = F.linear(feat, wf, flat[spec.fc_b:spec.fc_b + spec.classes])
print("logits", rel(tr.logits, logits))
loss = F.cross_entropy(logits, torch.from_numpy(y).to(DEV).long(), reduction="sum") / B
loss.backward()
print("dfeat_in", rel(tr.dfeat_in, nhwc(a.grad)))
for i in reversed(range(len(tr.blocks))):
    st = tr.blocks[i]
    print(f"block {i} dx {rel(st['dx'], nhwc(outs[i].grad)):.4f}")
for c in spec.convs():
    print(c.name, "dW rel", round(rel(g[c.off:c.off + c.numel], flat.grad[c.off:c.off + c.numel]), 4))

# ---- block-local check: fp32 torch backward of the LAST block from the engine's own tensors ----
st, blk = tr.blocks[-1], spec.blocks[-1]
f32 = lambda t: t.float().permute(0, 3, 1, 2).detach()  # noqa
xin = f32(st["x"]).requires_grad_(True)
wf32 = tr.shadow.float()
def conv_s(xx, c):
    return F.conv2d(xx, conv_weight_nchw(wf32, c), stride=c.stride, padding=c.pad)
def bn_s(xx, b):
    return F.batch_norm(xx, None, None, tr.params[b.g_off:b.g_off + b.c], tr.params[b.b_off:b.b_off + b.c], training=True)
c1 = conv_s(xin, blk.conv1)
o = F.relu(bn_s(c1, blk.bn1))
c2 = conv_s(o, blk.conv2)
yy = F.relu(bn_s(c2, blk.bn2) + xin)
yy.backward(f32(tr.dfeat_in))
print("LOCAL last block: y", rel(st["y"], nhwc(yy)), "dx", rel(st["dx"], nhwc(xin.grad)))
# same but BN-2 input taken as the engine's stored c2 (bf16) and mask from engine y
c2e = f32(st["c2"]).requires_grad_(True)
y2 = F.relu(bn_s(c2e, blk.bn2) + f32(st["x"]))
y2.backward(f32(tr.dfeat_in))
print("LOCAL bn2 only: dc2", rel(st["dc2"], nhwc(c2e.grad)), "dz", rel(st["dz"], nhwc(f32(tr.dfeat_in) * (y2 > 0))))
