"""Run the CNN engine's forward+backward repeatedly on the same batch and
report gradient/stat differences between runs (debug aid for atomics/folds)."""
import sys
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from serverless_learn_amd.data.synthetic import make_cifar_like
from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer

x, y = make_cifar_like(64, seed=8)
tr = FusedResNetTrainer(batch=32, device="cuda", seed=2)
tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
gs, sts = [], []
for i in range(4):
    g = tr.compute_grads().clone()
    torch.cuda.synchronize()
    gs.append(g)
    sts.append({n: (b.stats.clone(), b.sums.clone()) for n, b in tr.bn.items()})
def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-30))
for i in range(1, 4):
    print("run", i, "grad rel", rel(gs[i], gs[0]), "cos", float(F.cosine_similarity(gs[i], gs[0], dim=0)))
    worst = max(((n, rel(sts[i][n][0], sts[0][n][0]), rel(sts[i][n][1], sts[0][n][1])) for n in sts[0]), key=lambda t: max(t[1], t[2]))
    print("   worst BN stats/sums rel", worst)
spec = tr.spec
for c in list(spec.convs())[-3:]:
    print(c.name, rel(gs[1][c.off:c.off + c.numel], gs[0][c.off:c.off + c.numel]))

# ---- first backward tensor that differs between two identical runs ----
def snap():
    tr.compute_grads()
    torch.cuda.synchronize()
    d = {"dfeat": tr.dfeat.clone(), "dfeat_in": tr.dfeat_in.clone()}
    for i, st in enumerate(tr.blocks):
        for k in ("dz", "dc2", "da1", "dc1", "dx"):
            d[f"b{i}.{k}"] = st[k].clone()
        for nm in ("bn1", "bn2"):
            bn = tr.bn[getattr(spec.blocks[i], nm).name]
            d[f"b{i}.{nm}.sums"] = bn.sums.clone()
    return d
A, B = snap(), snap()
order = ["dfeat", "dfeat_in"] + [f"b{i}.{k}" for i in reversed(range(len(tr.blocks)))
                                 for k in ("bn2.sums", "dz", "dc2", "da1", "bn1.sums", "dc1", "dx")]
for k in order:
    r = rel(A[k].float(), B[k].float())
    print(f"{k:16s} {r:.3e}")
