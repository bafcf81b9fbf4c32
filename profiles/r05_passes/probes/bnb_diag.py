"""Per-layer gradient agreement of the ResNet engine: fused BN backward vs unfused, and
unfused vs unfused (run-to-run order noise of the atomics)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def grads(fuse, batch=32, hw=32, seed=3):
    from serverless_learn_amd.data.synthetic import make_cifar_like
    from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer

    os.environ["SL_BNB_FUSE"] = "1" if fuse else "0"
    tr = FusedResNetTrainer(batch=batch, device="cuda", stem="cifar", momentum=0.0, weight_decay=0.0, in_hw=hw)
    x, y = make_cifar_like(batch, seed=seed, hw=hw)
    tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
    g = tr.compute_grads().clone()
    torch.cuda.synchronize()
    return tr, g


tr, gf = grads(True)
_, gu = grads(False)
_, gu2 = grads(False)
_, gf2 = grads(True)
for c in tr.spec.convs():
    s = slice(c.off, c.off + c.numel)
    print(f"{c.name:12s} fused/unfused {float(F.cosine_similarity(gf[s], gu[s], dim=0)):.6f}  "
          f"unfused/unfused {float(F.cosine_similarity(gu[s], gu2[s], dim=0)):.6f}  "
          f"fused/fused {float(F.cosine_similarity(gf[s], gf2[s], dim=0)):.6f}")
print("all", float(F.cosine_similarity(gf, gu, dim=0)), float(F.cosine_similarity(gu, gu2, dim=0)),
      float(F.cosine_similarity(gf, gf2, dim=0)))
