#!/usr/bin/env python3
"""Whole-engine check of the ResNet-18 backward at a bench-sized batch, in
its own process so the kernel build can be chosen (SL_DETERMINISTIC=1: the deterministic
library; default: the shipped build with split-K atomics).  Two engine runs of the same batch
measure the build's own run-to-run noise per layer (cosine of the two gradients); each run is
compared with the fp32 autograd reference (models.resnet.ref_grads).  Prints one JSON line:
per conv / BN layer [name, cos(engine, fp32), cos(run 1, run 2)], the loss pair and the fc cosine."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F


def main() -> int:
    from serverless_learn_amd.data.synthetic import make_cifar_like
    from serverless_learn_amd.models.resnet import ref_grads, running_stats
    from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer

    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    tr = FusedResNetTrainer(batch=batch, device=dev, momentum=0.0, weight_decay=0.0)
    x, y = make_cifar_like(batch, seed=seed)
    tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
    g1 = tr.compute_grads().clone()
    loss = float(tr.loss.sum())
    g2 = tr.compute_grads().clone()
    torch.cuda.synchronize()
    loss_ref, _, g_ref = ref_grads(tr.spec, tr.params.detach().clone(), torch.from_numpy(x).to(dev),
                                   torch.from_numpy(y).to(dev), 1.0 / batch, running_stats(tr.spec, dev))
    spec = tr.spec
    rows = []
    for c in spec.convs():
        sl = slice(c.off, c.off + c.numel)
        rows.append([c.name, float(F.cosine_similarity(g1[sl], g_ref[sl], dim=0)),
                     float(F.cosine_similarity(g1[sl], g2[sl], dim=0))])
    for bn in spec.bns():
        a1 = torch.cat([g1[bn.g_off:bn.g_off + bn.c], g1[bn.b_off:bn.b_off + bn.c]])
        a2 = torch.cat([g2[bn.g_off:bn.g_off + bn.c], g2[bn.b_off:bn.b_off + bn.c]])
        ar = torch.cat([g_ref[bn.g_off:bn.g_off + bn.c], g_ref[bn.b_off:bn.b_off + bn.c]])
        rows.append([bn.name, float(F.cosine_similarity(a1, ar, dim=0)), float(F.cosine_similarity(a1, a2, dim=0))])
    fc = slice(spec.fc_w, spec.fc_w + spec.classes * 512)
    print(json.dumps({"batch": batch, "deterministic_build": os.environ.get("SL_DETERMINISTIC", "0") == "1",
                      "loss": loss / batch, "loss_ref": float(loss_ref) / batch,
                      "fc_cos": float(F.cosine_similarity(g1[fc], g_ref[fc], dim=0)),
                      "worst_ref": min(r[1] for r in rows), "worst_noise": min(r[2] for r in rows),
                      "layers": [[n, round(a, 5), round(b, 5)] for n, a, b in rows]}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
