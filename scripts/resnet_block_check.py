#!/usr/bin/env python3
"""Per-block fp32 check of the ResNet-18 engine's backward at a given batch (models.resnet
.block_backward_errors), in its own process so the kernel build can be chosen
(SL_DETERMINISTIC=1: the deterministic library).  Prints one JSON line: the batch, the build,
the worst relative error and every (conv, dx | dW, error)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main() -> int:
    from serverless_learn_amd.data.synthetic import make_cifar_like
    from serverless_learn_amd.models.resnet import block_backward_errors
    from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer

    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    tr = FusedResNetTrainer(batch=batch, device="cuda", momentum=0.0, weight_decay=0.0)
    x, y = make_cifar_like(batch, seed=seed)
    tr.load_shard(torch.from_numpy(x), torch.from_numpy(y))
    g = tr.compute_grads().clone()
    torch.cuda.synchronize()
    errs = block_backward_errors(tr, g)
    print(json.dumps({"batch": batch, "deterministic_build": os.environ.get("SL_DETERMINISTIC", "0") == "1",
                      "worst": max(e[2] for e in errs), "errors": [[a, b, round(c, 5)] for a, b, c in errs]}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
