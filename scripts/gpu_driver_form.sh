#!/bin/bash
# The driver's bench form (MLP, --steps 20 --warmup 5, fresh process each) three times on one box,
# then the 200-step default and the ResNet-18 bench once: the spread the round-end number sits in.
set -u
rm -rf gpurun_out/drv
mkdir -p gpurun_out/drv
for i in 1 2 3; do
  bash scripts/gpu_step.sh 200 drv/mlp_k20_$i.log python bench.py --steps 20 --warmup 5 || exit 1
done
bash scripts/gpu_step.sh 200 drv/mlp_k200.log python bench.py || exit 1
bash scripts/gpu_step.sh 200 drv/resnet.log python bench.py --model resnet18 --ingest device || exit 1
grep -ho '"value": [0-9.]*\|"steps": [0-9]*\|"model": "[a-z0-9-]*' gpurun_out/drv/*.log | paste - - -
