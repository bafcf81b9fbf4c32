#!/bin/bash
# Per-GPU batch sweep of both benches (one box): ResNet-18 at 1K/2K/4K images, the MLP at
# 16K-128K rows (200 steps), and the driver's 20-step MLP form at the default batch.
set -u
rm -rf gpurun_out/sw
mkdir -p gpurun_out/sw
for b in 1024 2048 4096; do
  bash scripts/gpu_step.sh 200 sw/resnet_b$b.log python bench.py --model resnet18 --ingest device --batch $b --steps 20 --warmup 5 || exit 1
done
for b in 16384 32768 65536 131072; do
  bash scripts/gpu_step.sh 200 sw/mlp_b$b.log python bench.py --ingest local --batch $b --steps 200 --warmup 20 || exit 1
done
bash scripts/gpu_step.sh 200 sw/mlp_k20.log python bench.py --steps 20 --warmup 5 || exit 1
grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"per_gpu_batch": [0-9]*\|"model": "[a-z0-9-]*' gpurun_out/sw/*.log | paste - - - -
