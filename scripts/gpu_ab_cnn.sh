#!/bin/bash
# A/B of kernel variants on the ResNet-18 bench (one box, back to back).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  so=""; [ "$v" != "base" ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 150 python bench.py --model resnet18 --ingest device --steps 20 --warmup 5 > gpurun_out/abc_$v.log 2>&1 || exit 1
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/abc_$v.log)"
done
