#!/bin/bash
# Timing knockouts of kernel-library builds on the ResNet-18 step (results of a knockout
# build are wrong, so no tests): one bench rep + kernel stats per variant ("base" = in-tree).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ko
so_of() { [ "$1" = base ] && echo "" || echo serverless_learn_amd/_native/variants/libslkernels_$1.so; }
for v in "$@"; do
  SL_KERNELS_SO=$(so_of $v) timeout -k 10 150 python bench.py --model resnet18 --ingest device --steps 30 --warmup 5 > gpurun_out/ko/${v}.log 2>&1 || exit 1
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ko/${v}.log)"
  SL_KERNELS_SO=$(so_of $v) bash scripts/gpu_step.sh 200 ko/prof_$v.log rocprofv3 --kernel-trace --stats -d gpurun_out/ko/prof_$v -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 || exit 1
done
