#!/bin/bash
# A/B of kernel-library builds (serverless_learn_amd/_native/variants/libslkernels_<v>.so, or "base"):
# the CNN GPU tests under EVERY build first, then interleaved ResNet-18 bench reps, then kernel stats.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/abs
so_of() { [ "$1" = base ] && echo "" || echo serverless_learn_amd/_native/variants/libslkernels_$1.so; }
for v in "$@"; do
  SL_KERNELS_SO=$(so_of $v) bash scripts/gpu_step.sh 300 abs/tests_$v.log python -u -m pytest tests/test_cnn_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
  grep -q "passed" gpurun_out/abs/tests_$v.log && ! grep -q "failed" gpurun_out/abs/tests_$v.log || exit 1
done
for rep in 1 2; do
for v in "$@"; do
  SL_KERNELS_SO=$(so_of $v) timeout -k 10 150 python bench.py --model resnet18 --ingest device --steps 30 --warmup 5 > gpurun_out/abs/${v}_$rep.log 2>&1 || exit 1
  echo "$v rep=$rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' gpurun_out/abs/${v}_$rep.log | tr '\n' ' ')"
done
done
for v in "$@"; do
  SL_KERNELS_SO=$(so_of $v) bash scripts/gpu_step.sh 200 abs/prof_$v.log rocprofv3 --kernel-trace --stats -d gpurun_out/abs/prof_$v -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 || exit 1
done
