#!/bin/bash
# A/B of kernel variants on one box: bench each (and BM=128) back to back.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_step.sh 300 ab_tests.log python -u -m pytest tests/test_mlp_fused_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/ab_tests.log && ! grep -q "failed" gpurun_out/ab_tests.log || exit 1
for v in "$@"; do
  so=""; [ "$v" != "base" ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  for bm in 64 128; do
    SL_KERNELS_SO=$so SL_MLP_ROWS_BM=$bm timeout -k 10 100 python bench.py --ingest local --steps 300 > gpurun_out/ab_${v}_$bm.log 2>&1 || exit 1
    echo "$v bm=$bm $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$bm.log)"
  done
done
