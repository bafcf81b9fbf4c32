#!/bin/bash
# A/B of MLP kernel variants on one box (64-row tiles only), each run twice interleaved.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_step.sh 300 ab_tests.log python -u -m pytest tests/test_mlp_fused_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/ab_tests.log && ! grep -q "failed" gpurun_out/ab_tests.log || exit 1
for rep in 1 2; do
for v in "$@"; do
  so=""; [ "$v" != "base" ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 100 python bench.py --ingest local --steps 400 > gpurun_out/ab_${v}_$rep.log 2>&1 || exit 1
  echo "$v rep=$rep $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log)"
done
done
