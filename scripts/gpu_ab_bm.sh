#!/bin/bash
# Rows-kernel tile A/B: 64-row tiles vs 128-row tiles (WMG 2 = default build, WMG 1 = variant w1).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
W1=serverless_learn_amd/_native/variants/libslkernels_w1.so
SL_KERNELS_SO=$W1 SL_MLP_ROWS_BM=128 bash scripts/gpu_step.sh 300 w1_tests.log python -u -m pytest tests/test_mlp_fused_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/w1_tests.log && ! grep -q "failed" gpurun_out/w1_tests.log || exit 1
for rep in 1 2; do
  for cfg in "64 base" "128 base" "128 w1"; do
    set -- $cfg; so=""; [ "$2" != "base" ] && so=$W1
    SL_KERNELS_SO=$so SL_MLP_ROWS_BM=$1 timeout -k 10 100 python bench.py --ingest local --steps 400 > gpurun_out/abbm_$1_$2_$rep.log 2>&1 || exit 1
    echo "bm=$1 $2 rep=$rep $(grep -o '"value": [0-9.]*' gpurun_out/abbm_$1_$2_$rep.log)"
  done
done
