#!/bin/bash
# MLP: steps-per-graph sweep (1 / 4 / 8 / 16) + a kernel trace of the default.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_step.sh 300 mlp_tests.log python -u -m pytest tests/test_mlp_fused_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/mlp_tests.log && ! grep -q "failed" gpurun_out/mlp_tests.log || exit 1
for u in 1 4 8 16; do
  bash scripts/gpu_step.sh 200 bench_u$u.log python bench.py --ingest local --unroll $u || exit 1
done
bash scripts/gpu_step.sh 200 bench_u8_16k.log python bench.py --ingest local --batch 16384 || exit 1
bash scripts/gpu_step.sh 200 rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 48 --warmup 16 --ingest local || exit 1
