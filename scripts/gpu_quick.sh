#!/bin/bash
# Quick MLP check: kernel tests, bench (auto and forced variants), kernel stats.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_step.sh 300 mlp_tests.log python -u -m pytest tests/test_mlp_fused_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/mlp_tests.log && ! grep -q "failed" gpurun_out/mlp_tests.log || exit 1
bash scripts/gpu_step.sh 200 bench1.log python bench.py --ingest local "$@" || exit 1
SL_MLP_ROWS_BM=64 bash scripts/gpu_step.sh 200 bench1_bm64.log python bench.py --ingest local "$@" || exit 1
bash scripts/gpu_step.sh 200 bench_16k.log python bench.py --ingest local --batch 16384 || exit 1
bash scripts/gpu_step.sh 200 rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 50 --warmup 10 --ingest local "$@" || exit 1
python scripts/rocprof_summary.py gpurun_out/prof/run_results.db | head -6
