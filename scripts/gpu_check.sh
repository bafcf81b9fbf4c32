#!/bin/bash
# One GPU validation pass: tests, bench, rocprof kernel stats.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_step.sh 900 pytest_gpu.log python -m pytest tests -m gpu -x -q || exit 1
bash scripts/gpu_step.sh 300 bench1.log python bench.py --steps 200 --warmup 20 || exit 1
bash scripts/gpu_step.sh 300 bench_local.log python bench.py --steps 200 --warmup 20 --ingest local --batch 65536 --shard-batches 4 || exit 1
bash scripts/gpu_step.sh 400 rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 100 --warmup 10 --ingest local || exit 1
find gpurun_out/prof -name '*kernel_stats.csv' | head -5
