#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_step.sh 600 mlp_tests.log python -m pytest tests/test_mlp_fused_gpu.py tests/test_runtime_gpu.py -x -q || exit 1
bash scripts/gpu_step.sh 300 bench1.log python bench.py --ingest local || exit 1
bash scripts/gpu_step.sh 300 bench_b65536.log python bench.py --ingest local --batch 65536 --shard-batches 4 || exit 1
bash scripts/gpu_step.sh 400 rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 100 --warmup 10 --ingest local || exit 1
