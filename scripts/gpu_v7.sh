#!/bin/bash
# Round-1 v7 validation: all gpu tests, MLP bench (default + 16k), CNN bench, rocprof of MLP + CNN.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_step.sh 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
bash scripts/gpu_step.sh 200 bench1.log python bench.py || exit 1
bash scripts/gpu_step.sh 200 bench_16k.log python bench.py --batch 16384 --ingest local || exit 1
bash scripts/gpu_step.sh 200 bench_cnn.log python bench.py --model resnet18 --ingest device --batch 512 || exit 1
bash scripts/gpu_step.sh 300 rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 100 --warmup 10 --ingest local || exit 1
bash scripts/gpu_step.sh 300 rocprof_cnn.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cnn -o run -- python bench.py --model resnet18 --ingest device --batch 512 --steps 10 --warmup 3 || exit 1
