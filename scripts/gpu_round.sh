#!/bin/bash
# Full GPU validation: all gpu tests, MLP + CNN benches, rocprof of both.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_step.sh 900 pytest_gpu.log python -m pytest tests -m gpu -x -q || exit 1
bash scripts/gpu_step.sh 300 bench1.log python bench.py || exit 1
bash scripts/gpu_step.sh 300 bench_dev.log python bench.py --ingest device --batch 65536 --shard-batches 4 || exit 1
bash scripts/gpu_step.sh 300 bench_cnn.log python bench.py --model resnet18 --ingest device --batch 512 || exit 1
bash scripts/gpu_step.sh 400 rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 100 --warmup 10 --ingest local || exit 1
bash scripts/gpu_step.sh 400 rocprof_cnn.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cnn -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 || exit 1
