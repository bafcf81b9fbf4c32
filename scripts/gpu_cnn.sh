#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_step.sh 600 cnn_tests.log python -m pytest tests/test_cnn_gpu.py -x -q || exit 1
bash scripts/gpu_step.sh 300 bench_cnn.log python bench.py --model resnet18 --ingest local || exit 1
bash scripts/gpu_step.sh 300 bench_cnn_b512.log python bench.py --model resnet18 --ingest local --batch 512 || exit 1
bash scripts/gpu_step.sh 400 rocprof_cnn.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cnn -o run -- python bench.py --model resnet18 --ingest local --steps 10 --warmup 3 || exit 1
