#!/bin/bash
# Full regression on one GPU: every gpu test, both benches, multi-rank gloo rehearsal of both,
# rocprof kernel stats of both.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_step.sh 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed" gpurun_out/pytest_gpu.log || exit 1
bash scripts/gpu_step.sh 200 bench1.log python bench.py || exit 1
bash scripts/gpu_step.sh 200 bench_cnn.log python bench.py --model resnet18 --ingest device || exit 1
bash scripts/gpu_step.sh 300 bench_gloo2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --ingest local || exit 1
bash scripts/gpu_step.sh 300 bench_gloo2_cnn.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --model resnet18 --batch 256 --steps 5 --warmup 2 --dist-backend gloo --ingest device || exit 1
bash scripts/gpu_step.sh 300 rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 100 --warmup 10 --ingest local || exit 1
bash scripts/gpu_step.sh 300 rocprof_cnn.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cnn -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 || exit 1
