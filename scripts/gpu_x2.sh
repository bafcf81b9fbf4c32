#!/bin/bash
# Two-shot xGMI exchange + fp16 dW1 check: xgmi / MLP GPU tests, 1-GPU MLP bench (both forms),
# 2- and 4-rank rehearsals on the one GPU, kernel stats of the MLP step.
set -u
export TMPDIR=/tmp
tag=${1:-x2}
mkdir -p gpurun_out/$tag
S=scripts/gpu_step.sh
bash $S 300 $tag/pytest.log python -u -m pytest tests/test_xgmi_gpu.py tests/test_mlp_fused_gpu.py tests/test_runtime_gpu.py -x -v --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/$tag/pytest.log && ! grep -q "failed" gpurun_out/$tag/pytest.log || exit 1
bash $S 200 $tag/bench_mlp.log python bench.py --steps 20 --warmup 5 || exit 1
bash $S 200 $tag/bench_mlp200.log python bench.py || exit 1
bash $S 200 $tag/bench2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29552 bench.py --gpus 2 --steps 40 --warmup 8 --dist-backend gloo --ingest local || exit 1
bash $S 200 $tag/bench4.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29553 bench.py --gpus 4 --steps 40 --warmup 8 --dist-backend gloo --ingest local --batch 16384 || exit 1
bash $S 300 $tag/rocprof_mlp.log rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof_mlp -o run -- python bench.py --steps 100 --warmup 10 --ingest local || exit 1
