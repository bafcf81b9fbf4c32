#!/bin/bash
# Round regression on one GPU: every GPU test, smoke(), the default benches (MLP + ResNet-18),
# the 2-rank xGMI rehearsal, and rocprofv3 kernel stats of both benches.
set -u
export TMPDIR=/tmp
tag=${1:-reg}
mkdir -p gpurun_out/$tag
S=scripts/gpu_step.sh
bash $S 600 $tag/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/$tag/pytest_gpu.log && ! grep -q "failed" gpurun_out/$tag/pytest_gpu.log || exit 1
bash $S 120 $tag/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash $S 200 $tag/bench_mlp.log python bench.py --steps 20 --warmup 5 || exit 1
bash $S 200 $tag/bench_mlp200.log python bench.py || exit 1
bash $S 200 $tag/bench_resnet.log python bench.py --model resnet18 --ingest device || exit 1
bash $S 200 $tag/bench2_xgmi.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29552 bench.py --gpus 2 --steps 40 --warmup 8 --dist-backend gloo --ingest local || exit 1
bash $S 300 $tag/rocprof_mlp.log rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof_mlp -o run -- python bench.py --steps 100 --warmup 10 --ingest local || exit 1
bash $S 300 $tag/rocprof_resnet.log rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof_resnet -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 || exit 1
