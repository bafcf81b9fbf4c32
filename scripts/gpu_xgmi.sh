#!/bin/bash
# xGMI exchange on one GPU: the multi-rank checks (2 and 3 ranks sharing the GPU), the GPU
# tests, then 2-rank MLP benches with the xGMI exchange and with the process-group all-reduce.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/xg
bash scripts/gpu_step.sh 120 xg/check2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 scripts/xgmi_check.py --same-device || exit 1
grep -q XGMI_CHECK_OK gpurun_out/xg/check2.log || exit 1
bash scripts/gpu_step.sh 120 xg/check3.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29547 scripts/xgmi_check.py --same-device || exit 1
bash scripts/gpu_step.sh 400 xg/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
bash scripts/gpu_step.sh 200 xg/bench2_xgmi.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 2 --steps 40 --warmup 8 --dist-backend gloo --ingest local --allreduce xgmi || exit 1
bash scripts/gpu_step.sh 200 xg/bench2_pg.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 2 --steps 40 --warmup 8 --dist-backend gloo --ingest local --allreduce pg || exit 1
grep -h "XGMI_CHECK_OK\|passed\|failed" gpurun_out/xg/*.log
