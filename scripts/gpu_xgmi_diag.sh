#!/bin/bash
set -u
mkdir -p gpurun_out/xg
bash scripts/gpu_step.sh 120 xg/diag.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29544 scripts/xgmi_check.py --same-device || exit 1

bash scripts/gpu_step.sh 120 xg/diag_b.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29545 scripts/xgmi_check.py --same-device || exit 1
bash scripts/gpu_step.sh 120 xg/diag_c.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29546 scripts/xgmi_check.py --same-device || exit 1
grep -h "DIAG\|XGMI_CHECK_OK\|Error" gpurun_out/xg/diag*.log
