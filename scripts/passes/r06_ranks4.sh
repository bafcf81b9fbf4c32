#!/bin/bash
# Round 6, pass 18b: why 4+ ranks sharing the one GPU run 25x slower than 2 (MLP over the xGMI
# exchange, W = 4): the exchange's waits (--allreduce pg instead) or the processes' hardware
# queues (GPU_MAX_HW_QUEUES=2 per process instead of 4).
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_ranks4; mkdir -p $O
timeout -k 10 300 python bench.py --gpus 4 --oversubscribe --dist-backend gloo --steps 20 --warmup 5 --ingest local --allreduce pg > $O/pg.json 2> $O/pg.err || exit 1
echo "W=4 pg $(grep -o '"value": [0-9.]*\|"replicas_identical": [a-z]*\|"collective_backend": "[a-z0-9-]*"' $O/pg.json | tr '\n' ' ')"
GPU_MAX_HW_QUEUES=2 timeout -k 10 300 python bench.py --gpus 4 --oversubscribe --dist-backend gloo --steps 20 --warmup 5 --ingest local > $O/q2.json 2> $O/q2.err || exit 2
echo "W=4 xgmi queues=2 $(grep -o '"value": [0-9.]*\|"replicas_identical": [a-z]*\|"collective_backend": "[a-z0-9-]*"' $O/q2.json | tr '\n' ' ')"
timeout -k 10 300 python bench.py --gpus 3 --oversubscribe --dist-backend gloo --steps 20 --warmup 5 --ingest local > $O/w3.json 2> $O/w3.err || exit 3
echo "W=3 xgmi $(grep -o '"value": [0-9.]*\|"replicas_identical": [a-z]*\|"collective_backend": "[a-z0-9-]*"' $O/w3.json | tr '\n' ' ')"
