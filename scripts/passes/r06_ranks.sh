#!/bin/bash
# Round 6 (also re-run on the final tree with PASS_TAG=r06_ranks_final): multi-rank rehearsals on the round-6 kernels, ranks sharing the one GPU:
# ResNet-18 (gloo, B = 256 per rank) at W = 2 and 4, the MLP over the xGMI exchange at W = 2, 4, 8.
# Every run must report bit-identical replicas.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${PASS_TAG:-r06_ranks}; mkdir -p $O
timeout -k 10 200 python -c "import torch; print(torch.__version__)" > $O/torch.txt 2>&1 || exit 1
for w in ${RESNET_W:-2 4}; do
  SL_BENCH_PROGRESS=1 timeout -k 10 170 python bench.py --gpus $w --oversubscribe --dist-backend gloo --model resnet18 --batch 256 --steps 4 --warmup 2 --ingest device > $O/resnet_w$w.json 2> $O/resnet_w$w.err || exit 2
  echo "resnet W=$w $(grep -o '"value": [0-9.]*\|"replicas_identical": [a-z]*' $O/resnet_w$w.json | tr '\n' ' ')"
done
for w in ${MLP_W:-2 4 8}; do
  timeout -k 10 300 python bench.py --gpus $w --oversubscribe --dist-backend gloo --steps 20 --warmup 5 --ingest local > $O/mlp_w$w.json 2> $O/mlp_w$w.err || exit 3
  echo "mlp W=$w $(grep -o '"value": [0-9.]*\|"replicas_identical": [a-z]*\|"collective_backend": "[a-z0-9-]*"' $O/mlp_w$w.json | tr '\n' ' ')"
done
