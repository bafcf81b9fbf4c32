#!/bin/bash
# Round 6, pass 22: BASELINE config 5 on the GPU with the round-6 kernels and the shared-GPU
# queue cap -- 4 worker processes on the one GPU: kill2 and whole-group replacement, MLP over the
# live xGMI exchange and ResNet-18 over gloo; then the whole GPU suite once more.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${PASS_TAG:-r06_elastic}; mkdir -p $O
i=0
for cfg in "mlp kill2 --xgmi-gloo" "mlp all --xgmi-gloo" "resnet18 kill2" "resnet18 all"; do
  set -- $cfg
  i=$((i+1))
  timeout -k 10 280 python -u scripts/elastic_demo.py --device cuda --dp-backend gloo --model $1 --scenario $2 ${3:-} \
    --batch 256 --timeout 240 --logdir $O/run$i > $O/run$i.json 2> $O/run$i.err || { echo "elastic $cfg failed"; tail -3 $O/run$i.err; exit 1; }
  echo "elastic $cfg: $(tail -1 $O/run$i.json | cut -c1-300)"
done
