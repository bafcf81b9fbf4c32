#!/bin/bash
# Round 6, pass 16: stability soaks of the graph-replayed 1-GPU step (scripts/soak.py): MLP and
# ResNet-18 for 8 minutes each, one progress line per 20 s (throughput, loss, device memory).
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_soak2; mkdir -p $O
timeout -k 10 120 python -u scripts/soak.py --model mlp --seconds 20 --interval 10 > $O/mlp_short.jsonl 2>$O/mlp_short.err || exit 1
tail -1 $O/mlp_short.jsonl
timeout -k 10 150 python -u scripts/soak.py --model resnet18 --seconds 20 --interval 10 > $O/resnet_short.jsonl 2>$O/resnet_short.err || exit 2
tail -1 $O/resnet_short.jsonl
timeout -k 10 600 python -u scripts/soak.py --model mlp --seconds ${SOAK_S:-480} > $O/mlp.jsonl 2>$O/mlp.err || exit 3
tail -1 $O/mlp.jsonl
timeout -k 10 600 python -u scripts/soak.py --model resnet18 --seconds ${SOAK_S:-480} > $O/resnet.jsonl 2>$O/resnet.err || exit 4
tail -1 $O/resnet.jsonl
