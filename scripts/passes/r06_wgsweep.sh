#!/bin/bash
# Round 6, pass 11: split-K targets of the weight-gradient kernels re-swept on the lean kernels
# (round 5 picked 384 = 192 big workgroups: 198-216 of 256 CUs busy in stages 3-4).
# SL_WGRAD_BIG_TARGET = big-kernel workgroups; SL_WGRAD_WGS = the 64/128-wide kernels' target.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${PASS_TAG:-r06_wgsweep}; mkdir -p $O
CFGS=("0 384" "256 384" "320 384" "512 384" "0 512" "0 768")
[ -n "${WGS_CFGS:-}" ] && IFS=, read -r -a CFGS <<< "$WGS_CFGS"
for rep in 1 2; do
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    tag="big$1_w$2"
    SL_WGRAD_BIG_TARGET=$1 SL_WGRAD_WGS=$2 timeout -k 10 300 python bench.py --model resnet18 --ingest device > $O/r_${tag}_$rep.json 2> $O/r_${tag}_$rep.err || exit 4
    echo "$tag rep=$rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/r_${tag}_$rep.json | tr '\n' ' ')"
  done
done
