#!/bin/bash
# Round 6, pass 7: issue-priority knobs on the lean conv k-loops (ResNet-18 driver form,
# interleaved): base, SL_MFMA_PRIO=1 (setprio around MFMA clusters), SL_WAVE_PRIO=1 (younger
# half of each workgroup at priority 1).
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_prio; mkdir -p $O
for rep in 1 2 3; do
  for v in base prio yp; do
    so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 300 python bench.py --model resnet18 --ingest device > $O/resnet_${v}_$rep.json 2> $O/resnet_${v}_$rep.err || exit 4
    echo "$v rep=$rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/resnet_${v}_$rep.json | tr '\n' ' ')"
  done
done
