#!/bin/bash
# Round 6, pass 9b: is conv_gemm_wide_kernel exact?  Its k-order and epilogue equal
# conv_gemm_big_kernel's, so in the deterministic build (fixed-point cross-workgroup sums) a
# ResNet-18 run must give the same losses with SL_GEMM_WIDE=1 (twice) and 0.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_widedet; mkdir -p $O
for v in 1 0 1; do
  SL_DETERMINISTIC=1 SL_GEMM_WIDE=$v timeout -k 10 300 python bench.py --model resnet18 --ingest device --steps 20 --warmup 5 > $O/det_w$v.json 2> $O/det_w$v.err || exit 4
  echo "det wide=$v $(grep -o '"value": [0-9.]*\|"train_loss_[a-z]*": [0-9.]*\|"train_acc_last": [0-9.]*' $O/det_w$v.json | tr '\n' ' ')"
done
for i in 1 2 3; do
  SL_GEMM_WIDE=1 timeout -k 10 300 python bench.py --model resnet18 --ingest device > $O/w1_$i.json 2> $O/w1_$i.err || exit 4
  echo "wide=1 $(grep -o '"train_loss_last": [0-9.]*\|"train_acc_last": [0-9.]*' $O/w1_$i.json | tr '\n' ' ')"
  SL_GEMM_WIDE=0 timeout -k 10 300 python bench.py --model resnet18 --ingest device > $O/w0_$i.json 2> $O/w0_$i.err || exit 4
  echo "wide=0 $(grep -o '"train_loss_last": [0-9.]*\|"train_acc_last": [0-9.]*' $O/w0_$i.json | tr '\n' ' ')"
done
