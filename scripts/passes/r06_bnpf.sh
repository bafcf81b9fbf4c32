#!/bin/bash
# Round 6, pass 21: BN streams with the next chunk's loads in flight during this chunk's math
# (SL_BN_PF) vs SL_BN_PF=0 (variant "bnpf0"): conv/BN numerics, ResNet-18 A/B, kernel tables.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${PASS_TAG:-r06_bnpf}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_cnn_gpu.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
V=serverless_learn_amd/_native/variants/libslkernels_bnpf0.so
for rep in 1 2 3; do
  for v in base bnpf0; do
    so=""; [ $v = bnpf0 ] && so=$V
    SL_KERNELS_SO=$so timeout -k 10 300 python bench.py --model resnet18 --ingest device > $O/resnet_${v}_$rep.json 2> $O/resnet_${v}_$rep.err || exit 4
    echo "$v rep=$rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/resnet_${v}_$rep.json | tr '\n' ' ')"
  done
done
for v in base bnpf0; do
  so=""; [ $v = bnpf0 ] && so=$V
  SL_KERNELS_SO=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 \
    > $O/prof_$v.log 2>&1 || exit 5
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.txt 2>&1 || true
  echo "== $v"; head -10 $O/kernels_$v.txt
done
