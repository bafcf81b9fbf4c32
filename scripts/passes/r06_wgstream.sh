#!/bin/bash
# Round 6, pass 25: ResNet-18 weight gradients on a second stream (SL_WGRAD_STREAM=1: forked per
# weight gradient once its inputs are ready, joined before the optimizer / each bucket) vs inline:
# engine numerics on the stream form, deterministic-build equality, interleaved A/B.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_wgstream; mkdir -p $O
SL_WGRAD_STREAM=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cnn_gpu.py -k "engine or block" \
  > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  SL_DETERMINISTIC=1 SL_WGRAD_STREAM=$v timeout -k 10 300 python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 > $O/det_s$v.json 2> $O/det_s$v.err || exit 3
  echo "det stream=$v $(grep -o '"train_loss_[a-z]*": [0-9.]*\|"train_acc_last": [0-9.]*' $O/det_s$v.json | tr '\n' ' ')"
done
for rep in 1 2 3; do
  for v in 1 0; do
    SL_WGRAD_STREAM=$v timeout -k 10 300 python bench.py --model resnet18 --ingest device > $O/r_s${v}_$rep.json 2> $O/r_s${v}_$rep.err || exit 4
    echo "stream=$v rep=$rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/r_s${v}_$rep.json | tr '\n' ' ')"
  done
done
