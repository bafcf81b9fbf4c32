#!/bin/bash
# Round 6, pass 23: deferred weight-gradient slab reduces (one multi-slab launch before the
# optimizer instead of one per layer) vs SL_WGRAD_DEFER=0: conv / engine / resume GPU tests,
# deterministic-build equality of the two forms, interleaved ResNet-18 A/B, kernel table.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_defer; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cnn_gpu.py tests/test_resume_gpu.py \
  > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for d in 1 0; do
  SL_DETERMINISTIC=1 SL_WGRAD_DEFER=$d timeout -k 10 300 python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 > $O/det_d$d.json 2> $O/det_d$d.err || exit 3
  echo "det defer=$d $(grep -o '"train_loss_[a-z]*": [0-9.]*\|"train_acc_last": [0-9.]*' $O/det_d$d.json | tr '\n' ' ')"
done
for rep in 1 2 3; do
  for d in 1 0; do
    SL_WGRAD_DEFER=$d timeout -k 10 300 python bench.py --model resnet18 --ingest device > $O/r_d${d}_$rep.json 2> $O/r_d${d}_$rep.err || exit 4
    echo "defer=$d rep=$rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/r_d${d}_$rep.json | tr '\n' ' ')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 > $O/prof.log 2>&1 || exit 5
python scripts/kstats.py $O/prof/run_results.db 73 24 > $O/per_step.txt 2>&1; grep -i "slab\|total" $O/per_step.txt
rm -rf $O/prof
