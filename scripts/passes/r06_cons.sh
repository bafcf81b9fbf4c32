#!/bin/bash
# Round 6, pass 10: BN-statistics folds without the 37 fold launches per ResNet step.
# cons2 = workgroup 0 of the consuming kernel folds and raises a write-through flag, the other
# workgroups wait for it (SL_RSUM_CONSUMER=2); cons1 = every consuming workgroup folds (round 5,
# measured -1.6 %).  Conv / engine numerics on cons2, then an interleaved ResNet-18 A/B.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${PASS_TAG:-r06_cons}; mkdir -p $O
V=serverless_learn_amd/_native/variants
SL_KERNELS_SO=$V/libslkernels_cons2.so timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_cnn_gpu.py -k "not deterministic" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in base cons2 cons1; do
    so=""; [ $v != base ] && so=$V/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 300 python bench.py --model resnet18 --ingest device > $O/resnet_${v}_$rep.json 2> $O/resnet_${v}_$rep.err || exit 4
    echo "$v rep=$rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/resnet_${v}_$rep.json | tr '\n' ' ')"
  done
done
SL_KERNELS_SO=$V/libslkernels_cons2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 \
  > $O/prof.log 2>&1 || exit 5
python scripts/kstats.py $O/prof/run_results.db 73 16 > $O/per_step_cons2.txt 2>&1; cat $O/per_step_cons2.txt
rm -rf $O/prof
