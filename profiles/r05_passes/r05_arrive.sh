# BN-statistics replicas folded by the producer launch's last-arriving workgroup (SL_RSUM_ARRIVE,
# no rsum_fold launches) vs b0 (separate fold launches): CNN + resume GPU tests (default and
# deterministic builds), ResNet-18 driver-form A/B (B = 1024), kernel tables.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_arrive}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_cnn_gpu.py tests/test_resume_gpu.py > $O/pytest_cnn.log 2>&1
rc=$?; tail -2 $O/pytest_cnn.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in new b0; do
    so=""; [ $v != new ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
for v in new b0; do
  so=""; [ $v != new ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --model resnet18 --steps 20 --warmup 5 --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; echo "== $v"; head -14 $O/kernels_$v.csv | cut -c1-110; rm -rf $O/prof_$v
done
