# Consumer-side BN-sum fold with a parallel prologue (every thread issues its <= 16 replica loads at
# once) -- variant cons (SL_RSUM_CONSUMER=1) vs main (fold launches): CNN + resume tests on the
# variant, ResNet-18 driver-form A/B x3, kernel tables.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_cons2}
mkdir -p $O
SL_KERNELS_SO=serverless_learn_amd/_native/variants/libslkernels_cons.so timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_cnn_gpu.py tests/test_resume_gpu.py -k "not deterministic_build and not det" > $O/pytest_cnn.log 2>&1
rc=$?; tail -1 $O/pytest_cnn.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for v in cons main; do
    so=""; [ $v != main ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -o '"value": [0-9.]*' $O/bench_${v}_$rep.log)"
  done
done
for v in cons main; do
  so=""; [ $v != main ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --model resnet18 --steps 20 --warmup 5 --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; rm -rf $O/prof_$v
  echo "== $v"; grep "bn_\|rsum" $O/kernels_$v.csv | cut -c1-40,150-200
done
