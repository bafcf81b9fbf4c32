# dW1 tiles on a 4-slot LDS-DMA ring (3 stages in flight): MLP GPU tests, interleaved driver-form
# A/B against the 3-slot build (variant r3 = round-4 kernels), kernel tables, per-workgroup stamps.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${PASS_TAG:-r05_ring4}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; tail -2 $O/pytest_mlp.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for v in base r3; do
    so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
for v in base r3; do
  so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; echo "== $v"; head -4 $O/kernels_$v.csv | cut -c1-100; rm -rf $O/prof_$v
done
timeout -k 10 120 python3 scripts/stamps_wgrad.py > $O/stamps_wgrad.txt 2>&1; cat $O/stamps_wgrad.txt
