# Write-through (sc1) stores for every output handed to the next launch (rows kernel H1/dH2/dH1 +
# w3p partials, weight-gradient slabs): variant sc1 (-DSL_STORE_AUX=16) against the default
# write-back stores. MLP tests on the variant, interleaved driver-form A/B, kernel tables, stamps.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_sc1}
V=${VARIANT:-sc1}
mkdir -p $O
SL_KERNELS_SO=serverless_learn_amd/_native/variants/libslkernels_$V.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; tail -2 $O/pytest_mlp.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for v in base $V; do
    so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
for v in base $V; do
  so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; echo "== $v"; head -4 $O/kernels_$v.csv | cut -c1-100; rm -rf $O/prof_$v
  SL_KERNELS_SO=$so timeout -k 10 120 python3 scripts/stamps_mlp.py > $O/stamps_$v.txt 2>&1 && grep "clock\|spread\|total cycles" $O/stamps_$v.txt
  SL_KERNELS_SO=$so timeout -k 10 120 python3 scripts/stamps_wgrad.py > $O/stampsw_$v.txt 2>&1 && tail -1 $O/stampsw_$v.txt
done
