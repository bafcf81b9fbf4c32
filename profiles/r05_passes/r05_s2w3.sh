# Fused stride-2 data gradient for >= 128 input channels as 64 x 64 tiles with a 4-slot ring (three
# stages in flight, two workgroups per CU: SL_CONV_S2_WIDE=3) vs 128 x 64 / 3 slots (0).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_s2w3}
mkdir -p $O
for v in 3; do
  SL_CONV_S2_WIDE=$v timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_cnn_gpu.py > $O/pytest_cnn_$v.log 2>&1
  rc=$?; echo "wide=$v $(tail -1 $O/pytest_cnn_$v.log)"; [ $rc -eq 0 ] || exit 1
done
for rep in 1 2 3; do
  for v in 0 3; do
    SL_CONV_S2_WIDE=$v timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "wide=$v $rep $(grep -o '"value": [0-9.]*' $O/bench_${v}_$rep.log)"
  done
done
for v in 0 3; do
  SL_CONV_S2_WIDE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --model resnet18 --steps 20 --warmup 5 --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; rm -rf $O/prof_$v
  echo "== wide=$v"; grep "s2_kernel" $O/kernels_$v.csv | cut -c1-120
done
