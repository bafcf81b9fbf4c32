# Stride-2 fused dgrad tile variants re-measured after the LDS-layout and epilogue fixes: 128 x 64 / 3 slots
# (SL_CONV_S2_WIDE=0, default) vs 64 x 128 / 2 slots for the 128- and 256-channel stages (2).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_s2w2}
mkdir -p $O
for rep in 1 2 3; do
  for v in 0 2; do
    SL_CONV_S2_WIDE=$v timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "wide=$v $rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
for v in 0 2; do
  SL_CONV_S2_WIDE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --model resnet18 --steps 20 --warmup 5 --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; rm -rf $O/prof_$v
  echo "== wide=$v"; grep "s2_kernel" $O/kernels_$v.csv | cut -c1-130
done
