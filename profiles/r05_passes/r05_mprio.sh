# s_setprio 1 around the MFMA clusters of the big implicit GEMM and big weight-gradient k-loops
# (variant mprio, SL_MFMA_PRIO=1) vs main: ResNet-18 driver form x4 interleaved + kernel tables.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_mprio}
V=${V:-mprio}
mkdir -p $O
for rep in 1 2 3 4; do
  for v in new $V; do
    so=""; [ $v != new ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/rn_${v}_$rep.log 2>&1 || exit 1
    echo "resnet $v $rep $(grep -o '"value": [0-9.]*' $O/rn_${v}_$rep.log)"
  done
done
for v in new $V; do
  so=""; [ $v != new ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --model resnet18 --steps 20 --warmup 5 --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; rm -rf $O/prof_$v
  echo "== $v"; head -4 $O/kernels_$v.csv | cut -c1-100
done
