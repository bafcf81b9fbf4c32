# Driver-form A/B, 5 interleaved runs: base vs variant ${V:-prio1} (MLP GPU tests on the variant first).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
V=${V:-prio1}
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_ab5_$V}
mkdir -p $O
SL_KERNELS_SO=serverless_learn_amd/_native/variants/libslkernels_$V.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; tail -1 $O/pytest_mlp.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3 4 5; do
  for v in base $V; do
    so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -o '"value": [0-9.]*\|"settled_samples_per_s": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
