# Rows-kernel epilogue VALU cuts (ReLU-1 mask by v_med3_i32 + v_lshl_or, packed fma, dH2 mask by
# packed u16 min/sub + and) vs b1 (previous build): MLP GPU tests, stamps, driver form x5.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_valu}
B=${BASEV:-b1}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; tail -1 $O/pytest_mlp.log; [ $rc -eq 0 ] || exit 1
for v in new $B; do
  so=""; [ $v != new ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 120 python3 scripts/stamps_mlp.py > $O/stamps_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -A10 "CU pairs" $O/stamps_$v.txt; grep "WG total" $O/stamps_$v.txt
done
for rep in 1 2 3 4 5; do
  for v in new $B; do
    so=""; [ $v != new ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -o '"value": [0-9.]*\|"settled_samples_per_s": [0-9.]*\|"train_loss_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
