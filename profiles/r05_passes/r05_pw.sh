# Direct 3x3 weight gradient: per-tap partial LDS waits inside each k-step (SL_HWG_PW=1, HEAD) vs one
# lgkmcnt(0) before all the k-step's MFMAs (variant pw0).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_pw}
mkdir -p $O
V=serverless_learn_amd/_native/variants
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_cnn_gpu.py tests/test_resume_gpu.py > $O/pytest_cnn.log 2>&1
rc=$?; tail -2 $O/pytest_cnn.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for v in new pw0; do
    so=""; [ $v != new ] && so=$V/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
for v in new pw0; do
  so=""; [ $v != new ] && so=$V/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --model resnet18 --steps 20 --warmup 5 --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; rm -rf $O/prof_$v
  echo "== $v"; grep "wgrad_c64\|s2_kernel" $O/kernels_$v.csv | cut -c1-130
done
for v in new pw0; do
  so=""; [ $v != new ] && so=$V/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $O/pmc_$v -o run -- python3 bench.py --model resnet18 --steps 4 --warmup 2 --settle 0 > $O/pmc_$v.log 2>&1 || { echo "pmc failed"; exit 1; }
  python scripts/pmc_table.py $(find $O/pmc_$v -name "*counter_collection.csv") --match wgrad_c64 > $O/pmc_pw_$v.txt || true
  rm -rf $O/pmc_$v
  echo "== pmc $v"; cat $O/pmc_pw_$v.txt
done
