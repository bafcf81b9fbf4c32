# Fused stride-2 data gradient epilogue: each class's operand loads issued before its LDS staging and
# unconditionally (no wait-count drain between them), HEAD, vs the committed epilogue (variant s2head).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_s2epi}
mkdir -p $O
V=serverless_learn_amd/_native/variants
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_cnn_gpu.py tests/test_resume_gpu.py > $O/pytest_cnn.log 2>&1
rc=$?; tail -2 $O/pytest_cnn.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for v in new s2head; do
    so=""; [ $v != new ] && so=$V/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
for v in new s2head; do
  so=""; [ $v != new ] && so=$V/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --model resnet18 --steps 20 --warmup 5 --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; rm -rf $O/prof_$v
  echo "== $v"; grep "s2_kernel" $O/kernels_$v.csv | cut -c1-130
done
for v in new s2head; do
  so=""; [ $v != new ] && so=$V/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $O/pmc_$v -o run -- python3 bench.py --model resnet18 --steps 4 --warmup 2 --settle 0 > $O/pmc_$v.log 2>&1 || { echo "pmc failed"; exit 1; }
  python scripts/pmc_table.py $(find $O/pmc_$v -name "*counter_collection.csv") --match s2 > $O/pmc_s2e_$v.txt || true
  rm -rf $O/pmc_$v
  echo "== pmc $v"; cat $O/pmc_s2e_$v.txt
done
# HBM bytes per kernel of the ResNet-18 step (read and written in separate runs: one run holds 4 TCC counters)
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/b_$c -o run -- python3 bench.py --model resnet18 --steps 4 --warmup 2 --settle 0 > $O/b_$c.log 2>&1 || { echo "bytes $c failed"; exit 1; }
  python scripts/pmc_table.py $(find $O/b_$c -name "*counter_collection.csv") > $O/bytes_$c.txt || true
  rm -rf $O/b_$c
done
grep -A2 "s2_kernel\|conv3x3_kernel<64, false" $O/bytes_*.txt | head -24
