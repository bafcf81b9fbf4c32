# Round-4 GPU pass t: XOR-swizzled H1 nibble masks in the MLP rows kernel (LDS bank conflicts).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_t
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mlp_fused_gpu.py \
  > $O/pytest_mlp.log 2>&1 || { tail -30 $O/pytest_mlp.log; exit 1; }
tail -1 $O/pytest_mlp.log
OLD=$GRAFT_REPO_ROOT/serverless_learn_amd/_native/ab/libslkernels_old.so
rm -f gpurun_out/abenv/summary.txt
bash scripts/ab_env.sh 4 "SL_AB_ARM=swizzled" "SL_KERNELS_SO=$OLD" -- --gpus 1 --steps 200 --warmup 20 --ingest local || exit 1
cp gpurun_out/abenv/summary.txt $O/abenv_summary.txt
for v in new old; do
  if [ $v = new ]; then unset SL_KERNELS_SO; else export SL_KERNELS_SO=$OLD; fi
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d $O/lds_$v -o run -- python3 bench.py --steps 30 --warmup 5 --ingest local --settle 0 > $O/lds_$v.log 2>&1 || exit 1
  python scripts/pmc_table.py $(find $O/lds_$v -name "*counter_collection.csv") --match mlp_rows > $O/lds_$v.txt || true
  rm -rf $O/lds_$v
  echo "== $v"; cat $O/lds_$v.txt
done
unset SL_KERNELS_SO
echo r04_t done
