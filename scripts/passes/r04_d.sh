# Round-4 GPU pass d: HBM traffic of the MLP step kernels (FETCH_SIZE and WRITE_SIZE, one pass
# each: they do not fit one pass together), default path and the fwd1 path.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_d
mkdir -p $O
for v in base fwd1; do
  [ $v = fwd1 ] && export SL_MLP_FWD1=1 || unset SL_MLP_FWD1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch_$v -o run -- python3 bench.py --steps 30 --warmup 5 --ingest local --settle 0 > $O/fetch_$v.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write_$v -o run -- python3 bench.py --steps 30 --warmup 5 --ingest local --settle 0 > $O/write_$v.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --output-format csv -d $O/sq_$v -o run -- python3 bench.py --steps 30 --warmup 5 --ingest local --settle 0 > $O/sq_$v.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d $O/lds_$v -o run -- python3 bench.py --steps 30 --warmup 5 --ingest local --settle 0 > $O/lds_$v.log 2>&1 || exit 1
done
echo r04_d done
