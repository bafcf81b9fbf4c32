# Round-4 GPU pass s: counter campaign at HEAD for the next round's plan -- L2 hit rates, LDS
# bank conflicts and instruction mix per kernel, MLP and ResNet-18 (one rocprofv3 pass per group).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_s
mkdir -p $O
run() {  # tag model-args counters...
  local tag=$1 margs=$2; shift 2
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $O/$tag -o run -- python3 bench.py $margs > $O/$tag.log 2>&1 || return 1
  python scripts/pmc_table.py $(find $O/$tag -name "*counter_collection.csv") > $O/$tag.txt || true
  rm -rf $O/$tag
}
MLP="--steps 30 --warmup 5 --ingest local --settle 0"
RN="--model resnet18 --ingest device --steps 5 --warmup 2"
run mlp_l2 "$MLP" TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit 1
run mlp_lds "$MLP" SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY || exit 1
run mlp_mix "$MLP" SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES || exit 1
run rn_l2 "$RN" TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit 1
run rn_lds "$RN" SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY || exit 1
ls $O
echo r04_s done
