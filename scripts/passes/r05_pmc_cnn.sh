# Counter campaign on the ResNet-18 conv kernels (B = 1024): is the big implicit GEMM bound by
# LDS reads (8 waves of 64 x 64 read as many LDS bytes per k-stage as the MFMAs take cycles)?
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${PASS_TAG:-r05_pmc_cnn}
mkdir -p $O
i=0
for pass in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS" \
            "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE" \
            "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $O/p$i -o run -- python3 bench.py --model resnet18 --steps 4 --warmup 2 --settle 0 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
  python scripts/pmc_table.py $(find $O/p$i -name "*counter_collection.csv") --match ${PMC_MATCH:-conv} > $O/p$i.txt || true
  rm -rf $O/p$i
done
cat $O/p1.txt
