#!/bin/bash
# PMC passes for the MLP bench kernels incl. LDS conflicts (one counter group per run).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
B=${1:-65536}
run() {  # name counters...
  local name=$1; shift
  bash scripts/gpu_step.sh 120 pmc_$name.log timeout -s KILL 100 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc_$name -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --ingest local --batch $B || exit 1
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_BUSY_CYCLES
run lds SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_WR
run fetch FETCH_SIZE GRBM_GUI_ACTIVE
