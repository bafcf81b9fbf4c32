#!/bin/bash
# PMC passes for the ResNet-18 bench kernels (one counter group per run).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name counters...
  local name=$1; shift
  bash scripts/gpu_step.sh 120 pmcc_$name.log timeout -s KILL 100 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmcc_$name -o run --output-format csv -- python bench.py --model resnet18 --ingest device --steps 4 --warmup 2 || exit 1
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_BUSY_CYCLES
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE
run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE
for f in gpurun_out/pmcc_*/run_counter_collection.csv; do echo $f; done
python scripts/pmc_table.py gpurun_out/pmcc_*/run_counter_collection.csv --match conv > gpurun_out/pmc_cnn_table.txt
cat gpurun_out/pmc_cnn_table.txt
