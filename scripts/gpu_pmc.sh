#!/bin/bash
# PMC counters for the MLP bench kernels (kernel-trace only; no sys/runtime trace with --pmc).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
B=${1:-16384}
bash scripts/gpu_step.sh 400 pmc_sq.log rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/pmc_sq -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --ingest local --batch $B || exit 1
bash scripts/gpu_step.sh 400 pmc_tcc.log rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d gpurun_out/pmc_tcc -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --ingest local --batch $B || exit 1
bash scripts/gpu_step.sh 300 prof65k.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof65k -o run -- python bench.py --steps 30 --warmup 5 --ingest local --batch 65536 --shard-batches 4 || exit 1
