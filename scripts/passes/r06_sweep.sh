#!/bin/bash
# Round 6, pass 15: batch sweeps of both models on the round-6 kernels (driver form, 1 GPU),
# then the MLP and ResNet-18 counter campaigns (3 PMC passes each, scripts/passes/r05_pmc_cnn.sh
# for ResNet; the same groups for the MLP step).
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_sweep; mkdir -p $O
for b in 256 512 2048 4096; do
  timeout -k 10 300 python bench.py --model resnet18 --ingest device --batch $b > $O/resnet_b$b.json 2> $O/resnet_b$b.err || exit 4
  echo "resnet B=$b $(grep -o '"value": [0-9.]*' $O/resnet_b$b.json)"
done
for b in 16384 32768 131072; do
  timeout -k 10 300 python bench.py --batch $b --steps 20 --warmup 5 > $O/mlp_b$b.json 2> $O/mlp_b$b.err || exit 4
  echo "mlp B=$b $(grep -o '"value": [0-9.]*' $O/mlp_b$b.json)"
done
PASS_TAG=r06_sweep/pmc_resnet PMC_MATCH=_ bash scripts/passes/r05_pmc_cnn.sh > /dev/null 2>&1 || { echo "resnet pmc failed"; exit 5; }
python scripts/pmc_summary.py $O/pmc_resnet | tee $O/pmc_resnet_summary.txt
i=0
for pass in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS" \
            "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $O/pmc_mlp/p$i -o run -- python3 bench.py --steps 20 --warmup 5 --settle 0 --ingest local > $O/pmc_mlp_p$i.log 2>&1 || { echo "mlp pmc pass $i failed"; exit 6; }
  python scripts/pmc_table.py $(find $O/pmc_mlp/p$i -name "*counter_collection.csv") --match mlp > $O/pmc_mlp/p$i.txt || true
  rm -rf $O/pmc_mlp/p$i
done
python scripts/pmc_summary.py $O/pmc_mlp 1 | tee $O/pmc_mlp_summary.txt
