#!/bin/bash
# Round 6, final metrics on the shipped tree, in the units the round-5 verdict asks for:
# MLP step timeline (step us, summed inter-launch gaps) and HBM bytes per step; ResNet-18
# per-kernel HBM bytes (FETCH_SIZE, WRITE_SIZE) and MFMA-busy / VALU-per-MFMA counters.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${PASS_TAG:-r06_metrics}; mkdir -p $O
timeout -k 10 120 python scripts/stamps_graph.py > $O/mlp_stamps.txt 2>&1 || exit 3
grep -v amdgpu.ids $O/mlp_stamps.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/mlp_$c -o run \
    -- python3 bench.py --steps 20 --warmup 3 --ingest local --settle 0 > $O/mlp_$c.log 2>&1 || { echo "mlp $c failed"; exit 5; }
  python scripts/pmc_table.py $(find $O/mlp_$c -name "*counter_collection.csv") --match mlp_ > $O/mlp_$c.txt || true
  rm -rf $O/mlp_$c
done
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS" \
            "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $O/cnn_p$i -o run \
    -- python3 bench.py --model resnet18 --ingest device --steps 6 --warmup 2 --settle 0 > $O/cnn_p$i.log 2>&1 || { echo "cnn pass $i failed"; tail -3 $O/cnn_p$i.log; exit 6; }
  python scripts/pmc_table.py $(find $O/cnn_p$i -name "*counter_collection.csv") --match _kernel > $O/cnn_p$i.txt || true
  rm -rf $O/cnn_p$i
done
cp $O/cnn_p3.txt $O/p1.txt && cp $O/cnn_p4.txt $O/p2.txt
python scripts/pmc_summary.py $O 5 > $O/cnn_mfma.txt && cat $O/cnn_mfma.txt
