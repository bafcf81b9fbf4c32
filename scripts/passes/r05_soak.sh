# Longer runs for the record: MLP and ResNet-18 engine benches over 1000 / 200 timed steps, the
# runtime-roles MLP path (file server -> gRPC shard -> worker graph chunks) over 2000 steps, and the
# counters of the class-fused stride-2 data gradient.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_soak}
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 1 --steps 1000 --warmup 20 > $O/mlp_1000.log 2>&1 || exit 1
echo "mlp 1000 $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*\|"train_acc_last": [0-9.]*' $O/mlp_1000.log | tr '\n' ' ')"
timeout -k 10 400 python3 bench.py --model resnet18 --gpus 1 --steps 200 --warmup 5 > $O/resnet_200.log 2>&1 || exit 1
echo "resnet 200 $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*\|"train_acc_last": [0-9.]*' $O/resnet_200.log | tr '\n' ' ')"
timeout -k 10 400 python3 bench.py --runtime --gpus 1 --steps 2000 --warmup 20 > $O/runtime_2000.log 2>&1 || exit 1
echo "runtime 2000 $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/runtime_2000.log | tr '\n' ' ')"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $O/pmc -o run -- python3 bench.py --model resnet18 --steps 4 --warmup 2 --settle 0 > $O/pmc.log 2>&1 || { echo "pmc failed"; exit 1; }
python scripts/pmc_table.py $(find $O/pmc -name "*counter_collection.csv") --match s2 > $O/pmc_s2.txt || true
rm -rf $O/pmc
cat $O/pmc_s2.txt
