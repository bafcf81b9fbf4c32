# Round-4 GPU pass o: evidence at HEAD -- wgrad slice count, MLP batch sweep and a long settled run,
# ResNet-18 per-kernel HBM traffic and SQ counters (BN-stream roofline claim, profiles/r04_resnet_aux).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_o
mkdir -p $O
timeout -k 10 300 python scripts/ab_mlp_inproc.py --slices 28,24,20,32 --rounds 6 --steps 50 > $O/ab_slices.json 2> $O/ab_slices.err || { tail -20 $O/ab_slices.err; exit 1; }
python - <<'PY'
import json
d = json.load(open('gpurun_out/r04_o/ab_slices.json'))
print("slices", {k: round(v['median_us'], 2) for k, v in d.items() if 'median_us' in v})
PY
for b in 32768 131072 262144; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --batch $b --ingest local > $O/bench_b$b.log 2>&1 || exit 1
  echo "B=$b $(grep -ho '"value": [0-9.]*\|"settled_samples_per_s": [0-9.]*' $O/bench_b$b.log | tr '\n' ' ')"
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 1000 --warmup 50 --ingest local > $O/bench_long.log 2>&1 || exit 1
echo "long $(grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/bench_long.log | tr '\n' ' ')"
timeout -k 10 300 python3 bench.py --model resnet18 --ingest device --batch 2048 > $O/bench_resnet_b2048.log 2>&1 || exit 1
echo "resnet B=2048 $(grep -ho '"value": [0-9.]*' $O/bench_resnet_b2048.log)"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/rfetch -o run -- python3 bench.py --model resnet18 --ingest device --steps 5 --warmup 2 > $O/rfetch.log 2>&1 || exit 1
python scripts/pmc_table.py $(find $O/rfetch -name "*counter_collection.csv") > $O/resnet_fetch.txt || true
rm -rf $O/rfetch
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/rwrite -o run -- python3 bench.py --model resnet18 --ingest device --steps 5 --warmup 2 > $O/rwrite.log 2>&1 || exit 1
python scripts/pmc_table.py $(find $O/rwrite -name "*counter_collection.csv") > $O/resnet_write.txt || true
rm -rf $O/rwrite
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --output-format csv -d $O/rsq -o run -- python3 bench.py --model resnet18 --ingest device --steps 5 --warmup 2 > $O/rsq.log 2>&1 || exit 1
python scripts/pmc_table.py $(find $O/rsq -name "*counter_collection.csv") > $O/resnet_sq.txt || true
rm -rf $O/rsq
echo r04_o done
