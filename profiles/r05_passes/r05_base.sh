# Round-5 baseline at the round-4 HEAD: driver-form MLP bench x3, MLP kernel table, HBM bytes per kernel.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_base
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_mlp_$i.log 2>&1 || exit 1
done
grep -ho '"value": [0-9.]*\|"settled_samples_per_s": [0-9.]*' $O/bench_mlp_*.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_mlp -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_mlp.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof_mlp/run_results.db > $O/kernels_mlp.csv; head -5 $O/kernels_mlp.csv; rm -rf $O/prof_mlp
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $O/pmc_$tag -o run -- python3 bench.py --steps 30 --warmup 5 --ingest local --settle 0 > $O/pmc_$tag.log 2>&1 || exit 1
  python scripts/pmc_table.py $(find $O/pmc_$tag -name "*counter_collection.csv") --match mlp_ > $O/pmc_$tag.txt || true
  rm -rf $O/pmc_$tag
done
cat $O/pmc_*.txt
echo r05_base done
