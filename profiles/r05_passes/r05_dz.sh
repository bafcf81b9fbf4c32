# dH2 recomputed in the weight gradient (dZ rows + ReLU-2 mask bits instead of the dH2 round trip):
# MLP GPU tests, driver-form bench x3, kernel table, HBM bytes.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${PASS_TAG:-r05_dz}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; tail -3 $O/pytest_mlp.log; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_mlp_$i.log 2>&1 || exit 1
done
grep -ho '"value": [0-9.]*\|"settled_samples_per_s": [0-9.]*\|"train_loss_last": [0-9.a-zA-Z]*' $O/bench_mlp_*.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_mlp -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_mlp.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof_mlp/run_results.db > $O/kernels_mlp.csv; head -5 $O/kernels_mlp.csv; rm -rf $O/prof_mlp
for pass in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $O/pmc_$pass -o run -- python3 bench.py --steps 30 --warmup 5 --ingest local --settle 0 > $O/pmc_$pass.log 2>&1 || exit 1
  python scripts/pmc_table.py $(find $O/pmc_$pass -name "*counter_collection.csv") --match mlp_ > $O/pmc_$pass.txt || true
  rm -rf $O/pmc_$pass
done
cat $O/pmc_*.txt
