# Round-4 validation at HEAD (last full pass): full GPU suite, driver-form MLP bench (x3), ResNet-18 bench,
# gloo rehearsals (MLP xGMI + ResNet), rocprofv3 kernel tables of both models, smoke().
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_final6
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_mlp_$i.log 2>&1 || exit 1
done
grep -ho '"value": [0-9.]*\|"settled_samples_per_s": [0-9.]*' $O/bench_mlp_*.log
timeout -k 10 300 python3 bench.py --model resnet18 --ingest device > $O/bench_resnet.log 2>&1 || exit 1
grep -ho '"value": [0-9.]*' $O/bench_resnet.log
timeout -k 10 300 python3 bench.py --gpus 2 --oversubscribe --dist-backend gloo --steps 20 --warmup 5 --ingest local > $O/bench2_mlp.log 2>&1 || exit 1
grep -ho '"value": [0-9.]*\|"replicas_identical": [a-z]*\|"collective_backend": "[a-z-]*"' $O/bench2_mlp.log | head -3
timeout -k 10 300 python3 bench.py --gpus 2 --oversubscribe --dist-backend gloo --model resnet18 --batch 256 --steps 5 --warmup 2 --ingest device > $O/bench2_resnet.log 2>&1 || exit 1
grep -ho '"value": [0-9.]*\|"replicas_identical": [a-z]*' $O/bench2_resnet.log | head -2
timeout -k 10 300 python3 bench.py --runtime --steps 64 --warmup 16 > $O/bench_runtime.log 2>&1 || exit 1
grep -ho '"value": [0-9.]*' $O/bench_runtime.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_mlp -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_mlp.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof_mlp/run_results.db > $O/kernels_mlp.csv; head -4 $O/kernels_mlp.csv; rm -rf $O/prof_mlp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_resnet -o run -- python3 bench.py --model resnet18 --ingest device --steps 10 --warmup 3 > $O/prof_resnet.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof_resnet/run_results.db > $O/kernels_resnet18.csv; head -6 $O/kernels_resnet18.csv; rm -rf $O/prof_resnet
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $O/pmc_$tag -o run -- python3 bench.py --steps 30 --warmup 5 --ingest local --settle 0 > $O/pmc_$tag.log 2>&1 || exit 1
  python scripts/pmc_table.py $(find $O/pmc_$tag -name "*counter_collection.csv") --match mlp_ > $O/pmc_$tag.txt || true
  rm -rf $O/pmc_$tag
done
echo r04_final6 done
