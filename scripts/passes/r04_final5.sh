# Round-4 validation at HEAD after the direct-3x3 instance split and the multi-tile conv test cases:
# full GPU suite, smoke(), driver-form MLP bench (x3), ResNet-18 bench, ResNet kernel table.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_final5
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
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_resnet -o run -- python3 bench.py --model resnet18 --ingest device --steps 10 --warmup 3 > $O/prof_resnet.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof_resnet/run_results.db > $O/kernels_resnet18.csv; head -6 $O/kernels_resnet18.csv; rm -rf $O/prof_resnet
echo r04_final5 done
