#!/bin/bash
# Round 6: full validation at HEAD -- smoke(), every GPU test, driver-form benches (MLP x3, ResNet-18 x2),
# 2-rank rehearsals, kernel tables of both models.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${PASS_TAG:-r06_full}; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || exit 2
tail -1 $O/smoke.log
timeout -k 10 1500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
  > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_mlp_$i.json 2> $O/bench_mlp_$i.err || exit 4
  tail -1 $O/bench_mlp_$i.json | cut -c1-220
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet18 --ingest device > $O/bench_resnet_$i.json 2> $O/bench_resnet_$i.err || exit 4
  tail -1 $O/bench_resnet_$i.json | cut -c1-220
done
timeout -k 10 300 python bench.py --gpus 2 --oversubscribe --dist-backend gloo --steps 20 --warmup 5 --ingest local \
  > $O/bench2_mlp.json 2> $O/bench2_mlp.err || exit 4
tail -1 $O/bench2_mlp.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mlp -o run -- python bench.py --steps 100 --warmup 10 --ingest local \
  > $O/prof_mlp.log 2>&1 || exit 5
python scripts/rocprof_summary.py $O/prof_mlp/run_results.db > $O/kernels_mlp.csv 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_resnet -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 \
  > $O/prof_resnet.log 2>&1 || exit 5
python scripts/rocprof_summary.py $O/prof_resnet/run_results.db > $O/kernels_resnet18.csv 2>&1 || true
head -6 $O/kernels_mlp.csv; head -8 $O/kernels_resnet18.csv
