#!/bin/bash
# A/B of an environment knob on the ResNet-18 bench: gpu_ab_env.sh VAR val1 val2 ...
# (CNN GPU tests first, with the default build), then interleaved reps and kernel stats per value.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/abe
var=$1; shift
for v in "$@"; do env $var=$v bash scripts/gpu_step.sh 400 abe/tests_$v.log python -u -m pytest tests/test_cnn_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1; grep -q "passed" gpurun_out/abe/tests_$v.log && ! grep -q "failed" gpurun_out/abe/tests_$v.log || exit 1; done
for rep in 1 2; do
for v in "$@"; do
  env $var=$v timeout -k 10 150 python bench.py --model resnet18 --ingest device --steps 30 --warmup 5 > gpurun_out/abe/${v}_$rep.log 2>&1 || exit 1
  echo "$var=$v rep=$rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' gpurun_out/abe/${v}_$rep.log | tr '\n' ' ')"
done
done
for v in "$@"; do
  export $var=$v
  bash scripts/gpu_step.sh 200 abe/prof_$v.log rocprofv3 --kernel-trace --stats -d gpurun_out/abe/prof_$v -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 || exit 1
  echo "== $var=$v"; python scripts/rocprof_summary.py gpurun_out/abe/prof_$v/run_results.db | head -12 | cut -c1-70,150-
done
