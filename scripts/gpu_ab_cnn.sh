#!/bin/bash
# A/B of kernel-library variants on the ResNet-18 bench (one box, two interleaved reps) + kernel stats.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_step.sh 400 abc_tests.log python -u -m pytest tests/test_cnn_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/abc_tests.log && ! grep -q "failed" gpurun_out/abc_tests.log || exit 1
for rep in 1 2; do
for v in "$@"; do
  so=""; [ "$v" != "base" ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 150 python bench.py --model resnet18 --ingest device --steps 30 --warmup 5 > gpurun_out/abc_${v}_$rep.log 2>&1 || exit 1
  echo "$v rep=$rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' gpurun_out/abc_${v}_$rep.log | tr '\n' ' ')"
done
done
for v in "$@"; do
  so=""; [ "$v" != "base" ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so bash scripts/gpu_step.sh 200 koc_$v.log rocprofv3 --kernel-trace --stats -d gpurun_out/koc_$v -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 || exit 1
  echo "== $v"; python scripts/rocprof_summary.py gpurun_out/koc_$v/run_results.db | head -8 | cut -c1-60,150-
done
