#!/bin/bash
# Kernel-time A/B of variant builds: rocprofv3 kernel stats of a short bench per variant.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  so=""; [ "$v" != "base" ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so bash scripts/gpu_step.sh 120 ko_$v.log rocprofv3 --kernel-trace --stats -d gpurun_out/ko_$v -o run -- python bench.py --steps 40 --warmup 8 --ingest local || exit 1
  echo "== $v"; python scripts/rocprof_summary.py gpurun_out/ko_$v/run_results.db | head -6
done
