#!/bin/bash
# Knockout timing: rocprof kernel stats of the MLP bench for each variant build.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  so=""; [ "$v" != "base" ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  rm -rf gpurun_out/kn_$v
  SL_KERNELS_SO=$so timeout -k 10 100 rocprofv3 --kernel-trace --stats -d gpurun_out/kn_$v -o run -- python bench.py --ingest local --steps 50 --warmup 5 > gpurun_out/kn_$v.log 2>&1 || exit 1
  echo "== $v"; python scripts/rocprof_summary.py gpurun_out/kn_$v/run_results.db | grep mlp_ | cut -d, -f1,4 
done
