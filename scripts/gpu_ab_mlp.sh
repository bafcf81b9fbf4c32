#!/bin/bash
# A/B of kernel-library builds on the MLP step (serverless_learn_amd/_native/variants/libslkernels_<v>.so,
# or "base"): interleaved 200-step bench reps, then rocprofv3 kernel stats per build.
# Knockout builds (wrong numerics) are timed only; run the MLP GPU tests separately for real variants.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/abm
so_of() { [ "$1" = base ] && echo "" || echo serverless_learn_amd/_native/variants/libslkernels_$1.so; }
for rep in 1 2 3; do
for v in "$@"; do
  SL_KERNELS_SO=$(so_of $v) timeout -k 10 150 python bench.py --ingest local > gpurun_out/abm/${v}_$rep.log 2>&1 || exit 1
  echo "$v rep=$rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' gpurun_out/abm/${v}_$rep.log | tr '\n' ' ')"
done
done
for v in "$@"; do
  SL_KERNELS_SO=$(so_of $v) bash scripts/gpu_step.sh 200 abm/prof_$v.log rocprofv3 --kernel-trace --stats -d gpurun_out/abm/prof_$v -o run -- python bench.py --steps 100 --warmup 10 --ingest local || exit 1
done
