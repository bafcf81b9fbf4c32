#!/bin/bash
# Round 6, pass 14: where the stage-1 direct 3x3 kernels spend their time now (SL_HALO_KO
# knockouts, results wrong, timing only): 1 no epilogue global traffic, 3 no MFMAs / fragment
# reads, 4 no epilogue.  Per-kernel averages from the ResNet-18 step.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_haloko; mkdir -p $O
for v in base hko1 hko3 hko4; do
  so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 \
    > $O/prof_$v.log 2>&1 || exit 5
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.txt 2>&1 || true
  echo "== $v"; grep "conv3x3" $O/kernels_$v.txt | cut -c1-110
  rm -rf $O/prof_$v
done
