#!/bin/bash
# Round 6, pass 17: the 128-wide weight-gradient kernel's ring / wave shape re-swept on the lean
# form: base (2 slots, 4 waves, two per CU), w3s (3 slots, one per CU), wks2 (8 waves splitting
# each stage's k in two, 4 slots).  Interleaved ResNet-18 + kernel table per variant.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_wg128; mkdir -p $O
V=serverless_learn_amd/_native/variants
for rep in 1 2; do
  for v in base w3s wks2; do
    so=""; [ $v != base ] && so=$V/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 300 python bench.py --model resnet18 --ingest device > $O/r_${v}_$rep.json 2> $O/r_${v}_$rep.err || exit 4
    echo "$v rep=$rep $(grep -o '"value": [0-9.]*' $O/r_${v}_$rep.json)"
  done
done
for v in base w3s wks2; do
  so=""; [ $v != base ] && so=$V/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 > $O/prof_$v.log 2>&1 || exit 5
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.txt 2>&1 || true
  echo "== $v"; grep "conv_wgrad_kernel<128" $O/kernels_$v.txt | cut -c1-120
  rm -rf $O/prof_$v
done
