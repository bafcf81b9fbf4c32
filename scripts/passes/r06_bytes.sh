#!/bin/bash
# Round 6, pass 2: one w3p partial row per rows workgroup + XCD-aligned weight-gradient placement.
# Numerics, interleaved A/B against the committed kernels (variant r05) and the placement knockout,
# per-kernel HBM bytes, GPU-clock timeline.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_bytes; mkdir -p $O
V=serverless_learn_amd/_native/variants
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mlp_fused_gpu.py \
  > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_task.sh ab 3 base,noplace,r05 --steps 20 --warmup 5 || exit 4
bash scripts/gpu_task.sh ab 2 base,r05 --steps 200 --warmup 10 || exit 4
cp -r gpurun_out/ab $O/
for v in base r05; do
  so=""; [ $v = base ] || so=$V/libslkernels_$v.so
  for c in FETCH_SIZE WRITE_SIZE; do
    SL_KERNELS_SO=$so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $O/pmc_${v}_$c -o run \
      --output-format csv -- python bench.py --steps 20 --warmup 3 --ingest local > $O/pmc_${v}_$c.log 2>&1 || exit 5
  done
done
timeout -k 10 120 python scripts/stamps_graph.py > $O/stamps_base.txt 2>&1 || exit 3
SL_KERNELS_SO=$V/libslkernels_r05.so timeout -k 10 120 python scripts/stamps_graph.py > $O/stamps_r05.txt 2>&1 || exit 3
cat $O/stamps_*.txt | grep -v amdgpu.ids
