#!/bin/bash
# One-box comparison of bench knobs: graph unroll depth and eager (the multi-GPU launch path).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for cfg in "u8:--unroll 8" "u16:--unroll 16" "eager:--graph off"; do
  tag=${cfg%%:*}; flags=${cfg#*:}
  timeout -k 10 100 python bench.py --ingest local --steps 400 $flags > gpurun_out/knob_${tag}_$rep.log 2>&1 || exit 1
  echo "$tag rep=$rep $(grep -o '"value": [0-9.]*' gpurun_out/knob_${tag}_$rep.log)"
done
done
