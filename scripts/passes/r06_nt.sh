#!/bin/bash
# Round 6, pass 20: non-temporal (nt) cache policy for the MLP kernels' hand-off stores (H1 / dH2
# rows and slabs: ntw; plus dH1 / w3p: nt) vs the default write-back.  Driver-form MLP bench,
# interleaved, 4 reps; then the GPU-clock step timeline of each (scripts/stamps_graph.py).
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_nt; mkdir -p $O
V=serverless_learn_amd/_native/variants
for rep in 1 2 3 4; do
  for v in base nt ntw; do
    so=""; [ $v != base ] && so=$V/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/m_${v}_$rep.json 2> $O/m_${v}_$rep.err || exit 4
    echo "$v rep=$rep $(grep -o '"value": [0-9.]*\|"settled_samples_per_s": [0-9.]*' $O/m_${v}_$rep.json | tr '\n' ' ')"
  done
done
for v in base nt ntw; do
  so=""; [ $v != base ] && so=$V/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 200 python scripts/stamps_graph.py > $O/stamps_$v.txt 2>&1 || exit 5
  echo "== $v"; grep -i "step\|gap\|span" $O/stamps_$v.txt | head -6
done
