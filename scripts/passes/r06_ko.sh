#!/bin/bash
# Round 6, pass 8: what bounds the big implicit-GEMM conv?  Kernel tables of the ResNet-18 step
# with the GEMM's DMA knocked out (ko1: none after the prologue; ko2: every stage re-reads
# stage 0, L2-hot; ko3: no epilogue; ko4: neither) vs the real kernel (results of the knockouts are wrong; timing only).
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_ko; mkdir -p $O
for v in ${KO_VARIANTS:-base ko1 ko2}; do
  so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 \
    > $O/prof_$v.log 2>&1 || exit 5
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.txt 2>&1 || true
  echo "== $v"; grep conv_gemm_big $O/kernels_$v.txt | cut -c1-120
  python3 - $O/prof_$v/run_results.db <<'PY' | tee $O/shapes_$v.txt
import sqlite3, sys
db = sqlite3.connect(sys.argv[1])
for r in db.execute("select name, grid_x/workgroup_x, count(*), avg(duration)/1e3 from kernels where name like "
                    "'%conv_gemm_big%' group by name, grid_x/workgroup_x order by name, grid_x/workgroup_x"):
    print(f"{r[0][:32]:32s} wgs {r[1]:5d} n {r[2]:4d} avg {r[3]:7.1f}")
PY
  rm -rf $O/prof_$v
done
