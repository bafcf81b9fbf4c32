#!/bin/bash
# Round 6, pass 9: conv_gemm_wide_kernel (two 4-wave workgroups per CU, so one's epilogue runs
# beside the other's k-loop) vs conv_gemm_big_kernel at >= 512 tiles (SL_GEMM_WIDE=0):
# conv numerics, interleaved ResNet-18 driver-form A/B, per-shape kernel times.
# WIDE_VALUES / TEST_WIDE: SL_GEMM_WIDE settings compared / tested (2: also 128-row tiles below 512).
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${PASS_TAG:-r06_wide}; mkdir -p $O
SL_GEMM_WIDE=${TEST_WIDE:-1} timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cnn_gpu.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in ${WIDE_VALUES:-1 0}; do
    SL_GEMM_WIDE=$v timeout -k 10 300 python bench.py --model resnet18 --ingest device > $O/resnet_w${v}_$rep.json 2> $O/resnet_w${v}_$rep.err || exit 4
    echo "wide=$v rep=$rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/resnet_w${v}_$rep.json | tr '\n' ' ')"
  done
done
for v in ${WIDE_VALUES:-1 0}; do
  SL_GEMM_WIDE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_w$v -o run -- python bench.py --model resnet18 --ingest device --steps 10 --warmup 3 \
    > $O/prof_w$v.log 2>&1 || exit 5
  python scripts/rocprof_summary.py $O/prof_w$v/run_results.db > $O/kernels_w$v.txt 2>&1 || true
  python3 - $O/prof_w$v/run_results.db <<'PY' | tee $O/shapes_w$v.txt
import sqlite3, sys
db = sqlite3.connect(sys.argv[1])
for r in db.execute("select name, grid_x/workgroup_x, count(*), avg(duration)/1e3 from kernels where name like "
                    "'%conv_gemm_%' group by name, grid_x/workgroup_x order by name, grid_x/workgroup_x"):
    print(f"{r[0][:32]:32s} wgs {r[1]:5d} n {r[2]:4d} avg {r[3]:7.1f}")
PY
  rm -rf $O/prof_w$v
done
