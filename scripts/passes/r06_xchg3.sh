#!/bin/bash
# Round 6, pass 3c: xGMI inline synchronisation, second form (consumer-prologue signal, step id
# advanced by the rows kernel).  Multi-rank bit-exactness, elastic respawn, fixed cost at W = 1.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_xchg3; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xgmi_gpu.py \
  tests/test_mlp_fused_gpu.py tests/test_rccl_gpu.py tests/test_elastic_gpu.py > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/xchg_probe.py 200 3 > $O/xchg.jsonl 2>&1 || exit 3
cat $O/xchg.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python scripts/xchg_probe.py 50 1 > $O/prof.log 2>&1 || exit 5
python scripts/rocprof_summary.py $O/prof/run_results.db > $O/kernels.txt 2>&1 || true
head -12 $O/kernels.txt
