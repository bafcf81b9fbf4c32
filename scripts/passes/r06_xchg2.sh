#!/bin/bash
# Round 6, pass 3b: elastic respawn with the xGMI exchange (after the probe fix), the exchange's
# fixed cost at W = 1 (inline vs barrier protocol) and its kernel table.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_xchg; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_elastic_gpu.py \
  > $O/pytest_elastic.log 2>&1; rc=$?; tail -3 $O/pytest_elastic.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/xchg_probe.py 200 3 > $O/xchg.jsonl 2>&1 || exit 3
cat $O/xchg.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python scripts/xchg_probe.py 50 1 > $O/prof.log 2>&1 || exit 5
python scripts/rocprof_summary.py $O/prof/run_results.db > $O/kernels.txt 2>&1 || true
head -20 $O/kernels.txt
