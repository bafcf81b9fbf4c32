#!/bin/bash
# Round 6: the conv GPU tests with the stage-4 lean weight-gradient cases added.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_cnntests; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cnn_gpu.py > $O/pytest.log 2>&1; rc=$?
grep -c PASSED $O/pytest.log; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
