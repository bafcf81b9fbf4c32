#!/bin/bash
# Round 6: the GPU elastic test twice after dropping the queue cap for elastic workers.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_elastic2; mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_elastic_gpu.py > $O/pytest_$i.log 2>&1 || { tail -5 $O/pytest_$i.log; exit 1; }
  tail -1 $O/pytest_$i.log
done
