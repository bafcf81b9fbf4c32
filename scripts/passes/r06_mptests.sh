#!/bin/bash
# Round 6, pass 19: the multi-process GPU tests (xGMI ranks on one GPU, elastic respawn, runtime
# roles, RCCL, resume) with the shared-GPU hardware-queue cap, and the 4/8-rank bench rehearsals.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_mptests; mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=15 tests/test_xgmi_gpu.py \
  tests/test_elastic_gpu.py tests/test_runtime_gpu.py tests/test_rccl_gpu.py tests/test_resume_gpu.py > $O/pytest.log 2>&1; rc=$?
tail -25 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
