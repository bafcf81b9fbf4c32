#!/bin/bash
# Round 6, pass 1: fused weight-gradient + SGD launch -- numerics, GPU-clock timeline, A/B.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_fuse
O=gpurun_out/r06_fuse
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mlp_fused_gpu.py \
  > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/stamps_graph.py > $O/stamps_fused.txt 2>&1 || exit 3
SL_MLP_FUSE_SGD=0 timeout -k 10 120 python scripts/stamps_graph.py > $O/stamps_sep.txt 2>&1 || exit 3
cat $O/stamps_fused.txt $O/stamps_sep.txt
bash scripts/ab_env.sh 3 "SL_MLP_FUSE_SGD=1" "SL_MLP_FUSE_SGD=0" -- --steps 20 --warmup 5 || exit 4
bash scripts/ab_env.sh 2 "SL_MLP_FUSE_SGD=1" "SL_MLP_FUSE_SGD=0" -- --steps 200 --warmup 10 || exit 4
cp -r gpurun_out/abenv $O/
