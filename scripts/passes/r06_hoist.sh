#!/bin/bash
# Round 6, pass 24: xGMI update kernel with the first work item's weight / momentum loads issued
# before the peer wait (SL_UPD_HOIST, the prologue otherwise unchanged) vs without (variant
# "nohoist"): exchange fixed cost at W = 1 (scripts/xchg_probe.py), interleaved twice; the
# exchange and MLP tests on the hoisted build.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_hoist; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xgmi_gpu.py tests/test_mlp_fused_gpu.py \
  > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in base nohoist; do
    so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 200 python scripts/xchg_probe.py 200 3 > $O/xchg_${v}_$rep.jsonl 2>&1 || exit 3
    echo "== $v rep=$rep"; grep '"mode"' $O/xchg_${v}_$rep.jsonl | cut -c1-120
  done
done
