#!/bin/bash
# Round 6: host-requested abort of the xGMI waits (XgmiExchange.abort, called by the worker on a
# broken group) -- the exchange tests (scripts/xgmi_check.py step 4 times the abort), the elastic
# kill/respawn test, then the MLP kill2 scenario, whose survivor regroup time the abort cuts.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${PASS_TAG:-r06_abort}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_xgmi_gpu.py tests/test_elastic_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; grep -h "XGMI_ABORT" $O/pytest.log | head -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 280 python -u scripts/elastic_demo.py --device cuda --dp-backend gloo --model mlp --scenario kill2 --xgmi-gloo \
  --batch 256 --timeout 240 --logdir $O/kill2 > $O/kill2.json 2> $O/kill2.err || { echo "elastic kill2 failed"; tail -3 $O/kill2.err; exit 1; }
echo "elastic mlp kill2: $(tail -1 $O/kill2.json | cut -c1-400)"
