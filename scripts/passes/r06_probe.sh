#!/bin/bash
# Round 6: the setup-time xGMI exchange probe -- the exchange tests (W = 2, 3, 4, 8, one- and
# two-shot; scripts/xgmi_check.py asserts the probe), the 4-rank bench rehearsal and the elastic
# kill/respawn test, then a 2-rank bench rehearsal that must still pick the exchange.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${PASS_TAG:-r06_probe}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xgmi_gpu.py tests/test_elastic_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 2 --oversubscribe --dist-backend gloo --steps 20 --warmup 5 --ingest local > $O/bench2_mlp.json 2> $O/bench2_mlp.err || exit 4
tail -1 $O/bench2_mlp.json | cut -c1-300
