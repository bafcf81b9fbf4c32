#!/bin/bash
# Round 6, pass 3: xGMI exchange with inline synchronisation (no barrier kernel) and the update
# kernel with fused W1 row sums.  Multi-rank bit-exactness on the one GPU (W = 2, 3, 4, 8; one-
# and two-shot), elastic respawn, then the fixed cost at W = 1 against the barrier protocol.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06_xchg; mkdir -p $O
# ResNet numerics in the shipped build: per-block at B = 1024, whole engine at 256
timeout -k 10 280 python scripts/resnet_block_check.py 1024 > $O/resnet_block_1024.json 2> $O/resnet_block.err || exit 6
timeout -k 10 280 python scripts/resnet_engine_check.py 256 > $O/resnet_engine_256.json 2> $O/resnet_engine.err || exit 6
python - <<'PY'
import json
for f in ("resnet_block_1024", "resnet_engine_256"):
    r = json.loads(open(f"gpurun_out/r06_xchg/{f}.json").read().strip().splitlines()[-1])
    print(f, {k: v for k, v in r.items() if k not in ("errors", "layers")})
PY
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xgmi_gpu.py \
  tests/test_mlp_fused_gpu.py tests/test_rccl_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_elastic_gpu.py \
  > $O/pytest_elastic.log 2>&1; rc=$?; tail -3 $O/pytest_elastic.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/xchg_probe.py 200 3 > $O/xchg.jsonl 2>&1 || exit 3
cat $O/xchg.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python scripts/xchg_probe.py 50 1 > $O/prof.log 2>&1 || exit 5
python scripts/rocprof_summary.py $O/prof/run_results.db > $O/kernels.txt 2>&1 || true
head -20 $O/kernels.txt
