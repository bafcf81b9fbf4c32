# The round-5 GPU tests that are new (xGMI W = 4 / 8, 4-rank bench rehearsal, per-block ResNet
# numerics at B = 256 / 1024), then the counter list of this rocprofv3.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xgmi_gpu.py \
  "tests/test_cnn_gpu.py::test_resnet_block_backward_at_bench_batch_deterministic_build" \
  "tests/test_cnn_gpu.py::test_resnet_block_backward_local" > $O/pytest_new.log 2>&1
rc=$?; tail -15 $O/pytest_new.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -c "" $O/counters.txt
