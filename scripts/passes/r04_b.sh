# Round-4 GPU pass b: validate mlp_fwd1 numerics first (short, alone), then the driver-form
# traces of r04_a, then an in-process A/B of layer 1 (fwd1 vs inside the rows kernel), kernel
# stats with fwd1, and the full GPU suite.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_b
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_mlp_fused_gpu.py -k "fwd1 or gradients_match" > $O/pytest_fwd1.log 2>&1
rc=$?; echo "fwd1 tests rc=$rc"; tail -4 $O/pytest_fwd1.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
bash scripts/r04_a.sh || exit 1
if [ $rc -eq 0 ]; then
  timeout -k 10 200 python scripts/ab_mlp_inproc.py --l1 fwd1,none --rounds 6 --steps 50 > $O/ab_fwd1.json 2>&1 || exit 1
  cat $O/ab_fwd1.json | tail -12
  SL_MLP_FWD1=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_fwd1 -o run -- python3 bench.py --steps 50 --warmup 5 --ingest local > $O/prof_fwd1.log 2>&1 || exit 1
  SL_MLP_FWD1=1 timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_fwd1.log 2>&1 || exit 1
  tail -1 $O/bench_fwd1.log | cut -c1-300
fi
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
echo "gpu tests rc=$?"; tail -5 $O/pytest_gpu.log
