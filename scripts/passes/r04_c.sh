# Round-4 GPU pass c: fwd1 v2 (software-pipelined chunk, LDS-staged epilogue) numerics + A/B +
# kernel stats; clock-probe timelines of the driver-form bench in the round-3 order and the
# round-4 order (one-time host work ahead of the warm-up tail); full GPU suite.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_c
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_mlp_fused_gpu.py -k "fwd1 or gradients_match" > $O/pytest_fwd1.log 2>&1
rc=$?; echo "fwd1 tests rc=$rc"; tail -3 $O/pytest_fwd1.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for i in 1 2; do
  SL_BENCH_LEGACY_ORDER=1 SL_CLOCK_PROBE=1 timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/probe20_legacy_$i.log 2>&1 || exit 1
  SL_CLOCK_PROBE=1 timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/probe20_new_$i.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_new_$i.log 2>&1 || exit 1
  SL_BENCH_LEGACY_ORDER=1 timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_legacy_$i.log 2>&1 || exit 1
done
grep -ho '"value": [0-9.]*' $O/bench20_*.log
if [ $rc -eq 0 ]; then
  timeout -k 10 200 python scripts/ab_mlp_inproc.py --l1 fwd1,none --rounds 6 --steps 50 > $O/ab_fwd1.json 2>&1 || exit 1
  tail -12 $O/ab_fwd1.json
  SL_MLP_FWD1=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_fwd1 -o run -- python3 bench.py --steps 50 --warmup 5 --ingest local > $O/prof_fwd1.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_fwd1/run_results.db | head -6
fi
bash scripts/r04_d.sh || exit 1
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
echo "gpu tests rc=$?"; tail -5 $O/pytest_gpu.log
