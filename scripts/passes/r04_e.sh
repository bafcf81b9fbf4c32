# Round-4 GPU pass e: the 4-wave 128-row rows tile (numerics, determinism, in-process A/B vs 64 / 256,
# phase stamps, kernel stats) and the per-XCD clock probe of the driver-form bench.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_e
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; echo "mlp tests rc=$rc"; grep -E "passed|failed" $O/pytest_mlp.log | tail -3
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/ab_mlp_inproc.py --bm 64,128 --rounds 8 --steps 50 > $O/ab_64_128.json 2>&1 || exit 1
tail -12 $O/ab_64_128.json
timeout -k 10 300 python scripts/ab_mlp_inproc.py --bm 128,256 --rounds 6 --steps 50 > $O/ab_128_256.json 2>&1 || exit 1
for bm in 64 128; do
  timeout -k 10 120 python scripts/stamps_mlp.py 65536 $bm > $O/stamps_$bm.txt 2>&1 || exit 1
done
cat $O/stamps_128.txt
SL_MLP_ROWS_BM=128 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_128 -o run -- python3 bench.py --steps 50 --warmup 5 --ingest local > $O/prof_128.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof_128/run_results.db > $O/prof_128.csv; head -4 $O/prof_128.csv
for i in 1 2; do
  SL_CLOCK_PROBE=1 timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/probe20_$i.log 2>&1 || exit 1
  SL_MLP_ROWS_BM=128 timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_128_$i.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_64_$i.log 2>&1 || exit 1
done
grep -ho '"value": [0-9.]*' $O/bench20_*.log
echo r04_e done
