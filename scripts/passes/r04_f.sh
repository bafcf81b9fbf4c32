# Round-4 GPU pass f: fp16-exact layer 1 in the wide rows tiles (numerics, stamps, kernel stats,
# driver-form bench), then the full GPU suite.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_f
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; echo "mlp tests rc=$rc"; grep -E "passed|failed|Error|assert" $O/pytest_mlp.log | tail -8
[ $rc -eq 0 ] || exit 1
for bm in 128 256; do
  timeout -k 10 120 python scripts/stamps_mlp.py 65536 $bm > $O/stamps_$bm.txt 2>&1 || exit 1
done
head -12 $O/stamps_128.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 50 --warmup 5 --ingest local > $O/prof.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof/run_results.db > $O/prof.csv; head -4 $O/prof.csv
timeout -k 10 300 python scripts/ab_mlp_inproc.py --bm 64,128 --rounds 6 --steps 50 > $O/ab_64_128.json 2>&1 || exit 1
grep -A2 ratio $O/ab_64_128.json
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_$i.log 2>&1 || exit 1
done
grep -ho '"value": [0-9.]*' $O/bench20_*.log
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
echo "gpu tests rc=$?"; tail -3 $O/pytest_gpu.log
