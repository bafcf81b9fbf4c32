# Round-4 GPU pass g: write-through (sc1) bulk stores vs plain stores (variant build), the
# reverted bf16 wide layer 1, kernel stats of both store policies.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_g
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; echo "mlp tests rc=$rc"; grep -E "passed|failed" $O/pytest_mlp.log | tail -2
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/ab_mlp_inproc.py --bm 64,128 --rounds 6 --steps 50 > $O/ab_64_128.json 2>&1 || exit 1
grep -A1 '"ratio' $O/ab_64_128.json
PLAIN=serverless_learn_amd/_native/variants/libslkernels_plain.so
bash scripts/ab_env.sh 4 "SL_AB_ARM=sc1" "SL_KERNELS_SO=$PLAIN" -- --steps 200 --warmup 20 --ingest local --settle 0 > $O/ab_store_200.txt 2>&1 || exit 1
bash scripts/ab_env.sh 3 "SL_AB_ARM=sc1" "SL_KERNELS_SO=$PLAIN" -- --steps 20 --warmup 5 > $O/ab_store_20.txt 2>&1 || exit 1
cat gpurun_out/abenv/summary.txt; cp gpurun_out/abenv/summary.txt $O/abenv_summary.txt
for v in sc1 plain; do
  [ $v = plain ] && export SL_KERNELS_SO=$PLAIN || unset SL_KERNELS_SO
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 50 --warmup 5 --ingest local --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/prof_$v.csv; head -4 $O/prof_$v.csv
  python scripts/trace_gaps.py $O/prof_$v/run_results.db --split-us 300 --min-kernels 100 > $O/gaps_$v.txt 2>&1 || true
done
unset SL_KERNELS_SO
echo r04_g done
