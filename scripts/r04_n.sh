# Round-4 GPU pass n: the SGD fused behind a grid barrier at the end of the MLP weight gradient.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_n
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mlp_fused_gpu.py \
  > $O/pytest_mlp.log 2>&1 || { tail -30 $O/pytest_mlp.log; exit 1; }
tail -1 $O/pytest_mlp.log
timeout -k 10 300 python scripts/ab_mlp_inproc.py --fuse 1,0 --rounds 8 --steps 50 > $O/ab_fuse.json 2> $O/ab_fuse.err || { tail -20 $O/ab_fuse.err; exit 1; }
python - <<'PY'
import json
d = json.load(open('gpurun_out/r04_n/ab_fuse.json'))
print({k: (round(v['median_us'], 2) if 'median_us' in v else round(v['median'], 4)) for k, v in d.items()})
PY
rm -f gpurun_out/abenv/summary.txt
bash scripts/ab_env.sh 3 "SL_AB_ARM=fused" "SL_MLP_FUSE_SGD=0" -- --gpus 1 --steps 20 --warmup 5 || exit 1
cp gpurun_out/abenv/summary.txt $O/abenv_summary.txt
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof/run_results.db > $O/kernels_mlp.csv
grep -E "mlp_" $O/kernels_mlp.csv | cut -c1-140 || true
rm -rf $O/prof
echo r04_n done
