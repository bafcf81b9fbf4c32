# Round-4 GPU pass k: weight gradient with dW1's 16 tail columns merged into its last tile
# (6 + 2 tile columns, default 32 slices) and the variant removal: full GPU suite, then A/B against
# the 7-tile library (same ABI, built from the previous mlp_fused.hip).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_k
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mlp_fused_gpu.py \
  > $O/pytest_mlp.log 2>&1 || { tail -30 $O/pytest_mlp.log; exit 1; }
tail -1 $O/pytest_mlp.log
OLD=$GRAFT_REPO_ROOT/serverless_learn_amd/_native/ab/libslkernels_7tile.so
rm -f gpurun_out/abenv/summary.txt
bash scripts/ab_env.sh 3 "SL_KERNELS_SO=$OLD" "SL_KERNELS_SO=$OLD SL_MLP_WG_S2=30" "SL_AB_ARM=tail32" "SL_MLP_WG_S1=31 SL_MLP_WG_S2=35" \
  -- --steps 200 --warmup 20 --ingest local || exit 1
cp gpurun_out/abenv/summary.txt $O/abenv_summary.txt
timeout -k 10 400 python scripts/ab_mlp_inproc.py --split 32:32,31:35,30:38,29:41 --rounds 6 --steps 50 \
  > $O/ab_split.json 2> $O/ab_split.err || { tail -20 $O/ab_split.err; exit 1; }
python - <<'PY'
import json
d = json.load(open('gpurun_out/r04_k/ab_split.json'))
print({k: round(v['median_us'], 2) for k, v in d.items() if 'median_us' in v})
PY
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof -o run \
  -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof/run_results.db > $O/kernels_mlp.csv
grep -E "mlp_" $O/kernels_mlp.csv | cut -c1-140 || true
rm -rf $O/prof
timeout -k 10 300 python scripts/ab_mlp_inproc.py --stagger 0,1,3 --rounds 5 --steps 50 > $O/ab_stagger.json 2> $O/ab_stagger.err || exit 1
python - <<'PY'
import json
d = json.load(open('gpurun_out/r04_k/ab_stagger.json'))
print("stagger", {k: round(v['median_us'], 2) for k, v in d.items() if 'median_us' in v})
PY
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu \
  > $O/pytest_gpu.log 2>&1; echo "gpu suite rc=$?"; tail -4 $O/pytest_gpu.log
echo r04_k done
