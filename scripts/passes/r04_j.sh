# Round-4 GPU pass j: per-problem split-K of the MLP weight gradient (dW1 : dW2 slices).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_j
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_fused_gpu.py \
  -k "split_k or headline or deterministic" > $O/pytest_split.log 2>&1 || { tail -30 $O/pytest_split.log; exit 1; }
tail -2 $O/pytest_split.log
timeout -k 10 500 python scripts/ab_mlp_inproc.py --split 28:28,28:30,27:32,26:37,24:42 --rounds 6 --steps 50 \
  > $O/ab_split.json 2> $O/ab_split.err || { tail -20 $O/ab_split.err; exit 1; }
python - <<'PY'
import json
d = json.load(open('gpurun_out/r04_j/ab_split.json'))
print({k: round(v['median_us'], 2) for k, v in d.items() if 'median_us' in v})
PY
for arm in 28:28 27:32 26:37; do
  s1=${arm%:*}; s2=${arm#*:}
  SL_MLP_WG_S1=$s1 SL_MLP_WG_S2=$s2 timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof_${s1}_${s2} -o run \
    -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/bench_${s1}_${s2}.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_${s1}_${s2}/run_results.db > $O/kernels_${s1}_${s2}.csv
  echo "== $arm"; grep -E "mlp_" $O/kernels_${s1}_${s2}.csv | cut -c1-140 || true
  rm -rf $O/prof_${s1}_${s2}
done
timeout -k 10 300 python scripts/ab_mlp_inproc.py --stagger 0,1,3 --rounds 5 --steps 50 > $O/ab_stagger.json 2> $O/ab_stagger.err || exit 1
python - <<'PY'
import json
d = json.load(open('gpurun_out/r04_j/ab_stagger.json'))
print("stagger", {k: round(v['median_us'], 2) for k, v in d.items() if 'median_us' in v})
PY
echo r04_j done
