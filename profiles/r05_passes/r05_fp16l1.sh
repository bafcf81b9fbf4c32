# Layer 1 on exact fp16 pixels (1024 + u, one v_perm per two pixels, f16 MFMA) with the offset
# removed through W1's exact fixed-point row sums: MLP GPU tests, interleaved driver-form A/B
# against the committed kernels (git worktree _old at HEAD), kernel tables, rows-kernel stamps.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_fp16l1}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; tail -3 $O/pytest_mlp.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for v in new old; do
    d=$GRAFT_REPO_ROOT; [ $v = old ] && d=$GRAFT_REPO_ROOT/_old
    (cd $d && timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1) || exit 1
    echo "$v $rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
for v in new old; do
  d=$GRAFT_REPO_ROOT; [ $v = old ] && d=$GRAFT_REPO_ROOT/_old
  (cd $d && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_$v.log 2>&1) || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; echo "== $v $(grep -o '"train_loss_last": [0-9.a-zN]*' $O/prof_$v.log)"; head -4 $O/kernels_$v.csv | cut -c1-100; rm -rf $O/prof_$v
  (cd $d && timeout -k 10 120 python3 scripts/stamps_mlp.py > $O/stamps_$v.txt 2>&1); head -6 $O/stamps_$v.txt
done
