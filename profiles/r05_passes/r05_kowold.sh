# The round-4 kernels (git worktree _old at HEAD~): dW1-only / dW2-only weight-gradient times.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05_kowold
mkdir -p $O
cd _old
for v in base kow1 kow2; do
  so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; echo "== $v"; head -4 $O/kernels_$v.csv | cut -c1-100; rm -rf $O/prof_$v
done
