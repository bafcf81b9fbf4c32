# Which tiles bound the weight gradient: kow1 = dW1 tiles return at once, kow2 = dW2 tiles return at once.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_kow
mkdir -p $O
for v in base kow1 kow2; do
  so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; echo "== $v"; head -4 $O/kernels_$v.csv | cut -c1-100; rm -rf $O/prof_$v
done
