# Knockouts (numerically wrong builds, timing only): koa = no dH2 operand DMA in the dW2 tiles,
# kob = no dH2 stores in the rows kernel, koab = both.  Kernel tables + interleaved driver-form A/B.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_ko1
mkdir -p $O
for v in base koa kob koab; do
  so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; echo "== $v"; head -4 $O/kernels_$v.csv | cut -c1-120; rm -rf $O/prof_$v
done
for rep in 1 2 3; do
  for v in base koab; do
    so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -o '"value": [0-9.]*' $O/bench_${v}_$rep.log)"
  done
done
