# MLP rows kernel: bias prologue (b1 + r1p fold, b2) issued after layer 1's first X chunks and weight-ring
# stages, all loads before one wait (SL_ROWS_PRO_LATE=1, HEAD) vs before them (variant pl0): MLP tests,
# stamped graph spans, driver form x4 interleaved, kernel tables.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_prolate}
mkdir -p $O
V=serverless_learn_amd/_native/variants
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; tail -2 $O/pytest_mlp.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3 4; do
  for v in new pl0; do
    so=""; [ $v != new ] && so=$V/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 150 python3 scripts/stamps_graph.py > $O/graph_${v}_$rep.txt 2>&1 || exit 1
    SL_KERNELS_SO=$so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "== $v $rep $(grep -o '"value": [0-9.]*\|"settled_samples_per_s": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
    grep "step (events\|^rows" $O/graph_${v}_$rep.txt | cut -c1-130
  done
done
for v in new pl0; do
  so=""; [ $v != new ] && so=$V/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; rm -rf $O/prof_$v
  echo "== $v"; head -4 $O/kernels_$v.csv | cut -c1-110
done
