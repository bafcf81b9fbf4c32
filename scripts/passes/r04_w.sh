# Round-4 GPU pass w: MLP SGD kernel with the db1 row totals summed once per workgroup.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_w
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mlp_fused_gpu.py tests/test_xgmi_gpu.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
OLD=$GRAFT_REPO_ROOT/serverless_learn_amd/_native/ab/libslkernels_old.so
rm -f gpurun_out/abenv/summary.txt
bash scripts/ab_env.sh 4 "SL_AB_ARM=dbrows" "SL_KERNELS_SO=$OLD" -- --gpus 1 --steps 200 --warmup 20 --ingest local || exit 1
cp gpurun_out/abenv/summary.txt $O/abenv_summary.txt
for v in new old; do
  if [ $v = new ]; then unset SL_KERNELS_SO; else export SL_KERNELS_SO=$OLD; fi
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv
  echo "== $v"; grep -E "mlp_" $O/kernels_$v.csv | cut -c1-120 || true
  rm -rf $O/prof_$v
done
unset SL_KERNELS_SO
echo r04_w done
