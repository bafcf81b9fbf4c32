# Round-4 GPU pass p: MLP SGD kernel shape -- 8 threads per float4 unit, or 512-thread workgroups.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_p
mkdir -p $O
AB=$GRAFT_REPO_ROOT/serverless_learn_amd/_native/ab
for v in tpg8 nt512; do
  SL_KERNELS_SO=$AB/libslkernels_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_mlp_fused_gpu.py -k "sgd_step or headline or graph_replay or allreduce_hook" > $O/pytest_$v.log 2>&1 \
    || { tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
rm -f gpurun_out/abenv/summary.txt
bash scripts/ab_env.sh 3 "SL_AB_ARM=base" "SL_KERNELS_SO=$AB/libslkernels_tpg8.so" "SL_KERNELS_SO=$AB/libslkernels_nt512.so" \
  -- --gpus 1 --steps 200 --warmup 20 --ingest local || exit 1
cp gpurun_out/abenv/summary.txt $O/abenv_summary.txt
for v in base tpg8 nt512; do
  if [ $v = base ]; then unset SL_KERNELS_SO; else export SL_KERNELS_SO=$AB/libslkernels_$v.so; fi
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv
  echo "== $v"; grep -E "mlp_" $O/kernels_$v.csv | cut -c1-120 || true
  rm -rf $O/prof_$v
done
echo r04_p done
