# Round-4 GPU pass v: software-pipelined fragment reads in the 256 x 128 conv GEMM (ResNet-18).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_v
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cnn_gpu.py \
  > $O/pytest_cnn.log 2>&1 || { tail -30 $O/pytest_cnn.log; exit 1; }
tail -1 $O/pytest_cnn.log
OLD=$GRAFT_REPO_ROOT/serverless_learn_amd/_native/ab/libslkernels_old.so
rm -f gpurun_out/abenv/summary.txt
bash scripts/ab_env.sh 3 "SL_AB_ARM=pipelined" "SL_KERNELS_SO=$OLD" -- --model resnet18 --ingest device --steps 20 --warmup 5 || exit 1
cp gpurun_out/abenv/summary.txt $O/abenv_summary.txt
for v in new old; do
  if [ $v = new ]; then unset SL_KERNELS_SO; else export SL_KERNELS_SO=$OLD; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --model resnet18 --ingest device --steps 10 --warmup 3 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv
  echo "== $v"; grep -E "conv_gemm_big" $O/kernels_$v.csv | cut -c1-120 || true
  rm -rf $O/prof_$v
done
unset SL_KERNELS_SO
echo r04_v done
