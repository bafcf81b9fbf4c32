# Round-4 GPU pass r: 256 x 64 large-tile data gradients into 64-channel tensors (ResNet stage 2).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cnn_gpu.py \
  > $O/pytest_cnn.log 2>&1 || { tail -30 $O/pytest_cnn.log; exit 1; }
tail -1 $O/pytest_cnn.log
rm -f gpurun_out/abenv/summary.txt
bash scripts/ab_env.sh 3 "SL_AB_ARM=bn64" "SL_GEMM_BIG=2" -- --model resnet18 --ingest device --steps 20 --warmup 5 || exit 1
cp gpurun_out/abenv/summary.txt $O/abenv_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --model resnet18 --ingest device --steps 10 --warmup 3 > $O/prof.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof/run_results.db > $O/kernels_resnet18.csv
grep -E "conv_gemm" $O/kernels_resnet18.csv | cut -c1-150 || true
rm -rf $O/prof
echo r04_r done
