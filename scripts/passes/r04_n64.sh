# Round-4 GPU pass: 64 x 64 tiles for the 64-column data gradients (SL_GEMM_N64_BM=64) vs the
# default 128 x 64: CNN tests under the knob, interleaved ResNet-18 A/B, kernel tables.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_n64
mkdir -p $O
SL_GEMM_N64_BM=64 timeout -k 10 400 python3 -u -m pytest tests/test_cnn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 1000 scripts/ab_env.sh 3 "SL_GEMM_N64_BM=0" "SL_GEMM_N64_BM=64" -- --model resnet18 --ingest device --steps 60 --warmup 10 || exit 1
cp gpurun_out/abenv/summary.txt $O/abenv_summary.txt
SL_GEMM_N64_BM=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof64 -o run -- python3 bench.py --model resnet18 --ingest device --steps 20 --warmup 5 > $O/prof64.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof64/run_results.db > $O/kernels_bm64.csv; rm -rf $O/prof64
grep -h "conv_gemm_kernel" $O/kernels_bm64.csv | cut -c1-120
echo r04_n64 done
