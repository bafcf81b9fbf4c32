# Round-4 GPU pass y (second run: the BNB template split only; first run: deferred dgrad epilogue):
# and fused BN backward, CIFAR stem): CNN GPU tests, interleaved ResNet-18 A/B against the previous
# build (variant libslkernels_halobase.so), kernel table.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_y
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_cnn_gpu.py tests/test_resume_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
B=serverless_learn_amd/_native/variants/libslkernels_halobase.so
timeout -k 10 900 scripts/ab_env.sh 3 "SL_KERNELS_SO=$B" "SL_AB_ARM=new" -- --model resnet18 --ingest device --steps 60 --warmup 10 || exit 1
cp gpurun_out/abenv/summary.txt $O/abenv_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --model resnet18 --ingest device --steps 40 --warmup 5 > $O/prof.log 2>&1 || exit 1
echo r04_y done
