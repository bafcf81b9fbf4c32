# Round-4 GPU pass z: BN streaming kernels (bn_apply_stats, bn_bwd_apply_sums, bn_bwd_apply_dual)
# with SL_BN_U chunks of loads in flight per thread: CNN tests on the in-tree build (U = 4),
# interleaved ResNet-18 A/B of U = 1 (the previous form) / 2 / 4, kernel table.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_z
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_cnn_gpu.py tests/test_resume_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
V=serverless_learn_amd/_native/variants
timeout -k 10 1000 scripts/ab_env.sh 3 "SL_KERNELS_SO=$V/libslkernels_bnu1.so" "SL_KERNELS_SO=$V/libslkernels_bnu2.so" "SL_AB_ARM=u4" -- --model resnet18 --ingest device --steps 60 --warmup 10 || exit 1
cp gpurun_out/abenv/summary.txt $O/abenv_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --model resnet18 --ingest device --steps 40 --warmup 5 > $O/prof.log 2>&1 || exit 1
SL_KERNELS_SO=$V/libslkernels_bnu1.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_u1 -o run -- python3 bench.py --model resnet18 --ingest device --steps 40 --warmup 5 > $O/prof_u1.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof/run_results.db > $O/kernels_u4.csv; python scripts/rocprof_summary.py $O/prof_u1/run_results.db > $O/kernels_u1.csv
grep -h "bn_" $O/kernels_u4.csv $O/kernels_u1.csv | cut -c1-40,150-
rm -rf $O/prof $O/prof_u1
echo r04_z done
