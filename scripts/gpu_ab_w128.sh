set -u
for v in w128 w128c; do
bash scripts/gpu_step.sh 300 ${v}_tests.log env SL_KERNELS_SO=serverless_learn_amd/_native/variants/libslkernels_$v.so python -u -m pytest tests/test_mlp_fused_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q passed gpurun_out/${v}_tests.log && ! grep -q failed gpurun_out/${v}_tests.log || { echo "$v tests failed"; exit 1; }
done
bash scripts/gpu_ab1.sh base w128 w128c cvt1 && bash scripts/gpu_ko.sh base w128 w128c
