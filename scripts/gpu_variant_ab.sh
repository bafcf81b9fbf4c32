#!/bin/bash
# MLP GPU tests under the kernel build $1 (serverless_learn_amd/_native/variants/libslkernels_$1.so),
# then the MLP A/B (scripts/gpu_ab_mlp.sh) of base and that build.
set -u
mkdir -p gpurun_out/abm
SL_KERNELS_SO=serverless_learn_amd/_native/variants/libslkernels_$1.so bash scripts/gpu_step.sh 200 abm/tests_$1.log python -u -m pytest tests/test_mlp_fused_gpu.py tests/test_xgmi_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/abm/tests_$1.log && ! grep -q failed gpurun_out/abm/tests_$1.log || exit 1
bash scripts/gpu_ab_mlp.sh base "$@"
