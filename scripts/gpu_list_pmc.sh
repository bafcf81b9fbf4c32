mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || rocprofv3 --list-avail > gpurun_out/counters.txt 2>&1
bash scripts/gpu_pmc.sh 16384
