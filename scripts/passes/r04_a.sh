# Round-4 first GPU pass: driver-form traces (K=20 vs K=200), graph-overhead probe, GRBM clock
# counters around the driver form, the hipBLASLt bar for the MLP GEMM shapes.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_a
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr20 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/tr20.log 2>&1 || { echo tr20 failed; tail -20 $O/tr20.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr200 -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 5 --settle 0 > $O/tr200.log 2>&1 || { echo tr200 failed; exit 1; }
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/plain20.log 2>&1 || exit 1
timeout -k 10 200 python3 scripts/graph_overhead_probe.py > $O/graph_overhead_probe.json 2> $O/graph_overhead_probe.err || exit 1
timeout -k 10 200 python3 scripts/mlp_vs_blas.py > $O/mlp_vs_blas.json 2> $O/mlp_vs_blas.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc20 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/pmc20.log 2>&1 || exit 1
echo r04_a done
