# Round-4 GPU pass m: the runtime path after loading torch's reduction kernel at trainer construction.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_m
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mlp_fused_gpu.py tests/test_runtime_gpu.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --runtime --steps 64 --warmup 16 > $O/rt64_$i.log 2>&1 || exit 1
  echo "runtime 64/16 $(grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/rt64_$i.log | tr '\n' ' ')"
done
timeout -k 10 200 python3 bench.py --runtime --steps 256 --warmup 32 > $O/rt256.log 2>&1 || exit 1
echo "runtime 256/32 $(grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/rt256.log | tr '\n' ' ')"
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
echo "driver form $(grep -ho '"value": [0-9.]*' $O/bench.log)"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/rt_prof -o run -- python3 bench.py --runtime --steps 64 --warmup 16 > $O/rt_prof.log 2>&1 || exit 1
f=$(find $O/rt_prof -name "*kernel_trace.csv" | head -1)
python scripts/trace_gaps.py $f --split-us 30 > $O/rt_gaps.txt 2>&1 || true
tail -12 $O/rt_gaps.txt
rm -rf $O/rt_prof
echo r04_m done
