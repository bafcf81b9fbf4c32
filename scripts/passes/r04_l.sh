# Round-4 GPU pass l: where the runtime path (bench.py --runtime, worker thread replaying graph
# chunks) loses against the bare engine: kernel trace gaps, host spans, chunk length.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_l
mkdir -p $O
for gs in 16 64 16 64; do
  timeout -k 10 200 python3 bench.py --runtime --steps 256 --warmup 32 --graph-steps $gs > $O/rt_gs$gs.log 2>&1 || exit 1
  echo "gs=$gs $(grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/rt_gs$gs.log | tr '\n' ' ')"
done
timeout -k 10 200 python3 bench.py --runtime --steps 64 --warmup 16 > $O/rt_64.log 2>&1 || exit 1
echo "driver-like runtime $(grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/rt_64.log | tr '\n' ' ')"
SL_TRACE=$O/rt_trace.json timeout -k 10 200 python3 bench.py --runtime --steps 256 --warmup 32 > $O/rt_trace.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/rt_prof -o run -- python3 bench.py --runtime --steps 256 --warmup 32 > $O/rt_prof.log 2>&1 || exit 1
f=$(find $O/rt_prof -name "*kernel_trace.csv" | head -1)
python scripts/trace_gaps.py $f --split-us 30 > $O/rt_gaps.txt 2>&1 || true
head -40 $O/rt_gaps.txt
cp $f $O/rt_kernel_trace.csv; rm -rf $O/rt_prof
echo r04_l done
