# Round-4 GPU pass h: wide-tile epilogue changes (packed ReLU, dword H1 masks, W3 prefetched before
# the ReLU-2 epilogue) against the previous build (variants/libslkernels_prev.so, plain stores).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_h
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; echo "mlp tests rc=$rc"; grep -E "passed|failed" $O/pytest_mlp.log | tail -2
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python scripts/stamps_mlp.py 65536 128 > $O/stamps_128.txt 2>&1 || exit 1
head -11 $O/stamps_128.txt
timeout -k 10 300 python scripts/ab_mlp_inproc.py --bm 64,128 --rounds 6 --steps 50 > $O/ab_64_128.json 2>&1 || exit 1
grep -A1 '"ratio' $O/ab_64_128.json
PREV=serverless_learn_amd/_native/variants/libslkernels_prev.so
rm -f gpurun_out/abenv/summary.txt
bash scripts/ab_env.sh 4 "SL_AB_ARM=new" "SL_KERNELS_SO=$PREV" -- --steps 200 --warmup 20 --ingest local --settle 0 > /dev/null 2>&1 || exit 1
bash scripts/ab_env.sh 3 "SL_AB_ARM=new" "SL_KERNELS_SO=$PREV" -- --steps 20 --warmup 5 > /dev/null 2>&1 || exit 1
cp gpurun_out/abenv/summary.txt $O/abenv_summary.txt; cat $O/abenv_summary.txt
echo r04_h done
