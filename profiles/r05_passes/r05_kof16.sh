# Knockout (numerically wrong, timing only): layer 1 of the rows kernel on exact fp16 pixels
# (1024 + u by one v_perm per two pixels, f16 MFMA) without the row-sum correction.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_kof16
mkdir -p $O
for v in base kof16 base kof16; do
  so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
  SL_KERNELS_SO=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_$v.log 2>&1 || exit 1
  python scripts/rocprof_summary.py $O/prof_$v/run_results.db > $O/kernels_$v.csv; echo "== $v $(grep -o '"train_loss_last": [0-9.a-zN]*' $O/prof_$v.log)"; head -3 $O/kernels_$v.csv | cut -c1-100; rm -rf $O/prof_$v
  SL_KERNELS_SO=$so timeout -k 10 120 python3 scripts/stamps_mlp.py > $O/stamps_$v.txt 2>&1; head -4 $O/stamps_$v.txt
done
