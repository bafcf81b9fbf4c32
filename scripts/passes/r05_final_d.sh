# Round-5 final validation (reusable): full GPU suite, smoke, driver-form benches (MLP x5, ResNet-18 x3),
# kernel tables, batch sweeps, the 8-rank same-GPU rehearsal, a 1000-step MLP run and per-kernel HBM
# bytes of the ResNet-18 step (FETCH_SIZE and WRITE_SIZE in separate runs: one run holds 4 TCC counters).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_final_d}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
for rep in 1 2 3 4 5; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_mlp_$rep.log 2>&1 || exit 1
  echo "mlp $rep $(grep -o '"value": [0-9.]*\|"settled_samples_per_s": [0-9.]*' $O/bench_mlp_$rep.log | tr '\n' ' ')"
done
for rep in 1 2 3; do
  timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/bench_resnet_$rep.log 2>&1 || exit 1
  echo "resnet $rep $(grep -o '"value": [0-9.]*' $O/bench_resnet_$rep.log | tr '\n' ' ')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mlp -o run -- python3 bench.py --steps 100 --warmup 10 --ingest local --settle 0 > $O/prof_mlp.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof_mlp/run_results.db > $O/kernels_mlp.csv; rm -rf $O/prof_mlp; head -4 $O/kernels_mlp.csv | cut -c1-100
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_resnet -o run -- python3 bench.py --model resnet18 --steps 20 --warmup 5 --settle 0 > $O/prof_resnet.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof_resnet/run_results.db > $O/kernels_resnet18.csv; rm -rf $O/prof_resnet; head -4 $O/kernels_resnet18.csv | cut -c1-100
for b in 16384 32768 65536 131072 262144; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --batch $b --ingest local > $O/sweep_mlp_$b.log 2>&1 || exit 1
  echo "mlp B=$b $(grep -o '"value": [0-9.]*\|"settled_samples_per_s": [0-9.]*' $O/sweep_mlp_$b.log | tr '\n' ' ')"
done
for b in 256 512 2048; do
  timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 --batch $b > $O/sweep_resnet_$b.log 2>&1 || exit 1
  echo "resnet B=$b $(grep -o '"value": [0-9.]*' $O/sweep_resnet_$b.log | tr '\n' ' ')"
done
timeout -k 10 400 python3 bench.py --gpus 8 --oversubscribe --dist-backend gloo --batch 4096 --steps 8 --warmup 3 --ingest local > $O/rehearsal_8rank.log 2>&1 || exit 1
echo "8-rank $(grep -o '"replicas_identical": [a-z]*\|"allreduce[a-z_]*": "[a-z0-9]*"\|"value": [0-9.]*' $O/rehearsal_8rank.log | tr '\n' ' ')"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 1000 --warmup 20 > $O/mlp_1000.log 2>&1 || exit 1
echo "mlp 1000 $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/mlp_1000.log | tr '\n' ' ')"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/b_$c -o run -- python3 bench.py --model resnet18 --steps 4 --warmup 2 --settle 0 > $O/b_$c.log 2>&1 || { echo "bytes $c failed"; exit 1; }
  python scripts/pmc_table.py $(find $O/b_$c -name "*counter_collection.csv") > $O/bytes_$c.txt || true
  rm -rf $O/b_$c
done
echo "bytes done"
