# Write-through whole-line stores (SL_STORE_AUX=16) + the SGD kernel at 6 waves per SIMD (583
# workgroups in one round) against b0 (write-back stores, SGD at 5 waves per SIMD): MLP GPU tests,
# graph spans/gaps (scripts/stamps_graph.py) and the driver form, interleaved.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_sgd6}
B=${BASEV:-b0}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; tail -2 $O/pytest_mlp.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for v in new $B; do
    so=""; [ $v != new ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 150 python3 scripts/stamps_graph.py > $O/graph_${v}_$rep.txt 2>&1 || exit 1
    echo "== $v $rep"; grep -v amdgpu.ids $O/graph_${v}_$rep.txt
    SL_KERNELS_SO=$so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
