# Wave priority for the younger workgroup of each CU pair (SL_ROWS_PRIO=1: after layer 1, 2: after
# the softmax) against base: rows-kernel CU-pair stamps, graph spans/gaps, driver form; interleaved.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_prio}
mkdir -p $O
for rep in 1 2; do
  for v in base ${VARIANTS:-prio1 prio2}; do
    so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 120 python3 scripts/stamps_mlp.py > $O/stamps_${v}_$rep.txt 2>&1 || exit 1
    SL_KERNELS_SO=$so timeout -k 10 150 python3 scripts/stamps_graph.py > $O/graph_${v}_$rep.txt 2>&1 || exit 1
    SL_KERNELS_SO=$so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "== $v $rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
    grep "step (events\|^rows\|younger\|WG total" $O/graph_${v}_$rep.txt $O/stamps_${v}_$rep.txt | cut -d: -f2- | cut -c1-130
  done
done
