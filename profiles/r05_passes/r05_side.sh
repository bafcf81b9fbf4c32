# Side-stream slab reduces of the split-K weight gradients (SL_WGRAD_SIDE=1) re-measured on the round-5
# kernels against the default (0): ResNet-18 driver form, 3 interleaved reps, plus kernel tables.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_side}
mkdir -p $O
for rep in 1 2 3; do
  for v in 0 1; do
    SL_WGRAD_SIDE=$v timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "side=$v $rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
