# Rows kernel: the label logit by one ds_bpermute and the argmax by a wave ballot instead of two
# 16-lane DPP reductions per row (-43 VALU per wave) vs b2: MLP GPU tests, driver form x5.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_ce}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/pytest_mlp.log 2>&1
rc=$?; tail -1 $O/pytest_mlp.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3 4 5; do
  for v in new b2; do
    so=""; [ $v != new ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -o '"value": [0-9.]*\|"settled_samples_per_s": [0-9.]*\|"train_loss_last": [0-9.]*\|"train_acc_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
# + younger-half wave priority in the 8-wave conv kernels (variant wprio, SL_WAVE_PRIO=1) vs main
for rep in 1 2 3; do
  for v in new wprio; do
    so=""; [ $v != new ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/rn_${v}_$rep.log 2>&1 || exit 1
    echo "resnet $v $rep $(grep -o '"value": [0-9.]*' $O/rn_${v}_$rep.log)"
  done
done
# + the MLP weight gradient (8 waves per workgroup) with the same priority (variant wprio) vs main
for rep in 1 2 3 4; do
  for v in new wprio; do
    so=""; [ $v != new ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/mw_${v}_$rep.log 2>&1 || exit 1
    echo "mlp-wprio $v $rep $(grep -o '"value": [0-9.]*\|"settled_samples_per_s": [0-9.]*' $O/mw_${v}_$rep.log | tr '\n' ' ')"
  done
done
