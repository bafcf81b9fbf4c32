# Compile-time knob variants of the ResNet conv kernels vs main, driver form, 3 interleaved reps:
# halo4 (direct-3x3 kernels with 4 waves), g128s3 (128x128 implicit GEMM with a 3-slot ring),
# wgm32 / wg128s3 (128-wide weight-gradient tile: 32-pixel stages / 3-slot ring); plus the big
# GEMM switched off at run time (SL_GEMM_BIG=0) as a control.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_ksweep}
mkdir -p $O
for rep in 1 2 3; do
  for v in main halo4 g128s3 wgm32 wg128s3 nobig; do
    so=""; case $v in main|nobig) ;; *) so=serverless_learn_amd/_native/variants/libslkernels_$v.so;; esac
    big=1; [ $v = nobig ] && big=0
    SL_GEMM_BIG=$big SL_KERNELS_SO=$so timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$rep.log 2>&1 || { echo "FAIL $v"; tail -3 $O/bench_${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/bench_${v}_$rep.log | tr '\n' ' ')"
  done
done
