# Third ResNet-18 sweep (new defaults: SL_WGRAD_WGS 384, BN apply cap 1024): the big weight-gradient
# kernel's own workgroup target (SL_WGRAD_BIG_TARGET; default = WGS / 2 = 192) and, with it pinned
# at 192, the small kernel's target (SL_WGRAD_WGS); driver form, 2 interleaved reps.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_sweep3}
mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift 1
  env "$@" timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' $O/$tag.log)"
}
for rep in 1 2; do
  run r${rep}_base SL_NOP=1
  for v in 96 128 160 256 320; do run r${rep}_big$v SL_WGRAD_BIG_TARGET=$v; done
  for v in 256 512 768 1024; do run r${rep}_small$v SL_WGRAD_BIG_TARGET=192 SL_WGRAD_WGS=$v; done
done
