# Second ResNet-18 sweep around the first one's winners (SL_WGRAD_WGS 384, SL_BN_APPLY_BLOCKS 1024),
# plus the two combined; driver form, 2 interleaved reps.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_sweep2}
mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift 1
  env "$@" timeout -k 10 300 python3 bench.py --model resnet18 --gpus 1 --steps 20 --warmup 5 > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' $O/$tag.log)"
}
for rep in 1 2; do
  run r${rep}_base SL_NOP=1
  for v in 192 256 320 384 448 640; do run r${rep}_wgs$v SL_WGRAD_WGS=$v; done
  for v in 512 768 1024; do run r${rep}_bnapply$v SL_BN_APPLY_BLOCKS=$v; done
  run r${rep}_both SL_WGRAD_WGS=384 SL_BN_APPLY_BLOCKS=1024
done
