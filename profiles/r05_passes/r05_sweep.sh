# Launch-shape knobs re-swept on round-5 kernels, driver form, 2 interleaved reps per setting:
# ResNet-18 (B = 1024): split-K workgroup target of the weight gradients (SL_WGRAD_WGS, default
# 768), 128-row tile threshold (SL_GEMM_SMALLM, 512), BN stream grid cap (SL_BN_APPLY_BLOCKS,
# 4096); MLP (B = 65,536): weight-gradient split-K slices (SL_MLP_WG_SLICES, 28).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_sweep}
mkdir -p $O
run() {  # tag, model, env...
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --model $model --gpus 1 --steps 20 --warmup 5 > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' $O/$tag.log)"
}
for rep in 1 2; do
  run r${rep}_base resnet18 SL_NOP=1
  for v in 384 512 1024 1536; do run r${rep}_wgs$v resnet18 SL_WGRAD_WGS=$v; done
  for v in 256 1024; do run r${rep}_smallm$v resnet18 SL_GEMM_SMALLM=$v; done
  for v in 1024 2048 8192; do run r${rep}_bnapply$v resnet18 SL_BN_APPLY_BLOCKS=$v; done
  run m${rep}_base mlp SL_NOP=1
  for v in 20 24 32 36; do run m${rep}_slices$v mlp SL_MLP_WG_SLICES=$v; done
done
