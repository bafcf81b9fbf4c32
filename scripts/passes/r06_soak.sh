# Round 6: longer runs on the lean / wide conv kernels -- MLP 1000 and ResNet-18 200 timed
# steps, ResNet-18 at B = 2048, the runtime-roles MLP path over 2000 steps, and a 4-rank
# same-GPU gloo rehearsal of both models (replicas must stay bit-identical).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r06_soak}
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 1 --steps 1000 --warmup 20 > $O/mlp_1000.log 2>&1 || exit 1
echo "mlp 1000 $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*\|"train_acc_last": [0-9.]*' $O/mlp_1000.log | tr '\n' ' ')"
timeout -k 10 400 python3 bench.py --model resnet18 --gpus 1 --steps 200 --warmup 5 > $O/resnet_200.log 2>&1 || exit 1
echo "resnet 200 $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*\|"train_acc_last": [0-9.]*' $O/resnet_200.log | tr '\n' ' ')"
timeout -k 10 400 python3 bench.py --model resnet18 --gpus 1 --batch 2048 > $O/resnet_b2048.log 2>&1 || exit 1
echo "resnet b2048 $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/resnet_b2048.log | tr '\n' ' ')"
timeout -k 10 400 python3 bench.py --runtime --gpus 1 --steps 2000 --warmup 20 > $O/runtime_2000.log 2>&1 || exit 1
echo "runtime 2000 $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' $O/runtime_2000.log | tr '\n' ' ')"
timeout -k 10 400 python3 bench.py --gpus 4 --oversubscribe --dist-backend gloo --steps 20 --warmup 5 --ingest local > $O/mlp_w4.log 2>&1 || exit 1
echo "mlp w4 $(grep -o '"value": [0-9.]*\|"replicas_identical": [a-z]*' $O/mlp_w4.log | tr '\n' ' ')"
timeout -k 10 400 python3 bench.py --gpus 4 --oversubscribe --dist-backend gloo --model resnet18 --batch 256 --steps 5 --warmup 2 --ingest device > $O/resnet_w4.log 2>&1 || exit 1
echo "resnet w4 $(grep -o '"value": [0-9.]*\|"replicas_identical": [a-z]*' $O/resnet_w4.log | tr '\n' ' ')"
