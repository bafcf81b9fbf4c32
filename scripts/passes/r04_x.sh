# Round-4 GPU pass x: long runs at HEAD (settled throughput and stability).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_x
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 1 --steps 5000 --warmup 100 --ingest local > $O/mlp_5000.log 2>&1 || exit 1
echo "mlp 5000 $(grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"train_loss_last": [0-9.]*\|"train_acc_last": [0-9.]*' $O/mlp_5000.log | tr '\n' ' ')"
timeout -k 10 300 python3 bench.py --runtime --steps 2000 --warmup 64 > $O/rt_2000.log 2>&1 || exit 1
echo "runtime 2000 $(grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/rt_2000.log | tr '\n' ' ')"
timeout -k 10 400 python3 bench.py --model resnet18 --ingest device --steps 300 --warmup 20 > $O/rn_300.log 2>&1 || exit 1
echo "resnet 300 $(grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"train_loss_last": [0-9.]*' $O/rn_300.log | tr '\n' ' ')"
timeout -k 10 400 python3 bench.py --model resnet18 --ingest device --batch 4096 --steps 20 --warmup 5 > $O/rn_b4096.log 2>&1 || exit 1
echo "resnet B=4096 $(grep -ho '"value": [0-9.]*' $O/rn_b4096.log)"
SL_DETERMINISTIC=1 timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --ingest local > $O/mlp_det.log 2>&1 || exit 1
echo "mlp deterministic build $(grep -ho '"value": [0-9.]*' $O/mlp_det.log)"
echo r04_x done
