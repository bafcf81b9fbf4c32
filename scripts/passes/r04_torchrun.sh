# Round-4 GPU pass: bench.py through the driver's multi-GPU launcher form (torch.distributed.run,
# one rank per GPU, rendezvous on 127.0.0.1) at N = 1 with RCCL, and N = 2 ranks sharing the one GPU
# over gloo (the only multi-rank form one GPU allows).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_torchrun
mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 > $O/torchrun_n1.log 2>&1 || { tail -20 $O/torchrun_n1.log; exit 1; }
grep -h '^{' $O/torchrun_n1.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --model resnet18 --steps 10 --warmup 3 > $O/torchrun_n1_resnet.log 2>&1 || { tail -20 $O/torchrun_n1_resnet.log; exit 1; }
grep -h '^{' $O/torchrun_n1_resnet.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --oversubscribe --dist-backend gloo --steps 20 --warmup 5 > $O/torchrun_n2.log 2>&1 || { tail -20 $O/torchrun_n2.log; exit 1; }
grep -h '^{' $O/torchrun_n2.log
echo r04_torchrun done
