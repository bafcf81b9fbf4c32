# Round-4 GPU pass u: driver-form MLP bench spread on a fresh box (3 runs, exactly the driver's command).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_u_$(date +%s)
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.log 2>&1 || exit 1
  echo "run $i $(grep -ho '"value": [0-9.]*' $O/bench_$i.log)"
done
echo r04_u done
