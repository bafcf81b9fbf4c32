#!/bin/bash
# Interleaved A/B of environment settings on one box (runs ON the GPU box):
#   scripts/ab_env.sh <reps> "<ENV=a ENV2=b>" "<ENV=c>" ... -- [bench.py args]
# One bench.py process per arm and rep, each under its own time limit; stops at the first failure.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/abenv
reps=$1; shift
arms=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do arms+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
for rep in $(seq 1 "$reps"); do
  for i in "${!arms[@]}"; do
    log="gpurun_out/abenv/arm${i}_$rep.log"
    env ${arms[$i]} timeout -k 10 150 python bench.py "$@" > "$log" 2>&1 || { echo "arm $i rep $rep failed"; tail -20 "$log"; exit 1; }
    echo "[${arms[$i]}] rep=$rep $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"train_loss_last": [0-9.]*' "$log" | tr '\n' ' ')" \
      | tee -a gpurun_out/abenv/summary.txt
  done
done
