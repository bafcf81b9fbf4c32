#!/bin/bash
# One parameterised driver for everything run on the GPU box (replaces the round-1/2 one-off
# gpu_*.sh files).  Runs ON the box (inside gpurun); every GPU step has its own time limit and
# the script stops at the first crash / timeout (gpu_step.sh exits 99 on anything but 0/1).
#
#   scripts/gpu_task.sh tests [pytest selectors...]          GPU test suite (default: tests -m gpu)
#   scripts/gpu_task.sh vtests <variant> <selectors...>       tests against a variant build (SL_KERNELS_SO)
#   scripts/gpu_task.sh bench <name> [bench.py args...]       one bench run -> gpurun_out/<name>.log
#   scripts/gpu_task.sh py <name> <script.py> [args...]       any probe script -> gpurun_out/<name>.log
#   scripts/gpu_task.sh prof <name> [bench.py args...]        rocprofv3 kernel stats -> gpurun_out/<name>/
#   scripts/gpu_task.sh pmc <name> <counters> [bench args]    one PMC pass (counters comma-separated)
#   scripts/gpu_task.sh ab <reps> <v1,v2,..> [bench args]     interleaved A/B of variant builds
#                                                             (scripts/build_variant.sh <v>; "base" = in-tree)
#   scripts/gpu_task.sh ko <v1,v2,..> [bench args]            rocprof kernel stats per variant build
#   scripts/gpu_task.sh full                                  tests + both benches + 2-rank rehearsals + profiles
#
# Several tasks chain with "+": scripts/gpu_task.sh tests + bench b1 --steps 20 + prof p1
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/.."
step() { bash scripts/gpu_step.sh "$@" || exit 1; }
so_of() { [ "$1" = base ] && echo "" || echo serverless_learn_amd/_native/variants/libslkernels_$1.so; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"

run_task() {
  local task=$1; shift
  case "$task" in
    tests)
      local sel=("$@"); [ ${#sel[@]} -eq 0 ] && sel=(tests -m gpu)
      step 900 pytest_gpu.log $PYT "${sel[@]}"
      grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q " failed" gpurun_out/pytest_gpu.log || exit 1 ;;
    vtests)
      local v=$1; shift
      SL_KERNELS_SO=$(so_of "$v") step 600 "pytest_$v.log" $PYT "$@"
      grep -q " passed" "gpurun_out/pytest_$v.log" && ! grep -q " failed" "gpurun_out/pytest_$v.log" || exit 1 ;;
    bench)
      local name=$1; shift
      step 300 "$name.log" python bench.py "$@" ;;
    py)
      local name=$1; shift
      step 300 "$name.log" python "$@" ;;
    prof)
      local name=$1; shift
      step 300 "$name.log" rocprofv3 --kernel-trace --stats -d "gpurun_out/$name" -o run -- python bench.py "$@"
      python scripts/rocprof_summary.py "gpurun_out/$name/run_results.db" > "gpurun_out/$name.summary.txt" 2>&1 || true
      head -12 "gpurun_out/$name.summary.txt" ;;
    pmc)
      local name=$1 ctrs=$2; shift 2
      step 150 "pmc_$name.log" timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${ctrs//,/ } \
        -d "gpurun_out/pmc_$name" -o run --output-format csv -- python bench.py "$@" ;;
    ab)
      local reps=$1 vs=$2; shift 2
      mkdir -p gpurun_out/ab
      for rep in $(seq 1 "$reps"); do
        for v in ${vs//,/ }; do
          SL_KERNELS_SO=$(so_of "$v") timeout -k 10 150 python bench.py "$@" > "gpurun_out/ab/${v}_$rep.log" 2>&1 || exit 1
          echo "$v rep=$rep $(grep -o '"value": [0-9.]*\|"train_loss_last": [0-9.]*' "gpurun_out/ab/${v}_$rep.log" | tr '\n' ' ')" \
            | tee -a gpurun_out/ab/summary.txt
        done
      done ;;
    ko)
      local vs=$1; shift
      for v in ${vs//,/ }; do
        SL_KERNELS_SO=$(so_of "$v") step 200 "ko_$v.log" rocprofv3 --kernel-trace --stats -d "gpurun_out/ko_$v" -o run -- python bench.py "$@"
        echo "== $v"; python scripts/rocprof_summary.py "gpurun_out/ko_$v/run_results.db" | head -8
      done ;;
    full)
      run_task tests
      run_task bench bench_mlp --steps 20 --warmup 5
      run_task bench bench_resnet --model resnet18 --ingest device
      run_task bench bench2_mlp --gpus 2 --oversubscribe --dist-backend gloo --steps 20 --warmup 5 --ingest local
      run_task bench bench2_resnet --gpus 2 --oversubscribe --dist-backend gloo --model resnet18 --batch 256 --steps 5 --warmup 2 --ingest device
      run_task prof prof_mlp --steps 100 --warmup 10 --ingest local
      run_task prof prof_resnet --model resnet18 --ingest device --steps 10 --warmup 3 ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
}

# split the argument list on "+" into tasks
args=()
for a in "$@" "+"; do
  if [ "$a" = "+" ]; then
    [ ${#args[@]} -gt 0 ] && run_task "${args[@]}"
    args=()
  else
    args+=("$a")
  fi
done
