#!/bin/bash
# Run one GPU step under a time limit; stop the whole script on a crash/timeout.
# usage: gpu_step.sh <seconds> <logname> <cmd...>
# exit code 0/1 (ordinary pass/fail) lets the caller continue; anything else aborts.
secs=$1; shift; log=$1; shift
mkdir -p gpurun_out
timeout -k 10 "$secs" "$@" > "gpurun_out/$log" 2>&1
rc=$?
echo "[gpu_step] $log rc=$rc"
tail -n 25 "gpurun_out/$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "[gpu_step] aborting after $log (rc=$rc)"
  exit 99
fi
exit 0
