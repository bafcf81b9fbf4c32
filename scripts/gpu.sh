#!/bin/bash
# Host-side wrapper: run one gpurun call; re-submit only when the harness reports a
# transient box problem (nothing ran on the GPU), never after a GPU-side failure.
# usage: scripts/gpu.sh <timeout_s> <command...>
t=$1; shift
mkdir -p gpurun_out/prev; mv -f gpurun_out/*.log gpurun_out/prev/ 2>/dev/null
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$rc" = "3" ] || [ "$st" = "transient" ]; then echo "[gpu.sh] transient ($st rc=$rc), retry in 60s"; sleep 60; continue; fi
  exit $rc
done
exit $rc
