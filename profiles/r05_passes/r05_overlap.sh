# does bucket communication run beside the ResNet-18 backward (B = 1024)?
# Step time without / with the comm proxy on a side stream, with and without CU-masked compute,
# then kernel traces of the proxy runs -> overlap fraction (scripts/overlap_trace.py).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_overlap
mkdir -p $O
run() { timeout -k 10 150 python3 scripts/overlap_probe.py "$@"; }
for rep in 1 2 3; do
  run --steps 10 > $O/none_$rep.json || exit 1
  run --steps 10 --proxy > $O/proxy_$rep.json || exit 1
  run --steps 10 --proxy --passes 1 > $O/proxy1_$rep.json || exit 1
done
run --steps 10 --proxy --mask-cus 1 > $O/proxy_mask1.json || exit 1
run --steps 10 --mask-cus 1 > $O/none_mask1.json || exit 1
cat $O/*.json
# (a rocprofv3 trace of the CU-masked external stream segfaulted the profiler: traces unmasked only)
for tag in "proxy:--proxy" "proxy1:--proxy --passes 1"; do
  name=${tag%%:*}; a=${tag#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$name -o run -- python3 scripts/overlap_probe.py --steps 5 --warmup 2 $a > $O/tr_$name.log 2>&1 || exit 1
  f=$(find $O/tr_$name -name "*kernel_trace.csv" | head -1)
  python3 scripts/overlap_trace.py "$f" > $O/overlap_$name.json; echo "$name $(cat $O/overlap_$name.json | cut -c1-200)"
  cp "$f" $O/kernel_trace_$name.csv; rm -rf $O/tr_$name
done
