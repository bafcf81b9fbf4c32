# the xGMI exchange's fixed per-step cost at W = 1 (one-shot / two-shot) against the
# fused 1-GPU update, graph-replayed, plus the kernel table of the same run.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_xchg
mkdir -p $O
timeout -k 10 200 python3 scripts/xchg_probe.py 200 3 > $O/xchg.jsonl 2>&1 || exit 1
cat $O/xchg.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 scripts/xchg_probe.py 50 1 > $O/prof.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof/run_results.db > $O/kernels.csv; head -12 $O/kernels.csv | cut -c1-110; rm -rf $O/prof
