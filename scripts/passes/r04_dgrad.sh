# Round-4 GPU pass: cost split of the stage-2 stride-2 data gradient into 64 channels
# (scripts/dgrad_probe.py: plain / + add / + fused BN backward / both), plus its kernel trace.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_dgrad
mkdir -p $O
timeout -k 10 200 python3 scripts/dgrad_probe.py > $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 scripts/dgrad_probe.py --reps 10 > $O/prof.log 2>&1 || exit 1
python scripts/rocprof_summary.py $O/prof/run_results.db > $O/kernels.csv; rm -rf $O/prof
head -8 $O/kernels.csv | cut -c1-150
timeout -k 10 200 python3 scripts/dgrad_probe.py --h 16 --cin 128 > $O/probe_s3.json 2>&1 || exit 1
cat $O/probe_s3.json
timeout -k 10 200 python3 scripts/dgrad_probe.py --h 8 --cin 256 > $O/probe_s4.json 2>&1 || exit 1
cat $O/probe_s4.json
echo r04_dgrad done
