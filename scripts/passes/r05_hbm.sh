# HBM bytes per MLP step at round-5 HEAD (TCC FETCH_SIZE / WRITE_SIZE, one counter group per
# run) plus MFMA-busy and the graph-step gap table (scripts/stamps_graph.py).
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_hbm
mkdir -p $O
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $O/p$i -o run -- python3 bench.py --steps 30 --warmup 5 --ingest local --settle 0 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
  python scripts/pmc_table.py $(find $O/p$i -name "*counter_collection.csv") --match mlp_ > $O/p$i.txt || true
  rm -rf $O/p$i
done
cat $O/p1.txt $O/p2.txt
timeout -k 10 150 python3 scripts/stamps_graph.py > $O/graph.txt 2>&1 && grep -v amdgpu $O/graph.txt
