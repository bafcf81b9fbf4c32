# Kernel spans and launch gaps of the graph-replayed MLP step (scripts/stamps_graph.py) for the
# base build and the write-through store variants (sc1: every handed-off store sc1; sc1w: only
# the whole-line 16-B ones), interleaved twice.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${PASS_TAG:-r05_gaps}
mkdir -p $O
for rep in 1 2; do
  for v in ${VARIANTS:-base sc1 sc1w}; do
    so=""; [ $v != base ] && so=serverless_learn_amd/_native/variants/libslkernels_$v.so
    SL_KERNELS_SO=$so timeout -k 10 150 python3 scripts/stamps_graph.py > $O/graph_${v}_$rep.txt 2>&1 || exit 1
    echo "== $v $rep"; grep -v amdgpu.ids $O/graph_${v}_$rep.txt
  done
done
