"""RCCL (the ``nccl`` backend) on the hardware: a one-rank ``ProcessGroupNCCL`` drives the MLP
all-reduce hook and the ResNet engine's bucketed async all-reduces, eager and captured in a
hipGraph, bit-identical to the hook-free step in the deterministic kernel build.  The
reference's gradient exchange this replaces is the gossip RPC (/root/reference/src/worker.cc:
194-219).  Runs in a child process (one kernel library and one process group per process)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_hooks_eager_and_graph_captured_are_bit_identical():
    env = dict(os.environ, SL_DETERMINISTIC="1", MASTER_ADDR="127.0.0.1")
    env.pop("MASTER_PORT", None)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_one_rank_check.py")],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["backend"] == "nccl" and r["world"] == 1 and r["deterministic_build"], r
    assert r["mlp_eager_identical"] and r["mlp_graph_identical"], r
    assert r["mlp_cursor"] == [5, 5], r
    assert r["resnet_buckets_per_step"] >= 2, r
    assert r["resnet_eager_identical"] and r["resnet_graph_identical"], r
    assert r["resnet_cursor"] == [4, 4] and r["finite"], r
