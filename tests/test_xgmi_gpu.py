"""xGMI exchange (parallel/xgmi.py): several ranks on the box's GPU map each other's
exchange buffers over IPC and run the generic all-reduce and the MLP step with the
all-reduce fused into its update kernel (scripts/xgmi_check.py does the checking)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    from serverless_learn_amd.utils.ports import reserve_port

    return reserve_port()


@pytest.mark.parametrize("world,two_shot", [(2, False), (3, False), (2, True), (3, True),
                                             (4, False), (4, True), (8, True)])
def test_xgmi_exchange_ranks_on_one_gpu(world, two_shot):
    """world 3 with two-shot: chunks of unequal fill (the last rank's chunk is short).  Worlds 4
    and 8 run the two-shot partition and barrier fan-out that ``default_two_shot`` selects on a
    4- or 8-GPU node (parallel/xgmi.py), with the ranks sharing the box's one GPU."""
    limit = 100 + 25 * world
    cmd = ["timeout", "-k", "10", str(limit), sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "scripts", "xgmi_check.py"), "--same-device"] + (["--two-shot"] if two_shot else [])
    from serverless_learn_amd.utils.gpu_share import share_gpu_env

    env = share_gpu_env(dict(os.environ), world)
    p = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=limit + 15,
                       env=env)
    assert p.returncode == 0, p.stdout[-4000:]
    assert p.stdout.count("XGMI_CHECK_OK") == world, p.stdout[-4000:]


def test_bench_four_rank_rehearsal_replicas_identical():
    """bench.py's own N = 4 path (the driver's scaling run launches exactly this code per GPU),
    rehearsed with 4 ranks sharing the one GPU over gloo: the autotuned exchange (one-shot,
    two-shot or the process group) must leave all replicas bit-identical."""
    import json

    cmd = ["timeout", "-k", "10", "200", sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4",
           "--oversubscribe", "--dist-backend", "gloo", "--batch", "4096", "--steps", "8", "--warmup", "3",
           "--ingest", "local"]
    p = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=215)
    assert p.returncode == 0, p.stdout[-4000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{") and '"metric"' in ln][-1]
    r = json.loads(line)
    assert r["n_gpus"] == 4 and r["dist"]["world_size"] == 4, r
    assert r["replicas_identical"] is True, r
    assert r["value"] > 0 and "replica_fallback" not in r, r
