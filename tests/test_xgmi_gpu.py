"""xGMI exchange (parallel/xgmi.py): several ranks on the box's GPU map each other's
exchange buffers over IPC and run the generic all-reduce and the MLP step with the
all-reduce fused into its update kernel (scripts/xgmi_check.py does the checking)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,two_shot", [(2, False), (3, False), (2, True), (3, True)])
def test_xgmi_exchange_ranks_on_one_gpu(world, two_shot):
    """world 3 with two-shot: chunks of unequal fill (the last rank's chunk is short)."""
    cmd = ["timeout", "-k", "10", "100", sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "scripts", "xgmi_check.py"), "--same-device"] + (["--two-shot"] if two_shot else [])
    p = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=115)
    assert p.returncode == 0, p.stdout[-4000:]
    assert p.stdout.count("XGMI_CHECK_OK") == world, p.stdout[-4000:]
