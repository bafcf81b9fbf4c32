"""BASELINE config 5 on the GPU: three worker PROCESSES sharing cuda:0 (gloo group, the MLP's
xGMI exchange live through IPC-mapped buffers, SL_XGMI_GLOO=1), one SIGKILLed mid-run and a
fresh one started.  Checks the regroup, that the survivors closed their old IPC maps and mapped
new ones for the new epoch, identical replicas afterwards, and no hang past the DP timeout
(scripts/elastic_demo.py drives the processes)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpu_workers_kill_one_respawn_with_xgmi(tmp_path):
    dp_timeout = 20.0
    logdir = os.path.join(ROOT, "gpurun_out", "elastic_gpu")  # merged back from the GPU box for post-mortems
    cmd = ["timeout", "-k", "10", "220", sys.executable, os.path.join(ROOT, "scripts", "elastic_demo.py"),
           "--device", "cuda:0", "--dp-backend", "gloo", "--xgmi-gloo", "--workers", "3", "--batch", "1024",
           "--timeout", "200", "--dp-timeout-s", str(dp_timeout), "--logdir", logdir]
    proc = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    assert lines, proc.stderr[-3000:]
    summary = json.loads(lines[-1])
    assert proc.returncode == 0 and summary["ok"], json.dumps(summary)[-3000:]
    assert summary["replicas_after"] and summary["replicas_after"]["distinct"] == 1, summary["replicas_after"]
    # survivors: the exchange was closed for the old epoch and re-mapped for a newer one
    for n in ("w0", "w1"):
        ev = summary["xgmi"][n]
        enabled = [e for k, e in ev if k == "xgmi_enabled"]
        closed = [e for k, e in ev if k == "xgmi_closed"]
        assert len(enabled) >= 2 and closed and max(enabled) > min(closed), (n, ev)
    # the fresh worker mapped its peers too, and everyone trains from graph chunks
    assert any(k == "xgmi_enabled" for k, _ in summary["xgmi"]["w3"]), summary["xgmi"]["w3"]
    assert all(summary["graph"].values()), summary["graph"]
    assert summary["survivor_regroup_s"] < 2 * dp_timeout + 30, summary["survivor_regroup_s"]
