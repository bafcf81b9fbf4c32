"""BASELINE config 5 with real OS processes (CLI roles over gRPC, gloo all-reduce):
SIGKILL two of four workers, survivors regroup, two fresh workers resume from the
file server's checkpoint and train in lock-step (scripts/elastic_demo.py)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.slow
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_kill_two_respawn_two_processes(tmp_path):
    proc = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "elastic_demo.py"), "--timeout", "240",
                           "--logdir", str(tmp_path)], capture_output=True, text=True, timeout=420)
    line = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")][-1]
    summary = json.loads(line)
    assert proc.returncode == 0 and summary["ok"], (summary, proc.stderr[-2000:])
    rejoined = summary["phases"]["rejoined"]
    assert summary["replicas_after"] and summary["replicas_after"]["distinct"] == 1, summary["replicas_after"]
    steps = {v[0] for v in rejoined.values()}
    epochs = {v[1] for v in rejoined.values()}
    assert len(epochs) == 1, rejoined          # one group after the rejoin
    assert max(steps) - min(steps) <= 5, rejoined  # lock-step (sampled from logs, log_every=5)
    for n, ev in summary["resumed_from_checkpoint"].items():
        assert ev is not None and ev["step"] > 0, (n, ev)


def test_whole_group_replaced_resumes_from_checkpoint(tmp_path):
    """Every original worker is SIGKILLed; fresh workers pull PeerList.resume_file from the
    file server before the group syncs, so training continues from the checkpoint (step > 0)
    instead of restarting from random weights."""
    proc = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "elastic_demo.py"), "--timeout", "240",
                           "--scenario", "all", "--workers", "2", "--logdir", str(tmp_path)],
                          capture_output=True, text=True, timeout=420)
    line = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")][-1]
    summary = json.loads(line)
    assert proc.returncode == 0 and summary["ok"], (summary, proc.stderr[-2000:])
    for n, ev in summary["resumed_from_checkpoint"].items():
        assert ev is not None and ev["step"] > 0, (n, ev)
    assert summary["replicas_after"]["distinct"] == 1, summary["replicas_after"]
