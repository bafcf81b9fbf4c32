#!/usr/bin/env python3
"""BASELINE config 5 as real processes: kill + respawn 2 workers mid-run.

Starts ``file-server``, ``master`` and 4 ``worker`` processes through the CLI
(one OS process per role, gRPC between them, gloo/RCCL all-reduce between the
workers), lets them train in one all-reduce group, SIGKILLs two workers (no
Deregister: the master must detect the failure by missed heartbeats), waits
for the survivors to regroup, starts two fresh workers, and checks that they
load the file server's latest checkpoint and join the group.  Prints one JSON
summary line; exit code 0 iff every phase happened.

    python scripts/elastic_demo.py [--device cpu|cuda] [--model mlp|resnet18] [--timeout 240]

The reference has leave-unhandled, log-only failure detection
(/root/reference/src/master.cc:240-266) and no checkpoints; this exercises the
eviction -> epoch bump -> regroup -> checkpoint resume path end to end.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def read_events(path: str) -> list[dict]:
    out = []
    try:
        with open(path) as f:
            for line in f:
                line = line.strip()
                if line.startswith("{"):
                    try:
                        out.append(json.loads(line))
                    except ValueError:
                        pass
    except FileNotFoundError:
        pass
    return out


def last(events, name):
    for e in reversed(events):
        if e.get("event") == name:
            return e
    return None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--model", default="mlp")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--timeout", type=float, default=240.0)
    ap.add_argument("--logdir", default=None)
    args = ap.parse_args(argv)

    logdir = args.logdir or tempfile.mkdtemp(prefix="sl_elastic_")
    os.makedirs(logdir, exist_ok=True)
    mport, fport = free_port(), free_port()
    common = ["--master-addr", f"127.0.0.1:{mport}", "--file-server-addr", f"127.0.0.1:{fport}",
              "--checkup-interval-ms", "300", "--push-interval-ms", "300", "--max-misses", "2",
              "--rpc-timeout-s", "2.0", "--log-every", "5", "--checkpoint-every", "20",
              "--shard-records", "4096", "--model", args.model, "--batch", str(args.batch),
              "--device", args.device, "--sync", "allreduce"]
    if args.model == "resnet18":
        common += ["--dataset", "synthetic-cifar"]
    procs: dict[str, subprocess.Popen] = {}
    logs: dict[str, str] = {}

    def spawn(name, role_args):
        path = os.path.join(logdir, name + ".log")
        env = dict(os.environ, SL_LOG_FILE=path, PYTHONPATH=ROOT)
        env.setdefault("OMP_NUM_THREADS", "2")
        procs[name] = subprocess.Popen([sys.executable, "-m", "serverless_learn_amd.cli", *role_args, *common],
                                       env=env, stdout=subprocess.DEVNULL, stderr=open(path + ".err", "w"))
        logs[name] = path

    def wait(pred, timeout, what):
        t0 = time.time()
        while time.time() - t0 < timeout:
            if pred():
                return True
            time.sleep(0.25)
        print(f"timeout waiting for: {what}", file=sys.stderr)
        return False

    def worker_state(name):
        ev = read_events(logs[name])
        tr = last(ev, "train")
        return (tr or {}).get("step", 0), (tr or {}).get("epoch", -1), ev

    summary = {"ok": False, "logdir": logdir, "phases": {}}
    try:
        spawn("file_server", ["file-server"])
        spawn("master", ["master"])
        time.sleep(1.0)
        names = [f"w{i}" for i in range(4)]
        for i, n in enumerate(names):
            spawn(n, ["worker", f"127.0.0.1:{free_port()}"])
        budget = args.timeout

        # phase 1: all four train together, a checkpoint exists
        ok = wait(lambda: all(worker_state(n)[0] >= 30 for n in names)
                  and last(read_events(logs["master"]), "checkpoint_reported") is not None, budget / 3,
                  "4 workers training + checkpoint")
        summary["phases"]["train4"] = {n: worker_state(n)[:2] for n in names}
        if not ok:
            return 1
        # phase 2: SIGKILL two workers (no Deregister)
        for n in names[2:]:
            procs[n].send_signal(signal.SIGKILL)
            procs[n].wait()
        killed_at = {n: worker_state(n)[0] for n in names[:2]}
        ok = wait(lambda: sum(1 for e in read_events(logs["master"]) if e.get("event") == "evicted") >= 2,
                  budget / 4, "eviction of 2 workers")
        ok = ok and wait(lambda: all(worker_state(n)[0] >= killed_at[n] + 15 for n in names[:2]), budget / 4,
                         "survivors training after regroup")
        summary["phases"]["survivors"] = {n: worker_state(n)[:2] for n in names[:2]}
        if not ok:
            return 1
        # phase 3: two fresh workers join, load the checkpoint, and train with the group
        fresh = ["w4", "w5"]
        for n in fresh:
            spawn(n, ["worker", f"127.0.0.1:{free_port()}"])
        ok = wait(lambda: all(last(read_events(logs[n]), "checkpoint_loaded") is not None or
                              last(read_events(logs[n]), "state_synced") is not None for n in fresh)
                  and all(worker_state(n)[0] >= killed_at[names[0]] + 20 for n in fresh), budget / 3,
                  "fresh workers resumed and training")
        summary["phases"]["rejoined"] = {n: worker_state(n)[:2] for n in names[:2] + fresh}
        summary["resumed_from_checkpoint"] = {n: last(read_events(logs[n]), "checkpoint_loaded") for n in fresh}
        summary["ok"] = bool(ok)
        return 0 if ok else 1
    finally:
        for p in procs.values():
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs.values():
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        print(json.dumps(summary, default=str))


if __name__ == "__main__":
    raise SystemExit(main())
