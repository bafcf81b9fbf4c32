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
        [--scenario kill2|all] [--dp-backend gloo] [--xgmi-gloo]

``--scenario all`` kills EVERY original worker and starts fresh ones, which must resume
from the file server's checkpoint (``PeerList.resume_file``) -- the whole-group
replacement case.  ``--device cuda --dp-backend gloo --xgmi-gloo`` runs the workers as
GPU processes sharing one GPU with the MLP's xGMI exchange live (IPC maps dropped and
re-made on every regroup), the GPU rehearsal of BASELINE config 5.

The reference has leave-unhandled, log-only failure detection
(/root/reference/src/master.cc:240-266) and no checkpoints; this exercises the
eviction -> epoch bump -> regroup -> checkpoint resume path end to end.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def free_port() -> int:
    from serverless_learn_amd.utils.ports import reserve_port

    return reserve_port()


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
    ap.add_argument("--scenario", choices=["kill2", "all"], default="kill2")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--dp-backend", default="auto")
    ap.add_argument("--dp-timeout-s", type=float, default=20.0)
    ap.add_argument("--xgmi-gloo", action="store_true", help="SL_XGMI_GLOO=1: xGMI exchange on a gloo group")
    args = ap.parse_args(argv)

    logdir = args.logdir or tempfile.mkdtemp(prefix="sl_elastic_")
    os.makedirs(logdir, exist_ok=True)
    mport, fport = free_port(), free_port()
    common = ["--master-addr", f"127.0.0.1:{mport}", "--file-server-addr", f"127.0.0.1:{fport}",
              "--checkup-interval-ms", "300", "--push-interval-ms", "300", "--max-misses", "2",
              "--rpc-timeout-s", "2.0", "--log-every", "5", "--checkpoint-every", "20",
              "--shard-records", "4096", "--model", args.model, "--batch", str(args.batch),
              "--device", args.device, "--sync", "allreduce", "--dp-backend", args.dp_backend,
              "--dp-timeout-s", str(args.dp_timeout_s)]
    if args.model == "resnet18":
        common += ["--dataset", "synthetic-cifar"]
    procs: dict[str, subprocess.Popen] = {}
    logs: dict[str, str] = {}

    def spawn(name, role_args):
        path = os.path.join(logdir, name + ".log")
        env = dict(os.environ, SL_LOG_FILE=path, PYTHONPATH=ROOT, SL_LOG_PARAM_SUM="1", SL_STALL_DUMP_S="3")
        if args.xgmi_gloo:
            env["SL_XGMI_GLOO"] = "1"
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

    def replicas_agree(group):
        """Parameter checksums the workers logged at the newest step they all logged: lock-step
        replicas must match (one value)."""
        per = {n: {e["step"]: e.get("param_sum") for e in read_events(logs[n])
                   if e.get("event") == "train" and "param_sum" in e} for n in group}
        common = set.intersection(*(set(v) for v in per.values())) if per else set()
        if not common:
            return None
        st = max(common)
        vals = {per[n][st] for n in group}
        return {"step": st, "distinct": len(vals), "sums": sorted(vals)}

    summary = {"ok": False, "logdir": logdir, "phases": {}}
    try:
        spawn("file_server", ["file-server"])
        spawn("master", ["master"])
        time.sleep(1.0)
        names = [f"w{i}" for i in range(args.workers)]
        for i, n in enumerate(names):
            spawn(n, ["worker", f"127.0.0.1:{free_port()}"])
        budget = args.timeout

        # phase 1: all train together, a checkpoint exists
        ok = wait(lambda: all(worker_state(n)[0] >= 30 for n in names)
                  and last(read_events(logs["master"]), "checkpoint_reported") is not None, budget / 3,
                  f"{len(names)} workers training + checkpoint")
        summary["phases"]["train_all"] = {n: worker_state(n)[:2] for n in names}
        summary["replicas_before"] = replicas_agree(names)
        if not ok:
            return 1
        # phase 2: SIGKILL workers (no Deregister: the master must notice missed heartbeats)
        victims = names[2:] if args.scenario == "kill2" else list(names)
        survivors = [n for n in names if n not in victims]
        t_kill = time.time()
        for n in victims:
            procs[n].send_signal(signal.SIGKILL)
            procs[n].wait()
        killed_at = {n: worker_state(n)[0] for n in names}
        ok = wait(lambda: sum(1 for e in read_events(logs["master"]) if e.get("event") == "evicted") >= len(victims),
                  budget / 4, f"eviction of {len(victims)} workers")
        if survivors:
            ok = ok and wait(lambda: all(worker_state(n)[0] >= killed_at[n] + 15 for n in survivors), budget / 4,
                             "survivors training after regroup")
            summary["survivor_regroup_s"] = round(time.time() - t_kill, 2)
        summary["phases"]["survivors"] = {n: worker_state(n)[:2] for n in survivors}
        if not ok:
            return 1
        # phase 3: fresh workers join, load the checkpoint, and train with the group
        fresh = [f"w{len(names) + i}" for i in range(len(victims))]
        for n in fresh:
            spawn(n, ["worker", f"127.0.0.1:{free_port()}"])
        base = max(killed_at.values()) if survivors else 0
        ok = wait(lambda: all(last(read_events(logs[n]), "checkpoint_loaded") is not None or
                              last(read_events(logs[n]), "state_synced") is not None or bool(survivors)
                              for n in fresh)
                  and all(worker_state(n)[0] >= base + 20 for n in fresh), budget / 3,
                  "fresh workers resumed and training")
        group = survivors + fresh
        summary["phases"]["rejoined"] = {n: worker_state(n)[:2] for n in group}
        summary["resumed_from_checkpoint"] = {n: last(read_events(logs[n]), "checkpoint_loaded") for n in fresh}
        summary["resume_pulled"] = {n: last(read_events(logs[n]), "resume_pulled") for n in fresh}
        # the fresh workers may have logged the step that met the wait a few ms before the
        # survivors logged it (each writes its own log after the chunk): give them a moment
        t_rep = time.time()
        while replicas_agree(group) is None and time.time() - t_rep < 10.0:
            time.sleep(0.2)
        summary["replicas_after"] = replicas_agree(group)
        summary["xgmi"] = {n: [(e.get("event"), e.get("epoch")) for e in read_events(logs[n])
                               if e.get("event") in ("xgmi_enabled", "xgmi_closed")] for n in group}
        summary["graph"] = {n: bool((last(read_events(logs[n]), "train") or {}).get("graph")) for n in group}
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
        if not summary.get("ok"):
            tails = {}
            for n, path in logs.items():
                try:
                    with open(path + ".err") as f:
                        tails[n] = f.read()[-1500:]
                except OSError:
                    pass
            summary["stderr_tails"] = tails
            summary["last_events"] = {n: [(e.get("event"), e.get("step"), e.get("epoch")) for e in read_events(path)[-8:]]
                                      for n, path in logs.items()}
        print(json.dumps(summary, default=str))


if __name__ == "__main__":
    raise SystemExit(main())
