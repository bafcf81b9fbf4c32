"""Command-line entry points: ``sl-master``, ``sl-file-server``, ``sl-worker ADDR``.

Reference binaries: ``master`` and ``file_server`` take no arguments
(/root/reference/src/master.cc:295-310, file_server.cc:150-165); ``worker ADDR``
takes its listen address (worker.cc:233-258).  These keep that shape -- the
positional worker address, defaults equal to the reference's constants -- and
add flags/env for every knob (:mod:`serverless_learn_amd.config`).

    python -m serverless_learn_amd.cli master
    python -m serverless_learn_amd.cli file-server
    python -m serverless_learn_amd.cli worker localhost:50061 [--device cuda:0]
"""
from __future__ import annotations

import argparse
import signal
import sys
import threading

from .config import add_cli_args, from_args


def _run_until_signal(obj, on_stop=None) -> int:
    done = threading.Event()

    def handler(signum, frame):
        done.set()

    signal.signal(signal.SIGINT, handler)
    signal.signal(signal.SIGTERM, handler)
    done.wait()
    (on_stop or obj.stop)()
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="serverless_learn_amd")
    sub = ap.add_subparsers(dest="role", required=True)
    pm = sub.add_parser("master")
    pf = sub.add_parser("file-server")
    pw = sub.add_parser("worker")
    pw.add_argument("addr", help="host:port to serve the Worker API on (e.g. localhost:50061)")
    for p in (pm, pf, pw):
        add_cli_args(p)
    args = ap.parse_args(argv)
    cfg = from_args(args)
    if args.role == "master":
        from .runtime.master import Master

        return _run_until_signal(Master(cfg).start())
    if args.role == "file-server":
        from .runtime.file_server import FileServer

        return _run_until_signal(FileServer(cfg).start())
    from .runtime.worker import Worker

    w = Worker(args.addr, cfg).start()
    return _run_until_signal(w, lambda: w.stop(leave=True))


def master_main():
    sys.exit(main(["master"] + sys.argv[1:]))


def file_server_main():
    sys.exit(main(["file-server"] + sys.argv[1:]))


def worker_main():
    sys.exit(main(["worker"] + sys.argv[1:]))


if __name__ == "__main__":
    sys.exit(main())
