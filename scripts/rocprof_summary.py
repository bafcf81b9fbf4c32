#!/usr/bin/env python3
"""Summarise a rocprofv3 SQLite result (``-d DIR -o NAME`` -> NAME_results.db)
into a per-kernel stats CSV (name, calls, total/avg/min/max ns, share), the
same columns as rocprofv3's ``--stats`` kernel_stats.csv.

usage: python scripts/rocprof_summary.py <results.db> [out.csv]
"""
import csv
import sqlite3
import sys


def main(argv):
    db = sqlite3.connect(argv[1])
    rows = db.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = open(argv[2], "w", newline="") if len(argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([name[:160], n, tot, round(avg, 1), round(100.0 * tot / total, 2), mn, mx])
    return 0


if __name__ == "__main__":
    raise SystemExit(main(sys.argv))
