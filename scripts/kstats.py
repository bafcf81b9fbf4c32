#!/usr/bin/env python3
"""Per-step kernel table of a rocprofv3 run of bench.py --steps 10 --warmup 3 (13 steps).

usage: python scripts/kstats.py <results.db> [steps=13] [rows=14]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 13.0
nrows = int(sys.argv[3]) if len(sys.argv) > 3 else 14
rows = db.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name "
                  "order by sum(duration) desc").fetchall()
print(f"total us/step {sum(r[2] for r in rows) / steps / 1e3:.1f}")
for name, n, tot, avg in rows[:nrows]:
    print(f"{tot / steps / 1e3:8.1f} {n / steps:5.1f} avg {avg / 1e3:7.1f}  {name[:70]}")
