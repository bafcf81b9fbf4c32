#!/usr/bin/env python3
"""Per-burst view of a rocprofv3 kernel trace: where does a graph replay's time go?

Reads ``kernel_trace.csv`` (``rocprofv3 --kernel-trace --output-format csv``) or a
``*_results.db``, sorts dispatches by start time and splits them into *bursts* at idle gaps
longer than ``--split-us`` (a host sync between two replays leaves such a gap).  For every
burst it prints the kernel count, the span, the summed kernel time and the summed
inter-kernel gaps, plus per kernel name the mean duration and the mean gap in front of it;
``--steps`` adds the per-step span of one burst (first kernel of step i to the first kernel
of step i+1) so the first steps of a replay can be compared with its last ones.

usage: python scripts/trace_gaps.py <kernel_trace.csv | results.db> [--split-us 30] [--json out.json]
       [--burst N --steps K]
"""
import argparse
import csv
import json
import os
import sqlite3
import statistics as st


def load(path):
    rows = []
    if path.endswith(".db"):
        db = sqlite3.connect(path)
        for name, s, e in db.execute("select name, start, end from kernels"):
            rows.append((int(s), int(e), name))
    else:
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").split("<")[0][-40:]


def bursts(rows, split_ns):
    out, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - cur[-1][1] > split_ns:
            out.append(cur)
            cur = []
        cur.append(r)
    out.append(cur)
    return out


def describe(b):
    span = b[-1][1] - b[0][0]
    busy = sum(e - s for s, e, _ in b)
    per = {}
    prev_end = None
    for s, e, n in b:
        d = per.setdefault(short(n), {"n": 0, "dur": [], "gap": []})
        d["n"] += 1
        d["dur"].append(e - s)
        if prev_end is not None:
            d["gap"].append(s - prev_end)
        prev_end = e
    return {
        "kernels": len(b), "span_us": round(span / 1e3, 1), "busy_us": round(busy / 1e3, 1),
        "gaps_us": round((span - busy) / 1e3, 1),
        "by_kernel": {k: {"n": v["n"], "mean_us": round(st.mean(v["dur"]) / 1e3, 2),
                          "min_us": round(min(v["dur"]) / 1e3, 2), "max_us": round(max(v["dur"]) / 1e3, 2),
                          "mean_gap_us": round(st.mean(v["gap"]) / 1e3, 2) if v["gap"] else None}
                      for k, v in per.items()},
    }


def steps_of(b, first_name):
    starts = [i for i, (_, _, n) in enumerate(b) if short(n) == first_name]
    out = []
    for a, z in zip(starts, starts[1:] + [len(b)]):
        seg = b[a:z]
        end = b[z][0] if z < len(b) else seg[-1][1]
        out.append({"step_us": round((end - seg[0][0]) / 1e3, 2),
                    "kernels_us": [round((e - s) / 1e3, 2) for s, e, _ in seg],
                    "gaps_us": [round((seg[i + 1][0] - seg[i][1]) / 1e3, 2) for i in range(len(seg) - 1)]})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--split-us", type=float, default=30.0)
    ap.add_argument("--burst", type=int, action="append", default=[])
    ap.add_argument("--steps", default=None, help="kernel name that starts a step (e.g. mlp_rows_kernel)")
    ap.add_argument("--min-kernels", type=int, default=1)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = load(a.trace)
    bs = bursts(rows, a.split_us * 1e3)
    report = []
    t0 = rows[0][0]
    for i, b in enumerate(bs):
        if len(b) < a.min_kernels:
            continue
        d = describe(b)
        d["burst"] = i
        d["t_start_ms"] = round((b[0][0] - t0) / 1e6, 3)
        d["idle_before_us"] = round((b[0][0] - bs[i - 1][-1][1]) / 1e3, 1) if i else None
        if a.steps and i in a.burst:
            d["steps"] = steps_of(b, a.steps)
        report.append(d)
        names = ", ".join(f"{k} x{v['n']} {v['mean_us']}us (gap {v['mean_gap_us']})" for k, v in d["by_kernel"].items())
        print(f"burst {i:4d} t={d['t_start_ms']:9.3f}ms idle_before={d['idle_before_us']}us kernels={d['kernels']} "
              f"span={d['span_us']}us busy={d['busy_us']}us gaps={d['gaps_us']}us :: {names}")
        for j, s in enumerate(d.get("steps", [])):
            print(f"    step {j:3d} {s['step_us']:8.2f}us kernels {s['kernels_us']} gaps {s['gaps_us']}")
    if a.json:
        os.makedirs(os.path.dirname(os.path.abspath(a.json)), exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(report, f)


if __name__ == "__main__":
    main()
