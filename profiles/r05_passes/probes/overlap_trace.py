#!/usr/bin/env python3
"""Overlap of the comm-proxy kernels with everything else, from a rocprofv3 kernel trace CSV
(scripts/overlap_probe.py).  For each proxy dispatch: the fraction of its lifetime during which
at least one other kernel was also running; prints per-dispatch rows and the totals as JSON."""
import csv
import json
import sys


def main() -> int:
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    prox = [k for k in ks if "comm_proxy" in k[2]]
    other = sorted((s, e) for s, e, n in ks if "comm_proxy" not in n)
    # union of the other kernels' intervals
    merged = []
    for s, e in other:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    tot = ov = 0
    per = []
    for s, e, _ in prox:
        d = e - s
        o = sum(max(0, min(e, me) - max(s, ms)) for ms, me in merged)
        tot += d
        ov += o
        per.append((round(d / 1e3, 1), round(o / max(1, d), 3)))
    out = {"proxy_dispatches": len(prox), "proxy_us_total": round(tot / 1e3, 1),
           "overlapped_us": round(ov / 1e3, 1), "overlap_fraction": round(ov / max(1, tot), 3),
           "per_dispatch_us_fraction": per[:40]}
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
