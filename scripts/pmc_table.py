#!/usr/bin/env python3
"""Per-kernel mean of each PMC counter from rocprofv3 --pmc CSV outputs.
usage: python scripts/pmc_table.py <counter_collection.csv>... [--match substr]"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = None
if "--match" in sys.argv:
    match = sys.argv[sys.argv.index("--match") + 1]
    args.remove(match)
acc = defaultdict(lambda: defaultdict(list))
for path in args:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"][:60]
        if match and match not in k:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        acc[k]["_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        acc[k]["_vgpr"].append(float(r.get("VGPR_Count") or 0) + float(r.get("Accum_VGPR_Count") or 0))
for k, cs in acc.items():
    if len(cs["_ns"]) < 8:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}")
