#!/usr/bin/env python3
"""Per-kernel summary of a PMC campaign (scripts/passes/r05_pmc_cnn.sh: p1.txt, p2.txt from
scripts/pmc_table.py): time, MFMA-busy, LDS bank-conflict share, wait share, VALU per MFMA.

usage: python scripts/pmc_summary.py <dir with p1.txt p2.txt> [min_us]

MFMA-busy = SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CU_CYCLES / 4 (four SIMDs per CU);
LDS conflicts = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; waiting = SQ_WAIT_INST_ANY /
SQ_WAVE_CYCLES; VALU/MFMA = SQ_INSTS_VALU / SQ_INSTS_MFMA (SQ_INSTS_VALU counts the MFMAs too).
"""
import os
import sys


def parse(path):
    out, cur = {}, None
    if not os.path.exists(path):
        return out
    for line in open(path):
        if not line.startswith("   "):
            cur = line.strip()
            out.setdefault(cur, {})
        elif cur is not None:
            name, val = line.split()
            out[cur][name] = float(val)
    return out


def main():
    d = sys.argv[1]
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    p1, p2 = parse(os.path.join(d, "p1.txt")), parse(os.path.join(d, "p2.txt"))
    rows = []
    for k, c in p1.items():
        if not c.get("SQ_INSTS_MFMA"):
            continue
        c2 = p2.get(k, {})
        us = c.get("_ns", 0) / 1e3
        if us < min_us:
            continue
        busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(c["SQ_BUSY_CU_CYCLES"], 1) / 4 * 100
        conf = c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1) * 100
        wait = c["SQ_WAIT_INST_ANY"] / max(c["SQ_WAVE_CYCLES"], 1) * 100
        vpm = c2.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_MFMA"]
        rows.append((us, k, busy, conf, wait, vpm))
    print(f"{'kernel':60s} {'us':>7s} {'MFMA-busy%':>10s} {'LDSconf%':>8s} {'wait%':>6s} {'VALU/MFMA':>9s}")
    for us, k, busy, conf, wait, vpm in sorted(rows, reverse=True):
        print(f"{k:60s} {us:7.1f} {busy:10.1f} {conf:8.1f} {wait:6.1f} {vpm:9.2f}")


if __name__ == "__main__":
    main()
