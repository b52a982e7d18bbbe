#!/usr/bin/env python3
"""Summarise a rocprofv3 PC-sampling CSV (stochastic or host-trap): samples per instruction (top N), per
stall reason and per instruction type, restricted to one kernel.  usage: pc_summary.py <csv> [kernel] [N]"""
import collections
import csv
import sys

path = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "k_analyze"
topn = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = list(csv.DictReader(open(path)))
if not rows:
    sys.exit("no samples")
cols = list(rows[0].keys())
print("columns:", cols)
kcol = next((c for c in cols if c.lower() in ("kernel_name", "kernel-name", "kernel")), None)
icol = next((c for c in cols if c.lower() == "instruction"), None)
ocol = next((c for c in cols if "offset" in c.lower()), None)
scol = next((c for c in cols if "stall" in c.lower() and "reason" in c.lower()), None)
tcol = next((c for c in cols if "instruction_type" in c.lower() or c.lower() == "inst_type"), None)
wcol = next((c for c in cols if "issued" in c.lower()), None)
if kcol:
    rows = [r for r in rows if kern in r[kcol]]
print(f"{len(rows)} samples for {kern}")
by = collections.Counter((r.get(ocol, ""), r.get(icol, "")) for r in rows)
tot = sum(by.values()) or 1
for (off, ins), n in by.most_common(topn):
    print(f"{n:7d} {100.0 * n / tot:6.2f}%  {off:>10s}  {ins}")
for col, name in ((scol, "stall reason"), (tcol, "instruction type"), (wcol, "wave issued")):
    if col:
        c = collections.Counter(r[col] for r in rows)
        print(f"--- {name}")
        for k, n in c.most_common(20):
            print(f"{n:8d} {100.0 * n / tot:6.2f}%  {k}")
