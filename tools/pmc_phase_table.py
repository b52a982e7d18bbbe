#!/usr/bin/env python3
"""Per-wave VALU / SALU / LDS instructions and wave cycles of k_analyze for each diagnostic stop collected by
tools/pmc_valu_phases.sh:  pmc_phase_table.py gpurun_out/<tag>"""
import collections
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
for s in sorted(d.glob("s*"), key=lambda p: p.name):
    f = next(s.rglob("*counter_collection.csv"), None)
    if f is None:
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "k_analyze" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not acc.get("SQ_WAVES"):
        continue
    i = max(range(len(acc["SQ_WAVES"])), key=lambda k: acc["SQ_WAVES"][k])  # the scene launch
    w = acc["SQ_WAVES"][i]
    print(f"stop {s.name[1:]:5s} waves {w:10.0f} " + " ".join(
        f"{k.replace('SQ_INSTS_', '').replace('SQ_', '')}={v[i] / w:8.1f}" for k, v in sorted(acc.items()) if k != "SQ_WAVES"))
