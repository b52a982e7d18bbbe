#!/usr/bin/env python3
"""Summarise tools/pmc_phases.sh output: per-wave counters of k_analyze per phase-stop build."""
import collections
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
for ph in ["d1", "d2", "d3", "d4", "full"]:
    f = d / ph / "run_counter_collection.csv"
    if not f.exists():
        print(ph, "missing")
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "k_analyze" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    w = sum(acc["SQ_WAVES"]) / len(acc["SQ_WAVES"])
    print(ph, " ".join(f"{k.replace('SQ_', '')}={sum(v) / len(v) / w:.0f}" for k, v in sorted(acc.items())
                       if k != "SQ_WAVES"))
t = d / "times.log"
if t.exists():
    print(t.read_text())
