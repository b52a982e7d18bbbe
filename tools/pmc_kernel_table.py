#!/usr/bin/env python3
"""Median per launch of every counter of every kernel in rocprofv3 --pmc output directories.
usage: pmc_kernel_table.py <dir> [<dir> ...]   (counters as reported: FETCH_SIZE / WRITE_SIZE in KiB)"""
import collections
import csv
import sys
from pathlib import Path


def short(name):
    return name.replace("void ", "").split("(")[0].replace("fra::", "").split("<")[0]


acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    parts = []
    for c, v in sorted(acc[k].items()):
        v = sorted(v)
        parts.append(f"{c}={v[len(v) // 2]:.6g} (n={len(v)})")
    print(f"{k:22s} " + "  ".join(parts))
