#!/usr/bin/env python3
"""Turn tools/profile_round.sh output into the committed profile files.

usage: traffic_summary.py gpurun_out/<tag> <tag>
writes profiles/<tag>_kernel_stats.csv, profiles/<tag>_pmc_traffic.txt, profiles/<tag>_bench.json and
profiles/traffic_c4_l5_n1.json (HBM bytes per launch of each kernel, read by bench.py as
roofline.traffic).  FETCH_SIZE is doubled (MI355X_MICROARCH.md: gfx950 reports half of the bytes of
wide coalesced reads); rocprofv3 reports both counters in KiB."""
import collections
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
src, tag = Path(sys.argv[1]), sys.argv[2]
prof = ROOT / "profiles"


def per_kernel(d, counter):
    f = next(d.rglob("*counter_collection.csv"))
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return acc


def short(name):
    s = name.replace("void ", "").split("(")[0]
    return s.replace("fra::", "")


fetch = per_kernel(src / "pmc_fetch", "FETCH_SIZE")
write = per_kernel(src / "pmc_write", "WRITE_SIZE")
lines = ["# rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), python bench.py --steps 3 "
         "--warmup 1 --no-cpu --no-e2e (C4, level 5, 1 GPU)",
         "# FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports 1/2 of wide coalesced reads); counters in KiB -> bytes",
         "# kernel, launches, median over launches: FETCH raw MB/launch, FETCH x2 MB, WRITE MB, traffic MB per launch (fetch x2 + write)"]
traffic = {}
for k in sorted(set(fetch) | set(write), key=short):
    f = fetch.get(k, [0.0])
    w = write.get(k, [0.0])
    fr = sorted(f)[len(f) // 2]  # median launch: the small in-run parity launches are not C4 launches
    wr = sorted(w)[len(w) // 2]
    t = 2 * fr + wr
    lines.append(f"{short(k):40s} {len(f):4d} {fr / 1e6:10.2f} {2 * fr / 1e6:10.2f} {wr / 1e6:10.2f} {t / 1e6:10.2f}")
    nm = short(k)
    base = nm.split("<")[0]
    if base in ("k_analyze", "k_assemble", "k_minmax_vec", "k_minmax", "k_norm_lut"):
        traffic[base] = max(traffic.get(base, 0), int(t))
(prof / f"{tag}_pmc_traffic.txt").write_text("\n".join(lines) + "\n")
traffic["source"] = f"profiles/{tag}_pmc_traffic.txt (FETCH_SIZE x2 + WRITE_SIZE, bytes per launch)"
(prof / "traffic_c4_l5_n1.json").write_text(json.dumps(traffic, indent=1) + "\n")
stats = next((src / "stats").rglob("*kernel_stats.csv"))
shutil.copy(stats, prof / f"{tag}_kernel_stats.csv")
b = (src / "bench.json").read_text().strip().splitlines()
(prof / f"{tag}_bench.json").write_text(b[-1] + "\n")
print("\n".join(lines))
print(open(prof / f"{tag}_kernel_stats.csv").read()[:1500])
