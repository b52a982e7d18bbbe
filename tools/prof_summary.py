#!/usr/bin/env python3
"""Summarise one tools/profile_config.sh run into committed profile files.

usage: prof_summary.py gpurun_out/<tag> <tag> [config]
writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.txt            per kernel: launches, median HBM traffic per launch (FETCH_SIZE x2 +
                                    WRITE_SIZE, MI355X_MICROARCH.md: gfx950 FETCH_SIZE counts 1/2 of wide
                                    reads; KiB -> bytes) and per-wave instruction counts (SQ_* / SQ_WAVES)
  profiles/traffic_<config>.json    {kernel: bytes per launch, "sources_sha": hash of csrc/} read by bench.py
"""
import collections
import csv
import hashlib
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def sources_sha():
    """Hash of the kernel sources: a committed traffic file is only valid for the build it measured."""
    h = hashlib.sha256()
    for p in sorted((ROOT / "flac-raster_amd" / "csrc").glob("*")):
        if p.suffix in (".hip", ".h", ".cpp"):
            h.update(p.name.encode())
            h.update(p.read_bytes())
    return h.hexdigest()[:16]


def short(name):
    return name.replace("void ", "").split("(")[0].replace("fra::", "")


def counters(d):
    f = next(d.rglob("*counter_collection.csv"), None)
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    if f is None:
        return acc
    for r in csv.DictReader(open(f)):
        acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else 0.0


def main():
    src, tag = Path(sys.argv[1]), sys.argv[2]
    cfg = sys.argv[3] if len(sys.argv) > 3 else None
    prof = ROOT / "profiles"
    fetch = counters(src / "pmc_fetch")
    write = counters(src / "pmc_write")
    valu = counters(src / "valu")
    lines = [f"# {tag}: rocprofv3 PMC passes of bench.py --config {cfg} (tools/profile_config.sh); one pass per "
             "counter group",
             "# traffic = FETCH_SIZE x2 + WRITE_SIZE per launch (median launch; KiB -> bytes; gfx950 FETCH_SIZE "
             "counts 1/2 of wide coalesced reads)",
             "# kernel | launches | fetch MB | write MB | traffic MB | per wave: VALU SALU LDS VMEM_RD VMEM_WR | waves"]
    traffic = {}
    names = sorted(set(fetch) | set(write) | set(valu))
    for k in names:
        f = med(fetch[k].get("FETCH_SIZE", [])) * 1024 * 2
        w = med(write[k].get("WRITE_SIZE", [])) * 1024
        n = len(fetch[k].get("FETCH_SIZE", [])) or len(valu[k].get("SQ_WAVES", []))
        v = valu[k]
        waves = med(v.get("SQ_WAVES", [])) or 0.0

        def pw(c):
            return med(v.get(c, [])) / waves if waves else 0.0
        lines.append(f"{k[:44]:44s} {n:4d} {f / 1e6:10.2f} {w / 1e6:10.2f} {(f + w) / 1e6:10.2f} | "
                     f"{pw('SQ_INSTS_VALU'):8.1f} {pw('SQ_INSTS_SALU'):7.1f} {pw('SQ_INSTS_LDS'):6.1f} "
                     f"{pw('SQ_INSTS_VMEM_RD'):6.1f} {pw('SQ_INSTS_VMEM_WR'):6.1f} | {waves:.0f}")
        base = k.split("<")[0]
        if f + w > traffic.get(base, 0):
            traffic[base] = int(f + w)
    (prof / f"{tag}_pmc.txt").write_text("\n".join(lines) + "\n")
    stats = next((src / "stats").rglob("*kernel_stats.csv"), None)
    if stats:
        shutil.copy(stats, prof / f"{tag}_kernel_stats.csv")
    if cfg:
        traffic["sources_sha"] = sources_sha()
        traffic["source"] = f"profiles/{tag}_pmc.txt"
        (prof / f"traffic_{cfg}.json").write_text(json.dumps(traffic, indent=1) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
