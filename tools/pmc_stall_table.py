#!/usr/bin/env python3
"""Stall table from tools/pmc_stall_phases.sh output: per phase stop, k_analyze counters per wave (median
launch) and the WAVE_CYCLES split WAIT_ANY (parked: s_waitcnt / barrier) + WAIT_INST_ANY (issue stall) +
ACTIVE_INST_ANY (issuing), plus the per-phase deltas.  Usage: pmc_stall_table.py <dir> [kernel]
(kernel k_analyze_w: the phase names of its FRA_WSTOP builds)"""
import csv
import sys
from pathlib import Path

ORDER = ["1", "9", "8", "2", "3", "5", "6", "7", "4", "full"]
NAMES = {"1": "load+normalise", "9": "FIXED sums", "8": "autocorrelation", "2": "LD/quantise (+FIXED search)",
         "3": "LPC residual sums", "5": "partition search", "6": "winner residuals + Rice sums",
         "7": "exact bits + scan", "4": "(slow path)", "full": "encode + slot write"}
WORDER = ["1", "2", "3", "4", "5", "6", "7", "full"]
WNAMES = {"1": "load + LUT + reduce", "2": "FIXED sums", "3": "FIXED guesses", "4": "autocorrelation",
          "5": "Levinson + quantise", "6": "LPC sums + searches", "7": "winner exact pass", "full": "encode + slot"}


def load(d, kernel):
    acc = {}
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            acc.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = {}
    for k, v in acc.items():
        vals = sorted(v.values())
        out[k] = vals[len(vals) // 2]
    return out


def main():
    d = Path(sys.argv[1])
    kernel = sys.argv[2] if len(sys.argv) > 2 else "k_analyze"
    global NAMES
    order = ORDER
    if kernel == "k_analyze_w":
        order, NAMES = WORDER, WNAMES
    rows = []
    for s in order:
        a, b = d / f"a{s}", d / f"b{s}"
        if not a.exists():
            continue
        c = load(a, kernel)
        c.update({k: v for k, v in load(b, kernel).items() if k != "SQ_WAVES"})
        w = c.get("SQ_WAVES", 0) or 1
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        rows.append((s, {
            "valu/w": c.get("SQ_INSTS_VALU", 0) / w, "salu/w": c.get("SQ_INSTS_SALU", 0) / w,
            "lds/w": c.get("SQ_INSTS_LDS", 0) / w, "vmem/w": c.get("SQ_INSTS_VMEM", 0) / w,
            "wcyc/w": wc / w, "wait": c.get("SQ_WAIT_ANY", 0) / w, "winst": c.get("SQ_WAIT_INST_ANY", 0) / w,
            "act": c.get("SQ_ACTIVE_INST_ANY", 0) / w, "actvalu": c.get("SQ_ACTIVE_INST_VALU", 0) / w,
            "winstlds": c.get("SQ_WAIT_INST_LDS", 0) / w, "bankc": c.get("SQ_LDS_BANK_CONFLICT", 0) / w,
            "actlds": c.get("SQ_ACTIVE_INST_LDS", 0) / w, "actsca": c.get("SQ_ACTIVE_INST_SCA", 0) / w,
            "busy": c.get("SQ_BUSY_CYCLES", 0)}))
    cols = ["valu/w", "salu/w", "lds/w", "wcyc/w", "wait", "winst", "act", "actvalu", "winstlds", "bankc"]
    print(f"k_analyze per wave ({kernel}; SQ cycle counters in quad-cycles per wave, median launch)")
    print(f"{'stop':>5} {'phase':30s}" + "".join(f"{c:>10s}" for c in cols) + "   wait% winst% act%")
    prev = None
    for s, r in rows:
        print(f"{s:>5} {NAMES.get(s, s):30s}" + "".join(f"{r[c]:10.1f}" for c in cols) +
              f"   {100 * r['wait'] / r['wcyc/w']:5.1f} {100 * r['winst'] / r['wcyc/w']:5.1f} {100 * r['act'] / r['wcyc/w']:5.1f}")
    print("\nper-phase deltas (this stop minus the previous one)")
    print(f"{'stop':>5} {'phase':30s}" + "".join(f"{c:>10s}" for c in cols))
    for s, r in rows:
        if prev is not None:
            print(f"{s:>5} {NAMES.get(s, s):30s}" + "".join(f"{r[c] - prev[c]:10.1f}" for c in cols))
        else:
            print(f"{s:>5} {NAMES.get(s, s):30s}" + "".join(f"{r[c]:10.1f}" for c in cols))
        prev = r


if __name__ == "__main__":
    main()
