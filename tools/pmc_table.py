#!/usr/bin/env python3
"""Per-wave averages of every counter collected by tools/pmc_stalls.sh for one kernel."""
import collections, csv, sys
from pathlib import Path
d, kern = Path(sys.argv[1]), (sys.argv[2] if len(sys.argv) > 2 else "k_analyze")
for f in sorted(d.glob("p*/run_counter_collection.csv")):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    w = sum(acc["SQ_WAVES"]) / max(1, len(acc["SQ_WAVES"]))
    print(f.parent.name, " ".join(f"{k}={sum(v)/len(v)/w:.1f}/wave" for k, v in sorted(acc.items()) if k != "SQ_WAVES"))
