#!/usr/bin/env python3
"""Phase timing of k_analyze (diagnostic builds, see csrc/Makefile `diag`): run the C4 bench
workload with a given library and print per-kernel ms.  Differences between builds that stop
after phase k give the cost of each phase.  Usage: diag_phases.py [lib.so] [config] [level]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "flac-raster_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

from flac_raster import _native as N  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] != "-":
    N._LIB_PATH = Path(sys.argv[1]).resolve()
cfgname = sys.argv[2] if len(sys.argv) > 2 else "c4"
import bench  # noqa: E402

cfg = dict(bench.CONFIGS[cfgname])
if len(sys.argv) > 3:
    cfg["level"] = int(sys.argv[3])
ctx = N.Context(0)
B, H, W = cfg["bands"], cfg["H"], cfg["W"]
dt = np.dtype(cfg["dtype"])
dev = ctx.alloc(B * H * W * dt.itemsize)
ctx.synth(cfg["kind"], bench.SEED, B, H, W, dev)
wins = bench.tiles(H, W, cfg["tile"])
plan = N.Plan(ctx, dev, True, dt, B, (H * W, W, 1), wins, cfg["level"], 4096, cfg["norm"])
plan.execute(); plan.sync()
plan.enable_timing(True)
for _ in range(5):
    plan.execute()
plan.sync()
ms, n = plan.timing()
_, total = plan.result()
print(f"{N._LIB_PATH.name:40s} minmax {ms[0]/n:8.3f}  analyze {ms[1]/n:8.3f}  scan {ms[2]/n:6.3f}  pack {ms[3]/n:8.3f} ms  out {total}")
