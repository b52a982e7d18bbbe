#!/usr/bin/env python3
"""Is the k_analyze_w instance or the measurement order behind the bench line's ms_per_step_forced_17bit < ms_per_step?
Alternates timed segments of 20 pipelined C4 executes: adaptive (16-bit after settling) and forced 17-bit, 4 times."""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "flac-raster_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

from flac_raster import _native as N  # noqa: E402
import bench  # noqa: E402

cfg = dict(bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4"])
ctx = N.Context(0)
B, H, W = cfg["bands"], cfg["H"], cfg["W"]
dt = np.dtype(cfg["dtype"])
dev = ctx.alloc(B * H * W * dt.itemsize)
ctx.synth(cfg["kind"], bench.SEED, B, H, W, dev)
plan = N.Plan(ctx, dev, True, dt, B, (H * W, W, 1), bench.tiles(H, W, cfg["tile"]), cfg["level"], 4096, cfg["norm"])
plan.execute()
plan.sync()
for _ in range(3):
    plan.execute()
plan.sync()
for rnd in range(4):
    for mode in ("auto", "17", "16"):
        if mode == "auto":
            os.environ.pop("FRA_KEEP17", None)
        else:
            os.environ["FRA_KEEP17"] = "1" if mode == "17" else "0"
        plan.execute()
        plan.sync()
        t0 = time.perf_counter()
        inst = []
        for _ in range(20):
            plan.execute()
            inst.append(17 if plan.flags() & 8 else 16)
        plan.sync()
        ms = (time.perf_counter() - t0) / 20 * 1e3
        print(f"round {rnd} {mode:4s} instance {sorted(set(inst))} step {ms:.4f} ms", flush=True)
os.environ.pop("FRA_KEEP17", None)
plan.close()
ctx.free(dev)
