#!/usr/bin/env python3
"""Same-box A/B of the pipelined step: ab_step.py <config> <lib.so|-> [NAME=VALUE ...]

Environment assignments are applied before the plan is created (FRA_CHUNK_MB, FRA_ANALYZE_WG, ...);
SHARD=R/N encodes only rank R's frame-split share of the scene (bench.py --shard).
Prints the serial per-kernel times (timing mode, 5 executes) and the pipelined step time (median of
5 runs of 20 back-to-back executes, wall clock around a sync), plus the output size as a bytes check."""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "flac-raster_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

from flac_raster import _native as N  # noqa: E402

cfgname = sys.argv[1] if len(sys.argv) > 1 else "c4"
if len(sys.argv) > 2 and sys.argv[2] != "-":
    N._LIB_PATH = Path(sys.argv[2]).resolve()
envs = [a for a in sys.argv[3:] if "=" in a]
for kv in envs:
    k, v = kv.split("=", 1)
    os.environ[k] = v
import bench  # noqa: E402

cfg = dict(bench.CONFIGS[cfgname])
ctx = N.Context(0)
B, H, W = cfg["bands"], cfg["H"], cfg["W"]
dt = np.dtype(cfg["dtype"])
dev = ctx.alloc(B * H * W * dt.itemsize)
ctx.synth(cfg["kind"], bench.SEED, B, H, W, dev)
wins = bench.tiles(H, W, cfg["tile"])
ranges = None
shard = os.environ.get("SHARD")  # R/N: rank R's frame-split share (bench.py --shard)
if shard:
    from flac_raster.tiles import frame_split
    sr, sn = (int(x) for x in shard.split("/"))
    pc = os.environ.get("SHARD_COST")  # partial_cost override (tiles.PARTIAL_FRAME_COST)
    items = (frame_split(wins, sn, partial_cost=int(pc)) if pc else frame_split(wins, sn))[sr]
    wins = [wins[i] for i, _, _ in items]
    ranges = [(f0, n) for _, f0, n in items]
plan = N.Plan(ctx, dev, True, dt, B, (H * W, W, 1), wins, cfg["level"], 4096, cfg["norm"], frame_ranges=ranges)
plan.execute(); plan.sync()
plan.enable_timing(True)
for _ in range(5):
    plan.execute()
plan.sync()
ms, n = plan.timing()
plan.enable_timing(False)
K = 20 if cfgname != "c5" else 4
steps = []
for _ in range(5):
    plan.execute(); plan.execute(); plan.sync()
    t0 = time.perf_counter()
    for _ in range(K):
        plan.execute()
    plan.sync()
    steps.append((time.perf_counter() - t0) * 1e3 / K)
_, total = plan.result()
print(f"{N._LIB_PATH.name:34s} {' '.join(envs) or '-':22s} analyze {ms[1]/n:7.3f}  scan {ms[2]/n:6.3f}  "
      f"pack {ms[3]/n:6.3f}  step {np.median(steps):7.3f} ms (min {min(steps):.3f})  out {total}", flush=True)
