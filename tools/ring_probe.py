#!/usr/bin/env python3
"""Ring-path e2e alone (bench.measure_e2e_ring) for one config: ring_probe.py <config> [NAME=VALUE ...]
(environment assignments applied before the library loads, e.g. FRA_D2H_THREADS=1)."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "flac-raster_amd"))
sys.path.insert(0, str(ROOT))
for kv in sys.argv[2:]:
    k, v = kv.split("=", 1)
    os.environ[k] = v
import numpy as np  # noqa: E402

import bench  # noqa: E402
from flac_raster import _native as N  # noqa: E402

cfg = dict(bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c5"])
ctx = N.Context(0)
B, H, W = cfg["bands"], cfg["H"], cfg["W"]
dt = np.dtype(cfg["dtype"])
dev = ctx.alloc(B * H * W * dt.itemsize)
ctx.synth(cfg["kind"], bench.SEED, B, H, W, dev)
wins = bench.tiles(H, W, cfg["tile"])
plan = N.Plan(ctx, dev, True, dt, B, (H * W, W, 1), wins, cfg["level"], 4096, cfg["norm"])
plan.execute()
plan.sync()
r = bench.measure_e2e_ring(N, ctx, cfg, dt, B, H, W, wins, H * W, dev, plan)
print(json.dumps({"env": sys.argv[2:], **{k: r[k] for k in ("ms", "value", "bytes_equal_device_path", "pcie_floor_ms",
                                                           "ratio_vs_pcie_floor", "producer_copy_gbs")}}), flush=True)
