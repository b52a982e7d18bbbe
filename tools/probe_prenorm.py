#!/usr/bin/env python3
"""Probe (GPU box): the 32-bps analysis of a float32 scene normalised inside k_analyze (norm 24) against the same
analysis of an int32 copy already normalised (norm 0: raw integer loads), to bound what moving normalize_to_audio
out of the analysis could gain.  Usage: probe_prenorm.py [config]  (c5q default)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "flac-raster_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from flac_raster import _native as N  # noqa: E402

cfg = dict(bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c5q"])
ctx = N.Context(0)
B, H, W = cfg["bands"], cfg["H"], cfg["W"]
dev = ctx.alloc(B * H * W * 4)
ctx.synth(cfg["kind"], bench.SEED, B, H, W, dev)
host = np.empty((B, H, W), np.float32)
ctx.d2h(host, dev)
aud, _, _ = ctx.normalize(host, 24)
aud = np.ascontiguousarray(aud.reshape(B, H, W).astype(np.int32))
dev32 = ctx.alloc(aud.nbytes)
ctx.h2d(dev32, aud)
del host
wins = bench.tiles(H, W, cfg["tile"])
for name, d, dt, norm in (("float32 norm 24", dev, np.float32, 24), ("int32 norm 0", dev32, np.int32, 0)):
    plan = N.Plan(ctx, d, True, np.dtype(dt), B, (H * W, W, 1), wins, cfg["level"], 4096, norm)
    plan.execute(); plan.sync()
    plan.enable_timing(True)
    for _ in range(5):
        plan.execute()
    plan.sync()
    ms, n = plan.timing()
    _, total = plan.result()
    print(f"{name:16s} minmax {ms[0]/n:7.3f}  analyze {ms[1]/n:7.3f}  pack {ms[3]/n:6.3f} ms  out {total}", flush=True)
    plan.close()
