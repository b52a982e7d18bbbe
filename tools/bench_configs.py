#!/usr/bin/env python3
"""All five BASELINE.json configurations on one MI355X (companion to bench.py, which reports C4).

C1 sample_dem.tif 512^2 int16 and C2 sample_rgb.tif 256^2x3 uint8 (standard format, one stream):
device-resident raster -> frames, K repeats timed (launch-latency bound at this size).
C3/C4/C5: `bench.py --config cN --no-cpu --no-e2e` (synthetic rasters of the named shapes).
Writes one JSON object per config to stdout (and --out FILE)."""
import argparse
import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "flac-raster_amd"))


def small(name, tif, level=5, reps=200):
    import numpy as np
    from flac_raster import _native as N
    from flac_raster.tiff import read_geotiff
    data, _ = read_geotiff(ROOT / "tests" / "golden" / tif)
    B, H, W = data.shape
    ctx = N.Context(0)
    dev = ctx.alloc(data.nbytes)
    ctx.h2d(dev, np.ascontiguousarray(data))
    plan = N.Plan(ctx, dev, True, data.dtype, B, (H * W, W, 1), [(0, 0, H, W)], level, 4096, 16)
    for _ in range(10):
        plan.execute()
    plan.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        plan.execute()
    plan.sync()
    dt = (time.perf_counter() - t0) / reps
    infos, total = plan.result()
    plan.close()
    ctx.free(dev)
    out = {"config": name, "pixels": H * W, "bands": B, "ms_per_encode": round(dt * 1e3, 4),
           "mpix_per_s": round(H * W / dt / 1e6, 2), "frame_bytes": int(total), "level": level}
    if tif == "sample_rgb.tif":
        out["size_ratio_vs_libflac"] = round(total / 178857.0, 5)
    return out


def big(cfg, steps):
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--config", cfg, "--no-cpu", "--no-e2e",
                        "--steps", str(steps), "--warmup", "1"], capture_output=True, text=True, timeout=900)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    return {"config": cfg.upper(), "workload": d["config"]["workload"], "mpix_per_s": d["value"],
            "ms_per_step": d["ms_per_step"], "compressed_bytes": d["config"]["compressed_bytes"],
            "compression_ratio": d["config"]["compression_ratio"], "kernel_ms": d["roofline"]["kernel_ms_per_launch"],
            "analyze_roofline_frac": d["roofline"]["frac"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = [small("C1 sample_dem.tif 512x512x1 int16 -c 5", "sample_dem.tif"),
           small("C2 sample_rgb.tif 256x256x3 uint8 -c 5", "sample_rgb.tif"),
           big("c3", 10), big("c4", 20), big("c5", 3)]
    for r in res:
        print(json.dumps(r), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
