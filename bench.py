#!/usr/bin/env python3
"""bench.py -- FLAC raster encode throughput on MI355X (driver contract: one JSON line on rank 0).

Workload (default ``--config c4``, the north-star configuration of BASELINE.json):
  C4  Sentinel-2 L1C-like 10980 x 10980 x 4 uint16 raster, ``--streaming --tile-size 1024``,
      ``-c 5``: 121 tiles -> 121 independent FLAC streams (100 x 1024^2, 20 x 1024x740, 1 x 740^2).
A *step* = one pass of the encode hot path over the whole scene: device-resident raster in HBM ->
per-tile nanmin/nanmax -> normalize_to_audio -> FLAC analysis -> bit-packed frames of every tile
in HBM (the bytes the reference's pyflac/libFLAC calls produce per tile, cli.py:553-622).
Multi-GPU (one process per GPU, torch.distributed.run): weak scaling by default -- every rank
encodes its own C4 scene (seed 20260227 + rank, generated in its HBM), i.e. the job is N scenes
sharded one per GPU with no collective on the data path; ``value`` = pixels of all ranks' scenes /
max-over-ranks time.  ``--scaling strong`` instead splits ONE scene's tiles over the ranks (LPT on
pixel count).

Also reported: ``roofline`` of the dominant kernel (HIP events on the plan's stream, algorithmic
bytes = input raster bytes + emitted frame bytes of the units one launch processes), and
``cpu_baseline`` = the CPU oracle (oracle/, C port, 1 core) timed on a bounded sample of the same
scene, whose bytes are also checked against the GPU's (in-run parity).
"""

from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "flac-raster_amd"))

CONFIGS = {
    "c3": dict(kind=3, bands=1, H=16384, W=16384, dtype=np.int16, tile=512, level=5, norm=16,
               workload="C3 synthetic DEM 16384x16384x1 int16, --streaming --tile-size 512, -c 5"),
    "c4": dict(kind=4, bands=4, H=10980, W=10980, dtype=np.uint16, tile=1024, level=5, norm=16,
               workload="C4 Sentinel-2 L1C-like 10980x10980x4 uint16, --streaming --tile-size 1024, -c 5"),
    "c5": dict(kind=5, bands=8, H=32768, W=32768, dtype=np.float32, tile=512, level=8, norm=24,
               workload="C5 multispectral 32768x32768x8 float32 (normalize->int32, 32-bps), --streaming "
                        "--tile-size 512, -c 8"),
}
SEED = 20260227
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip-level parameters)


def tiles(H, W, t):
    return [(r, c, min(t, H - r), min(t, W - c)) for r in range(0, H, t) for c in range(0, W, t)]


def lpt_shard(wins, nranks):
    """Longest-processing-time static assignment of tiles to ranks (deterministic)."""
    order = sorted(range(len(wins)), key=lambda i: (-(wins[i][2] * wins[i][3]), i))
    load = [0] * nranks
    owner = [0] * len(wins)
    for i in order:
        r = min(range(nranks), key=lambda k: (load[k], k))
        owner[i] = r
        load[r] += wins[i][2] * wins[i][3]
    return owner


def cpu_baseline(cfg, wins, gpu_frames, gpu_infos, budget_s):
    """Time the CPU oracle (C port of the encode path, 1 thread) on the first tiles of the scene
    until ~budget_s of CPU work; verify its bytes equal the GPU's for those tiles."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O  # test/baseline infrastructure only
    from flac_raster.synth import synth_window

    px = 0
    t_cpu = 0.0
    checked = 0
    mismatches = 0
    for idx, (r0, c0, h, w) in enumerate(wins):
        tile = synth_window(cfg["kind"], SEED, cfg["bands"], cfg["H"], cfg["W"], r0, c0, h, w)
        t0 = time.perf_counter()
        inter = tile.transpose(1, 2, 0).reshape(-1, cfg["bands"])
        audio, _, _ = O.normalize(inter, 16 if cfg["norm"] == 16 else 24)
        frames = O.encode(audio, O.sample_rate_for_pixels(h * w), level=cfg["level"], with_header=False)
        t_cpu += time.perf_counter() - t0
        px += h * w
        if idx in gpu_infos:
            info = gpu_infos[idx]
            checked += 1
            if gpu_frames[info.offset: info.offset + info.frame_bytes] != frames:
                mismatches += 1
        if t_cpu >= budget_s:
            break
    return dict(value=px / t_cpu / 1e6, seconds=t_cpu, pixels=px, tiles=idx + 1, checked=checked,
                mismatches=mismatches)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--level", type=int, default=None)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU oracle work (rank 0)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the in-run rocprofv3 counter passes")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.level is not None:
        cfg["level"] = args.level

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_mod
        # RCCL over xGMI on a GPU node; FRA_DIST_BACKEND=gloo rehearses several ranks on one GPU
        backend = os.environ.get("FRA_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist_mod.init_process_group(backend=backend)
        dist = dist_mod

    from flac_raster import _native as N

    def barrier():
        if dist is not None:
            dist.barrier()

    def allmax(x: float) -> float:
        if dist is None:
            return x
        import torch
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def allsum(x: float) -> float:
        if dist is None:
            return x
        import torch
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    ctx = N.Context(local if N.device_count() > local else 0)
    B, H, W = cfg["bands"], cfg["H"], cfg["W"]
    dt = np.dtype(cfg["dtype"])
    raster_bytes = B * H * W * dt.itemsize
    dev_raster = ctx.alloc(raster_bytes)
    weak = args.scaling == "weak"
    ctx.synth(cfg["kind"], SEED + (rank if weak else 0), B, H, W, dev_raster)
    wins = tiles(H, W, cfg["tile"])
    owner = [rank] * len(wins) if weak else lpt_shard(wins, world)
    mine = [i for i in range(len(wins)) if owner[i] == rank]
    my_wins = [wins[i] for i in mine]
    plan = N.Plan(ctx, dev_raster, True, dt, B, (H * W, W, 1), my_wins, cfg["level"], 4096, cfg["norm"])

    for _ in range(args.warmup):
        plan.execute()
    plan.sync()
    barrier()
    plan.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.execute()  # frame groups pipelined over streams
    plan.sync()
    t1 = time.perf_counter()
    barrier()
    dt_s = t1 - t0
    T = allmax(dt_s)
    # per-kernel launch times (roofline): the same steps again, serial, HIP events between kernels
    plan.enable_timing(True)
    for _ in range(args.steps):
        plan.execute()
    plan.sync()
    kms, nexec = plan.timing()
    plan.enable_timing(False)
    infos, total = plan.result()
    my_px = sum(w[2] * w[3] for w in my_wins)
    my_in_bytes = my_px * B * dt.itemsize
    out_bytes_all = allsum(float(total))

    # dominant kernel: the larger of analyze (1) and pack (3); algorithmic bytes per launch =
    # input bytes + frame bytes of the units this rank's launch processes
    per_launch_ms = [k / max(1, nexec) for k in kms]
    dom = 1 if per_launch_ms[1] >= per_launch_ms[3] else 3
    dom_name = {1: "k_analyze", 3: "k_pack"}[dom]
    alg_bytes = my_in_bytes + total
    achieved = alg_bytes / (per_launch_ms[dom] * 1e-3) / 1e9
    step_ms_local = sum(per_launch_ms)
    path_gbps = alg_bytes / (step_ms_local * 1e-3) / 1e9

    traffic = None
    tfile = ROOT / "profiles" / f"traffic_{args.config}_l{cfg['level']}_n{world}.json"
    if tfile.exists():
        try:
            traffic = json.loads(tfile.read_text()).get(dom_name)
        except Exception:
            traffic = None

    result = None
    if rank == 0:
        scene_px = H * W
        job_px = scene_px * (world if weak else 1)
        value = job_px * args.steps / T / 1e6
        cpu = None
        if not args.no_cpu and world >= 1:
            _, frames = plan.download()
            gi = {i: infos[j] for j, i in enumerate(mine)}
            cb = cpu_baseline(cfg, wins, frames, gi, args.cpu_budget)
            cpu = {"value": round(cb["value"], 3), "unit": "MPix/s", "cores": 1, "kind": "port",
                   "sample": f"first {cb['tiles']} tiles ({cb['pixels']} px, {cb['seconds']:.1f} s) of the same "
                             f"scene through oracle/fr_oracle.c normalize+encode (FRA-1, 1 thread, "
                             f"{platform.processor() or platform.machine()}, os.cpu_count()={os.cpu_count()}); "
                             f"bytes equal to GPU for {cb['checked'] - cb['mismatches']}/{cb['checked']} tiles"}
        # PCIe-inclusive end-to-end (not `value`): host numpy raster -> H2D -> encode -> D2H frames
        e2e = None
        if not args.no_e2e:
            host = np.empty((B, H, W), dtype=dt)
            ctx.d2h(host, dev_raster)
            p2 = N.Plan(ctx, host.ctypes.data, False, dt, B, (H * W, W, 1), my_wins, cfg["level"], 4096, cfg["norm"],
                        keepalive=host)
            p2.execute()
            p2.download()
            reps = 3
            t0e = time.perf_counter()
            for _ in range(reps):
                p2.set_raster(host.ctypes.data, False, keepalive=host)
                p2.execute()
                _, fr2 = p2.download()
            te = (time.perf_counter() - t0e) / reps
            e2e = {"value": round(my_px / te / 1e6, 2), "unit": "MPix/s", "ms": round(te * 1e3, 2),
                   "what": "pageable host raster -> H2D -> all kernels -> D2H of all frames (1 GPU)",
                   "bytes_equal_device_path": bool(fr2 == plan.download()[1])}
            p2.close()
            del host
        # size vs libFLAC: only pinned for C2 (sample_rgb, 178,857 frame bytes at -c 5)
        size_c2 = None
        try:
            from flac_raster.tiff import read_geotiff
            rgb, _ = read_geotiff(ROOT / "tests" / "golden" / "sample_rgb.tif")
            _, fr = N.encode_windows(rgb, [(0, 0, 256, 256)], level=5, norm=16, device=ctx.device)
            size_c2 = round(len(fr) / 178857.0, 5)
        except Exception:
            size_c2 = None
        result = {
            "metric": "raster MPixels/sec encoded at -c 5 + size ratio vs libFLAC, 1/2/4/8 GPU",
            "value": round(value, 2),
            "unit": "MPix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(T / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u16->i16 (int32 analysis, f32 chunk partials + f64 autocorr tree)" if cfg["norm"] == 16 else "f32->i32 (int64 analysis)",
            "data": "synthetic (flac_raster.synth, seed 20260227; device-generated, integer-exact numpy mirror)",
            "config": {"workload": cfg["workload"], "level": cfg["level"], "tiles": len(wins),
                       "raster_bytes": raster_bytes, "compressed_bytes": int(out_bytes_all),
                       "compression_ratio": round(raster_bytes * (world if weak else 1) / max(1.0, out_bytes_all), 4),
                       "msamples_per_s": round(job_px * B * args.steps / T / 1e6, 1),
                       "parallelism": (f"{world} scene(s), one per GPU, no collective" if weak else
                                       f"one scene's tiles sharded LPT over {world} GPU(s), no collective"),
                       "frame_groups": int(os.environ.get("FRA_GROUPS", "1")),
                       "serial_ms_per_step": round(step_ms_local, 4)},
            "roofline": {"bound": "hbm", "kernel": dom_name, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": traffic,
                         "alg_bytes_per_launch": int(alg_bytes),
                         "kernel_ms_per_launch": {"minmax": round(per_launch_ms[0], 4),
                                                  "analyze": round(per_launch_ms[1], 4),
                                                  "frame_bytes+scan": round(per_launch_ms[2], 4),
                                                  "pack": round(per_launch_ms[3], 4)},
                         "whole_path_gbps": round(path_gbps, 2)},
            "cpu_baseline": cpu,
            "size_ratio_vs_libflac_c2": size_c2,
            "e2e": e2e,
        }
        print(json.dumps(result), flush=True)
    plan.close()
    ctx.free(dev_raster)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
