#!/usr/bin/env python3
"""Per-phase wall time of k_analyze workgroups inside the real steady state (csrc/Makefile `stamps`):
wave 0 of the first 2^17 workgroups stores s_memtime after every phase barrier of the fast path.  Runs the
bench workload (pipelined executes, so k_assemble and the next norm stage co-run as in the bench), then
prints the median / mean cycles of each phase over the workgroups that took the fast path.
Usage: stamp_phases.py [config] [level] [--serial] [--fine]   (--fine: the load phase split by the
stampsfine build: metadata loaded / raw samples landed / LUT values landed / LDS + wave reductions)"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "flac-raster_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

from flac_raster import _native as N  # noqa: E402

FINE = "--fine" in sys.argv
N._LIB_PATH = ROOT / "flac-raster_amd" / "flac_raster" / "_lib" / "diag" / (
    "libflac_raster_amd_stampsfine.so" if FINE else "libflac_raster_amd_stamps.so")
import bench  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
cfgname = args[0] if args else "c4"
cfg = dict(bench.CONFIGS[cfgname])
if len(args) > 1:
    cfg["level"] = int(args[1])
KWG, KN = 1 << 17, 20
NAMES = ["load+normalise+reduce", "FIXED sums", "autocorrelation", "LD/quantise + FIXED search",
         "LPC residual sums", "partition search", "winner residuals + Rice sums", "exact bits + scan",
         "encode", "slot write"]

ctx = N.Context(0)
lib = N.load()
lib.fra_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong]
B, H, W = cfg["bands"], cfg["H"], cfg["W"]
dt = np.dtype(cfg["dtype"])
dev = ctx.alloc(B * H * W * dt.itemsize)
ctx.synth(cfg["kind"], bench.SEED, B, H, W, dev)
wins = bench.tiles(H, W, cfg["tile"])
plan = N.Plan(ctx, dev, True, dt, B, (H * W, W, 1), wins, cfg["level"], 4096, cfg["norm"])
if "--serial" in sys.argv:
    plan.enable_timing(True)
for _ in range(4):
    plan.execute()
plan.sync()
assert lib.fra_diag_stamps(None, 0) == 0
for _ in range(3):  # the stamped execute runs between two others (pipelined co-runners on both sides)
    plan.execute()
    if _ == 0:
        plan.sync()
        assert lib.fra_diag_stamps(None, 0) == 0
plan.sync()
st = np.zeros(KWG * KN, np.uint64)
assert lib.fra_diag_stamps(st.ctypes.data, st.nbytes) == 0
st = st.reshape(KWG, KN).astype(np.int64)
fast = np.all(st[:, :11] > 0, axis=1)
d = np.diff(st[fast, :11], axis=1)
tot = st[fast, 10] - st[fast, 0]
print(f"{cfgname} level {cfg['level']}: {int(fast.sum())} fast-path workgroups stamped of {min(KWG, len(plan.frames) if hasattr(plan, 'frames') else KWG)}")
print(f"{'phase':32s} {'median cyc':>11s} {'mean cyc':>10s} {'share':>7s}")
for k, nm in enumerate(NAMES):
    print(f"{nm:32s} {np.median(d[:, k]):11.0f} {d[:, k].mean():10.0f} {d[:, k].mean() / tot.mean():7.3f}")
print(f"{'workgroup total':32s} {np.median(tot):11.0f} {tot.mean():10.0f}")
if FINE:
    f = st[fast]
    ok = np.all(f[:, 11:15] > 0, axis=1)
    f = f[ok]
    sub = [("metadata (frame, stream, norm)", 0, 11), ("raw sample loads", 11, 12), ("LUT gathers", 12, 13),
           ("LDS stores + wave reductions", 13, 14), ("barrier (other waves)", 14, 1)]
    print(f"load phase split over {len(f)} workgroups (LUT path):")
    for nm, a, b in sub:
        x = f[:, b] - f[:, a]
        print(f"  {nm:34s} {np.median(x):9.0f} {x.mean():9.0f}")
if FINE:  # per-role finish times inside the Levinson-Durbin phase (from its start, stamp 3) and the search
    f = st[fast]
    for nm, k, a in (("LD/quantise wave done", 15, 3), ("FIXED search wave 1 done", 16, 3),
                     ("FIXED search wave 2 done", 17, 3), ("LD phase barrier passed", 4, 3),
                     ("LPC search wave done", 18, 5), ("search barrier passed", 6, 5)):
        ok = (f[:, k] > 0) & (f[:, a] > 0)
        if ok.any():
            x = f[ok, k] - f[ok, a]
            print(f"  {nm:34s} {np.median(x):9.0f} {x.mean():9.0f}  ({int(ok.sum())} workgroups)")
span = st[fast, 10].max() - st[fast, 0].min()
print(f"launch span of stamped workgroups: {span} cycles; mean concurrent workgroups {tot.sum() / span:.1f}")
plan.close()
ctx.free(dev)
