#!/usr/bin/env python3
"""Per-phase wall time of k_analyze_w waves inside the real steady state (csrc/Makefile `wstamps`): lane 0 of
the first 2^18 waves stores s_memtime after each phase.  Runs the bench workload (pipelined executes: the
assembly and the next norm stage co-run as in the bench), then prints the median / mean cycles per phase
over the waves that ran the full LPC path, and the mean number of waves resident over the stamped span.
--fine: the FRA_WSTAMP_FINE build (forced waits split the load phase: metadata, raw rows, LUT gathers).
Usage: wstamp_phases.py [config] [level] [--serial] [--fine]"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "flac-raster_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

from flac_raster import _native as N  # noqa: E402

N._LIB_PATH = ROOT / "flac-raster_amd" / "flac_raster" / "_lib" / "diag" / (
    "libflac_raster_amd_wstampsfine.so" if "--fine" in sys.argv else "libflac_raster_amd_wstamps.so")
import bench  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
cfgname = args[0] if args else "c4"
cfg = dict(bench.CONFIGS[cfgname])
if len(args) > 1:
    cfg["level"] = int(args[1])
KW, KN = 1 << 18, 16
NAMES = ["load + LUT + reduce", "wasted/FIXED sums", "FIXED searches", "autocorrelation", "Levinson + quantise",
         "LPC sums + search", "exact pass", "encode + slot"]
STOPS = [0, 1, 2, 3, 4, 5, 6, 7, 8]

ctx = N.Context(0)
lib = N.load()
lib.fra_diag_wstamps.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong]
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
assert lib.fra_diag_wstamps(None, 0) == 0
for i in range(3):  # the stamped execute runs between two others (pipelined co-runners on both sides)
    plan.execute()
    if i == 0:
        plan.sync()
        assert lib.fra_diag_wstamps(None, 0) == 0
plan.sync()
st = np.zeros(KW * KN, np.uint64)
assert lib.fra_diag_wstamps(st.ctypes.data, st.nbytes) == 0
st = st.reshape(KW, KN).astype(np.int64)
full = np.all(st[:, STOPS] > 0, axis=1)
d = np.diff(st[full][:, STOPS], axis=1)
tot = st[full, 8] - st[full, 0]
print(f"{cfgname} level {cfg['level']}: {int(full.sum())} waves with every stamp (of {int((st[:, 0] > 0).sum())} started)")
print(f"{'phase':28s} {'median cyc':>11s} {'mean cyc':>10s} {'share':>7s}")
for k, nm in enumerate(NAMES):
    print(f"{nm:28s} {np.median(d[:, k]):11.0f} {d[:, k].mean():10.0f} {d[:, k].mean() / tot.mean():7.3f}")
print(f"{'wave total':28s} {np.median(tot):11.0f} {tot.mean():10.0f}")
if "--fine" in sys.argv:  # load phase split: 0 -> 10 metadata, 10 -> 11 raw rows, 11 -> 12 gathers + LDS, 12 -> 1 reduce
    sel = full & np.all(st[:, [10, 11, 12]] > 0, axis=1)
    seq = st[sel][:, [0, 10, 11, 12, 1]]
    dd = np.diff(seq, axis=1)
    for k, nm in enumerate(["  load: metadata", "  load: raw rows", "  load: LUT gathers + LDS", "  load: reductions"]):
        print(f"{nm:28s} {np.median(dd[:, k]):11.0f} {dd[:, k].mean():10.0f}")
why = st[:, 9][st[:, 0] > 0]
names = {1: "partial frame", 2: "no LPC model", 3: "FIXED wins", 4: "other LPC window wins", 5: "residual >= 2^17",
         6: "not below VERBATIM", 7: "encode would overrun"}
hb = {names.get(int(k), str(k)): int((why == k).sum()) for k in np.unique(why) if k}
print(f"sample-path (non-kept) subframes: {int((why > 0).sum())} of {len(why)} stamped waves: {hb}")
s0 = st[full, 0]
span = st[full, 8].max() - s0.min()
print(f"stamped span {span} cycles; mean resident (stamped) waves {tot.sum() / span:.1f}")
plan.close()
ctx.free(dev)
