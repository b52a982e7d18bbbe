#!/usr/bin/env python3
"""Oracle size study: the working tree's FRA-1 rule against the one of a git revision (default HEAD).

usage: size_study.py [REV]
Builds REV's oracle into /tmp/fra_size_study/REV and encodes, with both, C1 (sample_dem) and C2 (sample_rgb) at
level 5, tiles of the C3 / C4 bench scenes (level 5), a two-band stereo window at levels 5 and 8 and a C5-like
float32 window at level 8; prints the frame bytes of each and the ratio.  Test infrastructure only (the oracle)."""
import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "flac-raster_amd"), str(ROOT)]
import oracle as O  # noqa: E402
from flac_raster.synth import synth_window  # noqa: E402
from flac_raster.tiff import read_geotiff  # noqa: E402

rev = sys.argv[1] if len(sys.argv) > 1 else "HEAD"
out = Path("/tmp/fra_size_study") / rev
out.mkdir(parents=True, exist_ok=True)
src = subprocess.run(["git", "-C", str(ROOT), "show", f"{rev}:oracle/fr_oracle.c"], check=True,
                     capture_output=True).stdout
(out / "fr_oracle.c").write_bytes(src)
subprocess.run(["gcc", "-O2", "-std=c99", "-D_GNU_SOURCE", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-shared",
                "-o", str(out / "libfr_oracle.so"), str(out / "fr_oracle.c"), "-lm"], check=True)
old = C.CDLL(str(out / "libfr_oracle.so"))
for f in ("ora_encode",):
    getattr(old, f).argtypes = O.lib().ora_encode.argtypes
    getattr(old, f).restype = O.lib().ora_encode.restype
old.ora_free.argtypes = [C.c_void_p]


def frame_bytes(L, audio, sr, level, bps):
    x = np.ascontiguousarray(audio.astype(np.int32))
    N, Ch = x.shape
    o = C.POINTER(C.c_uint8)()
    n = C.c_size_t()
    nfr = (N + 4095) // 4096
    fb = np.zeros(max(nfr, 1), dtype=np.int64)
    info = np.zeros((max(nfr, 1), Ch, 4), dtype=np.int32)
    rc = L.ora_encode(O._ptr(x), N, Ch, bps, sr, 4096, level, 0, C.byref(o), C.byref(n), O._ptr(fb), O._ptr(info))
    assert rc == 0
    L.ora_free(o)
    return int(fb[:nfr].sum())


def case(name, tile, level, norm=16):
    inter = tile.transpose(1, 2, 0).reshape(-1, tile.shape[0])
    bps = 16 if norm == 16 else 24
    audio, _, _ = O.normalize(inter, bps)
    sr = O.sample_rate_for_pixels(tile.shape[1] * tile.shape[2])
    sb = 16 if norm == 16 else 32
    a = frame_bytes(old, audio, sr, level, sb)
    b = frame_bytes(O.lib(), audio, sr, level, sb)
    print(f"{name:34s} level {level}  {rev}: {a:>11,d}  tree: {b:>11,d}  ratio {b / a:.5f}", flush=True)
    return a, b


g = ROOT / "tests" / "golden"
tot = [0, 0]
for nm in ("sample_dem", "sample_rgb"):
    d, _ = read_geotiff(g / f"{nm}.tif")
    case(nm, d, 5)
for cfg, kind, bands, H, t, tl in (("c3", 3, 1, 16384, 512, [(0, 0), (8192, 4096), (512 * 31, 512 * 31)]),
                                    ("c4", 4, 4, 10980, 1024, [(0, 0), (5120, 3072), (10240, 10240)])):
    for r0, c0 in tl:
        h, w = min(t, H - r0), min(t, H - c0)
        a, b = case(f"{cfg} tile ({r0},{c0}) {h}x{w}", synth_window(kind, 20260227, bands, H, H, r0, c0, h, w), 5)
        tot[0] += a
        tot[1] += b
st = synth_window(4, 7, 2, 1024, 1024, 0, 0, 512, 512)
case("stereo 2-band 512x512", st, 5)
case("stereo 2-band 512x512", st, 8)
case("c5-like float32 256x256", synth_window(5, 20260227, 2, 4096, 4096, 0, 0, 256, 256), 8, norm=24)
print(f"c3+c4 tiles total ratio {tot[1] / tot[0]:.5f}")
