#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (run in the BUILD container only).

Sources (reference = /root/reference, yharby/flac-raster @ 2026-02-27, read-only):
  * test_data/sample_rgb.tif, sample_rgb.flac, sample_dem.tif, sample_multispectral.tif are
    copied verbatim (data files the reference's own tests/CI use; MIT licensed).
  * The reference's ``src/flac_raster/normalization.py`` is imported BY FILE PATH (pure numpy)
    and run on
      - the three sample TIFFs after the converter's band interleave (converter.py:99-110),
      - per-dtype random vectors and edge cases (constant, NaN, +-inf, all-NaN, extremes),
    to produce (input, expected output, mn, mx) vectors.  The reference code itself is never
    copied; only its outputs are stored.
  * ``calculate_audio_params`` outputs for representative shapes/dtypes.

The GPU box never reads /root/reference: tests there use only these fixtures.
"""

from __future__ import annotations

import hashlib
import importlib.util
import json
import shutil
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
REF = Path("/root/reference")
sys.path.insert(0, str(REPO / "flac-raster_amd"))

from flac_raster.tiff import read_geotiff  # noqa: E402


def load_ref_normalization():
    spec = importlib.util.spec_from_file_location(
        "ref_normalization", REF / "src" / "flac_raster" / "normalization.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    norm = load_ref_normalization()
    meta = {"generator": "tests/golden/make_golden.py", "reference": "yharby/flac-raster@2026-02-27",
            "tiffs": {}, "audio_params": []}
    for name in ["sample_rgb.tif", "sample_rgb.flac", "sample_dem.tif", "sample_dem.flac", "sample_multispectral.tif"]:
        shutil.copyfile(REF / "test_data" / name, HERE / name)

    # --- sample TIFFs through interleave + reference normalize (converter.py:93-113)
    for name in ["sample_rgb.tif", "sample_dem.tif", "sample_multispectral.tif"]:
        data, info = read_geotiff(HERE / name)
        sr, bps = norm.calculate_audio_params(data, data.dtype)
        C = data.shape[0]
        inter = data.transpose(1, 2, 0).reshape(-1, C)
        audio, p = norm.normalize_to_audio(inter, bps)
        meta["tiffs"][name] = {
            "shape": list(data.shape), "dtype": str(data.dtype), "sample_rate": sr, "bps": bps,
            "data_min": p.data_min, "data_max": p.data_max, "audio_dtype": str(audio.dtype),
            "raw_sha256": sha(data), "audio_sha256": sha(audio),
            "audio_head": audio[:8].tolist(), "transform": list(info.transform), "crs": info.crs,
        }

    # --- per-dtype vectors
    rng = np.random.default_rng(20260227)
    vec = {}
    cases = []
    for dt in ["uint8", "int8", "uint16", "int16", "uint32", "int32"]:
        ii = np.iinfo(dt)
        cases.append((f"{dt}_full", rng.integers(ii.min, ii.max, size=4096, endpoint=True, dtype=dt)))
        cases.append((f"{dt}_narrow", rng.integers(5, 120, size=4096, dtype=dt)))
        cases.append((f"{dt}_const", np.full(777, ii.max // 3, dtype=dt)))
        cases.append((f"{dt}_extremes", np.array([ii.min, ii.max, ii.min, 0 if ii.min < 0 else ii.min + 1, ii.max], dtype=dt)))
    for dt in ["float32", "float64"]:
        f = rng.normal(0.15, 0.1, size=4096).astype(dt)
        cases.append((f"{dt}_refl", f))
        g = f.copy(); g[::97] = np.nan
        cases.append((f"{dt}_nan", g))
        h = f.copy(); h[5] = np.inf; h[9] = -np.inf
        cases.append((f"{dt}_inf", h))
        cases.append((f"{dt}_allnan", np.full(100, np.nan, dtype=dt)))
        cases.append((f"{dt}_const", np.full(100, 0.25, dtype=dt)))
        cases.append((f"{dt}_wide", (rng.standard_normal(4096) * 1e6).astype(dt)))
        cases.append((f"{dt}_tiny", (rng.standard_normal(4096) * 1e-30).astype(dt)))
    import warnings
    for name, x in cases:
        for bps in (16, 24):
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                a, p = norm.normalize_to_audio(x.reshape(-1, 1), bps)
            vec[f"{name}__{bps}__in"] = x
            vec[f"{name}__{bps}__out"] = a.reshape(-1)
            vec[f"{name}__{bps}__mnmx"] = np.array([p.data_min, p.data_max], dtype=np.float64)
    np.savez_compressed(HERE / "normalize_vectors.npz", **vec)

    for dt in ["uint8", "int8", "uint16", "int16", "uint32", "int32", "float32", "float64"]:
        for shape in [(1, 512, 512), (3, 999, 1000), (4, 1024, 1024), (1, 3163, 3163), (1, 10000, 10000), (2, 10980, 10980)]:
            sr, bps = norm.calculate_audio_params(_Shape(shape), np.dtype(dt))
            meta["audio_params"].append({"dtype": dt, "shape": list(shape), "sample_rate": sr, "bps": bps})
    (HERE / "golden.json").write_text(json.dumps(meta, indent=1, sort_keys=True))
    extra_vectors(norm)
    print("wrote", HERE)


def extra_vectors(norm):
    """normalize_to_audio with data_min/data_max overrides and the bps-32 fallback,
    denormalize_from_audio (int16 / int32 / float64 PCM_16-style inputs) and
    estimate_precision_loss -> normalize_extra.npz + precision_loss.json."""
    import warnings
    rng = np.random.default_rng(77)
    vec = {}
    x16 = rng.integers(0, 10000, size=3000).astype(np.uint16)
    xf = rng.normal(0.2, 0.1, size=3000).astype(np.float32)
    xi = rng.integers(-2**31, 2**31 - 1, size=3000, dtype=np.int64).astype(np.int32)
    over = [("u16_override", x16, 16, 100.0, 9000.0), ("u16_override_lo", x16, 24, -5.5, None),
            ("f32_override_hi", xf, 24, None, 0.25), ("i32_bps32", xi, 32, None, None),
            ("u16_bps32", x16, 32, None, None), ("f32_inverted", xf, 16, 0.5, 0.1)]
    for name, x, bps, lo, hi in over:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            a, p = norm.normalize_to_audio(x.reshape(-1, 1), bps, lo, hi)
        vec[f"norm__{name}__in"] = x
        vec[f"norm__{name}__out"] = a.reshape(-1)
        vec[f"norm__{name}__args"] = np.array([bps, np.nan if lo is None else lo, np.nan if hi is None else hi,
                                               p.data_min, p.data_max], dtype=np.float64)
    cases = [
        ("i16", rng.integers(-32767, 32768, size=2000).astype(np.int16), 100.0, 9000.0, "uint16", 16, 32767),
        ("i16_i8", rng.integers(-32767, 32768, size=2000).astype(np.int16), -128.0, 127.0, "int8", 16, 32767),
        ("i32", rng.integers(-8388607, 8388608, size=2000).astype(np.int32), -3.5, 1e6, "float32", 24, 8388607),
        ("i32_u32", rng.integers(-8388607, 8388608, size=2000).astype(np.int32), 0.0, 4e9, "uint32", 24, 8388607),
        ("f64_pcm16", rng.integers(-32768, 32768, size=2000).astype(np.float64) / 32768.0, 577.0, 1492.0,
         "int16", 24, 8388607),
        ("f64_float", rng.uniform(-1, 1, size=2000), 0.0, 0.4, "float64", 24, 8388607),
    ]
    for name, a, lo, hi, odt, bps, scale in cases:
        p = norm.NormalizationParams(lo, hi, odt, bps, scale)
        out = norm.denormalize_from_audio(a, p)
        vec[f"denorm__{name}__in"] = a
        vec[f"denorm__{name}__out"] = out
        vec[f"denorm__{name}__params"] = np.array([lo, hi, bps, scale], dtype=np.float64)
        vec[f"denorm__{name}__dtype"] = np.array(odt)
    np.savez_compressed(HERE / "normalize_extra.npz", **vec)
    rows = []
    for dt in ["uint8", "int8", "uint16", "int16", "uint32", "int32", "float32", "float64"]:
        for lo, hi in [(0.0, 255.0), (-1000.5, 30000.25), (0.0, 0.0), (577.0, 1492.0)]:
            for bps in (16, 24, 32):
                rows.append({"dtype": dt, "min": lo, "max": hi, "bps": bps,
                             "out": norm.estimate_precision_loss(np.dtype(dt), lo, hi, bps)})
    (HERE / "precision_loss.json").write_text(json.dumps(rows, indent=0))


class _Shape:
    """Shape-only stand-in (calculate_audio_params reads .ndim and .shape only)."""

    def __init__(self, shape):
        self.shape = shape
        self.ndim = len(shape)
        self.size = int(np.prod(shape))


if __name__ == "__main__":
    if "--extra-only" in sys.argv:
        extra_vectors(load_ref_normalization())
    else:
        main()
