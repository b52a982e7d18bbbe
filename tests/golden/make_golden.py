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
    for name in ["sample_rgb.tif", "sample_rgb.flac", "sample_dem.tif", "sample_multispectral.tif"]:
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
    print("wrote", HERE)


class _Shape:
    """Shape-only stand-in (calculate_audio_params reads .ndim and .shape only)."""

    def __init__(self, shape):
        self.shape = shape
        self.ndim = len(shape)
        self.size = int(np.prod(shape))


if __name__ == "__main__":
    main()
