"""Raster <-> audio-sample mapping (API of the reference's ``normalization.py``).

* ``calculate_audio_params`` / ``get_dtype_info`` / ``estimate_precision_loss`` are host
  arithmetic (``normalization.py:59-123, 256-303``).
* ``normalize_to_audio`` (``normalization.py:126-202``) runs on the GPU (``fra_normalize`` in
  ``csrc/fra_kernels.hip``).  The encoders never call it: they fuse the same arithmetic into
  ``k_analyze``.  There is no CPU fallback: without the HIP library or a
  device it raises ``NativeUnavailable``.
* ``denormalize_from_audio`` (``normalization.py:205-253``) is the read-side inverse, host numpy
  like the reference (8(f) f2/f4: not on the encode path).
"""

from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

logger = logging.getLogger("flac_raster.normalization")

SCALE_16 = 32767
SCALE_24 = 8388607
SCALE_32 = 2147483647


@dataclass
class NormalizationParams:
    """What the decoder needs to undo the mapping (``normalization.py:27-56``)."""

    data_min: float
    data_max: float
    original_dtype: str
    bits_per_sample: int
    scale_factor: int

    def to_dict(self) -> dict:
        return {"data_min": self.data_min, "data_max": self.data_max, "original_dtype": self.original_dtype,
                "bits_per_sample": self.bits_per_sample, "scale_factor": self.scale_factor}

    @classmethod
    def from_dict(cls, d: dict) -> "NormalizationParams":
        return cls(d["data_min"], d["data_max"], d["original_dtype"], d["bits_per_sample"],
                   d.get("scale_factor", SCALE_16))


def scale_for_bps(bits_per_sample: int) -> int:
    return {16: SCALE_16, 24: SCALE_24}.get(bits_per_sample, SCALE_32)


def get_dtype_info(dtype) -> Tuple[Optional[float], Optional[float], bool]:
    """(min, max, is_integer) of a dtype; floats have no fixed range (``normalization.py:59-75``)."""
    dt = np.dtype(dtype)
    if np.issubdtype(dt, np.integer):
        ii = np.iinfo(dt)
        return float(ii.min), float(ii.max), True
    if np.issubdtype(dt, np.floating):
        return None, None, False
    raise ValueError(f"Unsupported dtype: {dt}")


def bits_for_dtype(dtype) -> int:
    """16 for 8/16-bit integers, 24 for everything wider (``normalization.py:92-104``)."""
    dt = np.dtype(dtype)
    if dt in (np.uint8, np.int8, np.uint16, np.int16):
        return 16
    if dt not in (np.uint32, np.int32, np.float32, np.float64):
        logger.warning(f"Unknown dtype {dt}, defaulting to 24-bit")
    return 24


def sample_rate_for_pixels(total_pixels: int) -> int:
    """<1 MP 44.1 kHz, <10 MP 48 kHz, <100 MP 96 kHz, else 192 kHz (``normalization.py:108-120``)."""
    for limit, rate in ((1_000_000, 44100), (10_000_000, 48000), (100_000_000, 96000)):
        if total_pixels < limit:
            return rate
    return 192000


def calculate_audio_params(data: np.ndarray, dtype) -> Tuple[int, int]:
    """(sample_rate, bits_per_sample) for an encode unit; pixels = H*W of the last two axes."""
    total = data.shape[-2] * data.shape[-1] if data.ndim >= 2 else data.size
    return sample_rate_for_pixels(int(total)), bits_for_dtype(dtype)


def normalize_to_audio(data: np.ndarray, bits_per_sample: int, data_min: float = None, data_max: float = None,
                       device: int = 0) -> Tuple[np.ndarray, NormalizationParams]:
    """Map any raster array to int16 (bps 16) / int32 (bps 24 or other) audio samples on the GPU.

    mn/mx = nanmin/nanmax unless given; R = mx - mn (1.0 if mx <= mn);
    y = ((2.0*(x-mn))/R) - 1.0, clip [-1, 1], NaN -> 0, * scale, truncate.
    """
    from . import _native

    a = np.asarray(data)
    ctx = _native.default_context(device)
    audio, mn, mx = ctx.normalize(a, bits_per_sample, data_min, data_max)
    dmin = data_min if data_min is not None else float(mn)
    dmax = data_max if data_max is not None else float(mx)
    if dmax <= dmin:
        logger.warning(f"Data has no range (min={dmin}, max={dmax}), using zeros")
    params = NormalizationParams(dmin, dmax, str(a.dtype), bits_per_sample, scale_for_bps(bits_per_sample))
    return audio, params


def denormalize_from_audio(audio_data: np.ndarray, params: NormalizationParams) -> np.ndarray:
    """Inverse map (read side).  int16 samples use 32767, int32 the stored scale, floats are
    already in [-1, 1] (the PCM_16 decode path); integers round to nearest."""
    a = np.asarray(audio_data)
    if a.dtype == np.int16:
        scale = 32767.0
    elif a.dtype in (np.float32, np.float64):
        scale = 1.0
    else:
        scale = float(params.scale_factor)
    y = a.astype(np.float64) / scale
    span = params.data_max - params.data_min
    x = (y + 1.0) / 2.0 * span + params.data_min
    out_dt = np.dtype(params.original_dtype)
    if np.issubdtype(out_dt, np.integer):
        return np.round(x).astype(out_dt)
    return x.astype(out_dt)


def estimate_precision_loss(original_dtype, data_min: float, data_max: float, bits_per_sample: int) -> dict:
    """Quantisation error bound of the mapping (``normalization.py:256-303``)."""
    dt = np.dtype(original_dtype)
    span = data_max - data_min
    levels = 2 * scale_for_bps(bits_per_sample)
    max_err = span / levels
    rel = (max_err / span) * 100 if span > 0 else 0.0
    lossless = False
    if np.issubdtype(dt, np.integer):
        ii = np.iinfo(dt)
        lossless = (ii.max - ii.min) <= levels
    return {"max_absolute_error": max_err, "relative_error_percent": rel, "quantization_levels": levels,
            "is_lossless": lossless, "bits_per_sample": bits_per_sample}
