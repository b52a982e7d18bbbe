"""flac_raster -- MI355X-native (gfx950 HIP) FLAC encoder for rasters, API-compatible with
yharby/flac-raster's ``flac_raster`` package on the encode path.

Importing needs no GPU; every encode call goes through ``libflac_raster_amd.so`` and raises
``NativeUnavailable`` when the library or a device is missing (there is no CPU fallback).
"""

__version__ = "0.2.0"

from .compare import compare_tiffs, display_comparison_table  # noqa: E402
from .converter import RasterFLACConverter  # noqa: E402
from .normalization import (  # noqa: E402
    NormalizationParams,
    calculate_audio_params,
    denormalize_from_audio,
    estimate_precision_loss,
    normalize_to_audio,
)
from .spatial_encoder import SpatialFLACEncoder, SpatialFLACStreamer, SpatialIndex  # noqa: E402

__all__ = [
    "RasterFLACConverter", "compare_tiffs", "display_comparison_table", "SpatialFLACEncoder",
    "SpatialFLACStreamer", "SpatialIndex", "normalize_to_audio", "denormalize_from_audio",
    "calculate_audio_params", "NormalizationParams", "estimate_precision_loss",
]
