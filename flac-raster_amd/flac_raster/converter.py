"""``RasterFLACConverter`` (API of the reference's ``converter.py``) on the MI355X encoder.

``tiff_to_flac`` (``converter.py:41-172``): the whole raster is one encode unit.  Where the
reference does ``src.read()`` -> interleave -> ``normalize_to_audio`` -> ``pyflac.StreamEncoder``
-> mutagen, this does one GPU plan with one window (normalisation fused, no interleave copy) and
writes ``fLaC``/STREAMINFO/VORBIS_COMMENT(tags)/PADDING/frames with the mutagen-equivalent
writer (``flac_meta.rewrite_header``).

``flac_to_tiff`` (``converter.py:174-261``) decodes with the native decoder under pyflac
FileDecoder's PCM_16 semantics (F8) and denormalises like the reference.
"""

from __future__ import annotations

import json
import logging
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
from rich.console import Console

from . import flac_meta
from .decoder import FileDecoder
from .geo import Affine, bounds as geo_bounds
from .normalization import NormalizationParams, calculate_audio_params, denormalize_from_audio
from .tiff import GeoTIFF, write_geotiff
from .tiles import TileStream, encode_tiles

console = Console()

ENCODER_TAG = "FLAC-Raster v0.1.0"  # converter.py:272 / spatial_encoder.py:333


def raster_tags(metadata: Dict) -> List[Tuple[str, str]]:
    """Tag list and order of ``_embed_metadata_in_flac`` (``converter.py:269-294``)."""
    return [
        ("TITLE", "Geospatial Raster Data"),
        ("DESCRIPTION", "TIFF raster converted to FLAC with geospatial metadata"),
        ("ENCODER", ENCODER_TAG),
        ("GEOSPATIAL_CRS", str(metadata.get("crs", ""))),
        ("GEOSPATIAL_WIDTH", str(metadata.get("width", 0))),
        ("GEOSPATIAL_HEIGHT", str(metadata.get("height", 0))),
        ("GEOSPATIAL_COUNT", str(metadata.get("count", 1))),
        ("GEOSPATIAL_DTYPE", str(metadata.get("dtype", ""))),
        ("GEOSPATIAL_NODATA", str(metadata.get("nodata", ""))),
        ("GEOSPATIAL_DATA_MIN", str(metadata.get("data_min", ""))),
        ("GEOSPATIAL_DATA_MAX", str(metadata.get("data_max", ""))),
        ("GEOSPATIAL_TRANSFORM", json.dumps(metadata.get("transform", []))),
        ("GEOSPATIAL_BOUNDS", json.dumps(metadata.get("bounds", []))),
        ("GEOSPATIAL_SPATIAL_TILING", str(metadata.get("spatial_tiling", False))),
    ]


def raster_metadata(width: int, height: int, count: int, dtype, crs: Optional[str], transform: Affine,
                    data_min: float, data_max: float, nodata=None, scale_factor: int = 32767) -> Dict:
    """The ``raster_metadata`` dict of ``converter.py:114-134``."""
    left, bottom, right, top = geo_bounds(transform, width, height)
    return {
        "width": width, "height": height, "count": count, "dtype": str(np.dtype(dtype)),
        "crs": crs if crs else None,
        "transform": list(transform),
        "bounds": {"left": left, "bottom": bottom, "right": right, "top": top},
        "data_min": data_min, "data_max": data_max, "nodata": nodata, "driver": "GTiff",
        "scale_factor": scale_factor,
    }


def tagged_stream(ts: TileStream, metadata: Dict) -> bytes:
    """A GPU-encoded stream with the converter's tags embedded (what tiff_to_flac writes)."""
    return flac_meta.rewrite_header(ts.data, raster_tags(metadata))


class RasterFLACConverter:
    """TIFF <-> FLAC conversion (``converter.py:34-400``)."""

    def __init__(self, devices: Optional[Sequence[int]] = None):
        self.metadata_key = "RASTER_METADATA"
        self.logger = logging.getLogger("flac_raster.converter")
        self.devices = list(devices) if devices else None

    def tiff_to_flac(self, tiff_path: Path, flac_path: Path, compression_level: int = 5,
                     spatial_tiling: bool = False, tile_size: int = 512):
        tiff_path, flac_path = Path(tiff_path), Path(flac_path)
        self.logger.info(f"Starting TIFF to FLAC conversion: {tiff_path} -> {flac_path}")
        if spatial_tiling:
            from .spatial_encoder import SpatialFLACEncoder

            console.print("[cyan]Using spatial tiling for HTTP range streaming[/cyan]")
            enc = SpatialFLACEncoder(tile_size=tile_size, devices=self.devices)
            return enc.encode_spatial_flac(tiff_path, flac_path, compression_level)
        console.print(f"[cyan]Reading TIFF file: {tiff_path}[/cyan]")
        g = GeoTIFF(tiff_path)
        data = g.read()
        info = g.info
        sample_rate, bps = calculate_audio_params(data, data.dtype)
        console.print(f"[green]Raster info: {info.width}x{info.height}, {info.count} band(s), "
                      f"dtype: {info.dtype}[/green]")
        console.print(f"[yellow]Using sample rate: {sample_rate}Hz, bit depth: {bps}[/yellow]")
        ts = encode_tiles(data, [(0, 0, info.height, info.width)], compression_level, self.devices)[0]
        assert ts.sample_rate == sample_rate
        meta = raster_metadata(info.width, info.height, info.count, data.dtype, info.crs, Affine(*info.transform),
                               ts.data_min, ts.data_max, info.nodata, 32767 if bps == 16 else 8388607)
        self.logger.info(f"Data range: [{ts.data_min}, {ts.data_max}]")
        flac_path.write_bytes(ts.data)
        self._embed_metadata_in_flac(flac_path, meta)
        out_size = flac_path.stat().st_size
        ratio = (1 - out_size / tiff_path.stat().st_size) * 100
        console.print(f"[green]SUCCESS: Converted to FLAC: {flac_path}[/green]")
        console.print(f"[dim]File size: {out_size / 1024 / 1024:.2f} MB (compression: {ratio:.1f}%)[/dim]")
        return None

    def flac_to_tiff(self, flac_path: Path, tiff_path: Path):
        flac_path, tiff_path = Path(flac_path), Path(tiff_path)
        console.print(f"[cyan]Reading FLAC file: {flac_path}[/cyan]")
        audio, sample_rate = FileDecoder(flac_path).process()
        md = self._read_embedded_metadata(flac_path)
        if not md:
            raise ValueError("No metadata found in FLAC file or sidecar file")
        width, height, count = md["width"], md["height"], md["count"]
        if count > 1:
            raster = audio.reshape(height, width, count).transpose(2, 0, 1)
        else:
            raster = audio.reshape(height, width)
        params = NormalizationParams(md["data_min"], md["data_max"], str(np.dtype(md["dtype"])),
                                     16 if raster.dtype == np.int16 else 24,
                                     md.get("scale_factor", 32767 if raster.dtype == np.int16 else 8388607))
        out = denormalize_from_audio(raster, params)
        t = md.get("transform")
        write_geotiff(tiff_path, out, transform=tuple(t[:6]) if t else None, crs=md.get("crs") or None,
                      nodata=md.get("nodata"))
        console.print(f"[green]SUCCESS: Converted to TIFF: {tiff_path}[/green]")

    def _embed_metadata_in_flac(self, flac_path: Path, metadata: Dict):
        flac_meta.embed_tags_file(flac_path, raster_tags(metadata))

    def _read_embedded_metadata(self, flac_path: Path) -> Optional[Dict]:
        """Typed geospatial fields from the tags (``converter.py:329-379``), else the .json sidecar."""
        try:
            f = flac_meta.FLACFile(flac_path)
            if "GEOSPATIAL_CRS" not in f:
                raise ValueError("No embedded metadata found")
            md: Dict = {}
            for field in ("CRS", "WIDTH", "HEIGHT", "COUNT", "DTYPE", "NODATA", "DATA_MIN", "DATA_MAX", "TRANSFORM",
                          "BOUNDS", "SPATIAL_TILING"):
                key = "GEOSPATIAL_" + field
                if key not in f:
                    continue
                v = f[key][0]
                k = field.lower()
                if k in ("width", "height", "count"):
                    md[k] = int(v) if v else 0
                elif k in ("data_min", "data_max"):
                    md[k] = float(v) if v else 0.0
                elif k in ("transform", "bounds"):
                    md[k] = json.loads(v) if v else []
                elif k == "spatial_tiling":
                    md[k] = v.lower() == "true"
                elif k == "nodata":
                    md[k] = None if v == "None" else (float(v) if v else None)
                else:
                    md[k] = v
            return md
        except Exception as e:
            self.logger.warning(f"Failed to read embedded metadata: {e}")
            side = Path(flac_path).with_suffix(".json")
            if side.exists():
                return json.loads(side.read_text())
        return None
