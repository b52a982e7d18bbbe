"""``--spatial`` format: concatenated per-tile FLAC streams + gzip/base64 JSON index in the tags.

API of the reference's ``spatial_encoder.py``: ``SpatialFrame``, ``SpatialIndex``,
``SpatialFLACEncoder.encode_spatial_flac`` (``:155-258``) and the read side
``SpatialFLACStreamer`` (``:410-567``, local files; remote URLs are out of scope here).

Encode: all tiles in one batched GPU plan (``tiles.encode_tiles``) instead of one pyflac encoder
per tile.  File layout is the reference's: tile streams back to back (each the raw 86-byte
libFLAC-style header + frames), index offsets = running sum of stream sizes measured BEFORE the
tag rewrite grows the first stream's header (stale by design), then the
mutagen-equivalent tag rewrite of the first header (``:309-375``).
"""

from __future__ import annotations

import base64
import gzip
import json
import logging
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
from rich.console import Console

from . import flac_meta
from .converter import ENCODER_TAG
from .geo import CRS, Affine, Window
from .tiff import GeoTIFF
from .tiles import calculate_tiles, encode_tiles

console = Console()


class SpatialFrame:
    """One tile: id, bbox (xmin, ymin, xmax, ymax), pixel window, byte range."""

    def __init__(self, frame_id: int, bbox: Tuple[float, float, float, float], window: Window, byte_offset: int = 0,
                 byte_size: int = 0):
        self.frame_id = frame_id
        self.bbox = bbox
        self.window = window
        self.byte_offset = byte_offset
        self.byte_size = byte_size

    def to_dict(self) -> Dict:
        return {
            "frame_id": self.frame_id,
            "bbox": self.bbox,
            "window": {"row_off": self.window.row_off, "col_off": self.window.col_off, "height": self.window.height,
                       "width": self.window.width},
            "byte_offset": self.byte_offset,
            "byte_size": self.byte_size,
        }


class SpatialIndex:
    """Frames + CRS + transform with bbox lookup (``spatial_encoder.py:68-97``)."""

    def __init__(self, frames: List[SpatialFrame], crs, transform: Affine):
        self.frames = frames
        self.crs = crs
        self.transform = transform
        self.total_bytes = sum(f.byte_size for f in frames)

    def query_bbox(self, bbox: Tuple[float, float, float, float]) -> List[SpatialFrame]:
        xmin, ymin, xmax, ymax = bbox
        return [f for f in self.frames
                if xmin < f.bbox[2] and xmax > f.bbox[0] and ymin < f.bbox[3] and ymax > f.bbox[1]]

    def to_dict(self) -> Dict:
        return {"crs": str(self.crs), "transform": list(self.transform),
                "frames": [f.to_dict() for f in self.frames]}


def tile_bbox(transform: Affine, row_off: int, col_off: int, height: int, width: int):
    """``_tile_to_bbox`` (``spatial_encoder.py:123-133``): corners through the affine."""
    xmin, ymax = transform * (col_off, row_off)
    xmax, ymin = transform * (col_off + width, row_off + height)
    return (xmin, ymin, xmax, ymax)


def spatial_tags(index: SpatialIndex, tile_size: int, ntiles: int, width: int, height: int, count: int, dtype,
                 data_min: float, data_max: float, date: Optional[str] = None) -> List[Tuple[str, str]]:
    """Tag list and order of ``spatial_encoder.py:329-369``."""
    boxes = [f.bbox for f in index.frames]
    bnds = [min(b[0] for b in boxes), min(b[1] for b in boxes), max(b[2] for b in boxes), max(b[3] for b in boxes)]
    packed = base64.b64encode(gzip.compress(json.dumps(index.to_dict(), separators=(",", ":")).encode("utf-8")))
    return [
        ("TITLE", "Geospatial Raster Data"),
        ("DESCRIPTION", f"TIFF raster converted to spatial FLAC with {ntiles} tiles"),
        ("ENCODER", ENCODER_TAG),
        ("DATE", date if date is not None else str(np.datetime64("now", "D"))),
        ("GEOSPATIAL_CRS", str(index.crs)),
        ("GEOSPATIAL_WIDTH", str(width)),
        ("GEOSPATIAL_HEIGHT", str(height)),
        ("GEOSPATIAL_COUNT", str(count)),
        ("GEOSPATIAL_DTYPE", str(np.dtype(dtype))),
        ("GEOSPATIAL_DATA_MIN", str(float(data_min))),
        ("GEOSPATIAL_DATA_MAX", str(float(data_max))),
        ("GEOSPATIAL_TRANSFORM", json.dumps(list(index.transform))),
        ("GEOSPATIAL_BOUNDS", json.dumps(bnds)),
        ("GEOSPATIAL_SPATIAL_TILING", "true"),
        ("GEOSPATIAL_TILE_SIZE", str(tile_size)),
        ("GEOSPATIAL_NUM_TILES", str(ntiles)),
        ("GEOSPATIAL_SPATIAL_INDEX", packed.decode("ascii")),
    ]


class SpatialFLACEncoder:
    """Tiled encoder (``spatial_encoder.py:100-407``), all tiles in one batched GPU plan."""

    def __init__(self, tile_size: int = 512, devices: Optional[Sequence[int]] = None):
        self.tile_size = tile_size
        self.devices = list(devices) if devices else None
        self.logger = logging.getLogger("flac_raster.spatial_encoder")
        self.frames: List[SpatialFrame] = []
        self.current_frame_id = 0
        self.bytes_written = 0
        self.output_file = None

    def _calculate_tiles(self, height: int, width: int) -> List[Tuple[int, int, int, int]]:
        return calculate_tiles(height, width, self.tile_size)

    def _tile_to_bbox(self, row_off, col_off, height, width, transform):
        return tile_bbox(transform, row_off, col_off, height, width)

    def encode_spatial_flac(self, tiff_path: Path, flac_path: Path, compression_level: int = 5,
                            enable_streaming: bool = True) -> SpatialIndex:
        g = GeoTIFF(tiff_path)
        raster = g.read()
        info = g.info
        transform = Affine(*info.transform)
        crs = CRS(info.crs) if info.crs else None
        tiles = self._calculate_tiles(info.height, info.width)
        streams = encode_tiles(raster, tiles, compression_level, self.devices)
        self.frames, self.bytes_written = [], 0
        for i, ((r, c, h, w), ts) in enumerate(zip(tiles, streams)):
            fr = SpatialFrame(i, self._tile_to_bbox(r, c, h, w, transform), Window(c, r, w, h), self.bytes_written,
                              len(ts.data))
            self.frames.append(fr)
            self.bytes_written += len(ts.data)
        index = SpatialIndex(self.frames, crs, transform)
        body = b"".join(ts.data for ts in streams)
        tags = spatial_tags(index, self.tile_size, len(tiles), info.width, info.height, raster.shape[0], raster.dtype,
                            float(np.min(raster)), float(np.max(raster)))
        Path(flac_path).write_bytes(flac_meta.rewrite_header(body, tags))
        console.print(f"[green]SUCCESS: Encoded {len(tiles)} spatial tiles to FLAC: {flac_path}[/green]")
        return index


class SpatialFLACStreamer:
    """Byte-range access to a ``--spatial`` file by bbox (local files)."""

    def __init__(self, flac_path):
        if isinstance(flac_path, str) and flac_path.startswith(("http://", "https://", "s3://", "az://", "gs://")):
            raise NotImplementedError("remote URLs are outside this build's scope; download the file first")
        self.flac_path = Path(flac_path)
        self.is_remote = self.is_url = False
        self.logger = logging.getLogger("flac_raster.spatial_streamer")
        self.spatial_index = self._load_spatial_index()

    def _load_spatial_index(self) -> SpatialIndex:
        try:
            f = flac_meta.FLACFile(self.flac_path)
            if "GEOSPATIAL_SPATIAL_INDEX" not in f:
                raise ValueError("No embedded spatial index found")
            data = json.loads(gzip.decompress(base64.b64decode(f["GEOSPATIAL_SPATIAL_INDEX"][0])).decode("utf-8"))
        except Exception as e:
            self.logger.warning(f"Failed to read embedded metadata: {e}")
            side = self.flac_path.with_suffix(".spatial.json")
            if not side.exists():
                raise FileNotFoundError(f"Spatial index not found in FLAC metadata or sidecar file: {side}")
            data = json.loads(side.read_text())
        frames = [SpatialFrame(d["frame_id"], tuple(d["bbox"]),
                               Window(d["window"]["col_off"], d["window"]["row_off"], d["window"]["width"],
                                      d["window"]["height"]), d["byte_offset"], d["byte_size"])
                  for d in data["frames"]]
        return SpatialIndex(frames, CRS.from_string(data["crs"]), Affine(*data["transform"][:6]))

    def get_byte_ranges_for_bbox(self, bbox) -> List[Tuple[int, int]]:
        ranges = sorted((f.byte_offset, f.byte_offset + f.byte_size - 1)
                        for f in self.spatial_index.query_bbox(bbox) if f.byte_size > 0)
        merged: List[Tuple[int, int]] = []
        for s, e in ranges:
            if merged and s <= merged[-1][1] + 1:
                merged[-1] = (merged[-1][0], max(merged[-1][1], e))
            else:
                merged.append((s, e))
        return merged

    def stream_bbox_data(self, bbox) -> bytes:
        chunks = []
        with open(self.flac_path, "rb") as f:
            for s, e in self.get_byte_ranges_for_bbox(bbox):
                f.seek(s)
                chunks.append(f.read(e - s + 1))
        return b"".join(chunks)
