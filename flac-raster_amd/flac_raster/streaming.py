"""``--streaming`` container: ``[u32 BE index length][compact JSON index][tile FLAC streams]``.

Writer = ``cli._create_streaming_flac`` (``cli.py:521-639``), the north-star path: per tile the
reference writes a temp GeoTIFF, runs ``tiff_to_flac`` on it (normalise, pyflac, mutagen tags of
the TILE: its size, transform, bounds, min/max) and appends the bytes.  Here all tiles are encoded
by one batched GPU plan per device (``tiles.encode_tiles``), and the per-tile tag rewrite is the
same host byte assembly (``flac_meta``) with the values the temp GeoTIFF would have carried:
the window transform (rasterio ``windows.transform`` arithmetic), no nodata, the source CRS.

Reader = the index parse + byte-range slicing of ``cli.extract`` (``cli.py:238-313``).
"""

from __future__ import annotations

import json
import struct
import threading
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import flac_meta
from .converter import raster_metadata, raster_tags
from .geo import Affine, window_transform
from .tiff import GeoTIFF
from .tiles import TileStream, calculate_tiles, encode_tiles, encode_tiles_ring


def tile_flac_parts(ts: TileStream, transform: Affine, crs: Optional[str], row_off: int, col_off: int, height: int,
                    width: int, dtype):
    """One tile's file as ``converter.tiff_to_flac(temp_tile.tif)`` would write it, as (tagged metadata
    bytes, frames view, window transform): the frames are not copied."""
    tt = window_transform(transform, col_off, row_off)
    md = raster_metadata(width, height, ts.channels, dtype, crs, tt, ts.data_min, ts.data_max, None,
                         32767 if ts.bps == 16 else 8388607)
    return flac_meta.rewrite_header_parts(ts.header, len(ts.body), raster_tags(md)), ts.body, tt


def tile_flac_bytes(ts: TileStream, transform: Affine, crs: Optional[str], row_off: int, col_off: int, height: int,
                    width: int, dtype) -> Tuple[bytes, Affine]:
    head, body, tt = tile_flac_parts(ts, transform, crs, row_off, col_off, height, width, dtype)
    return head + bytes(body), tt


def streaming_parts(tiles: Sequence[Tuple[int, int, int, int]], streams: Sequence[TileStream], shape, dtype,
                    transform: Affine, crs: Optional[str], tile_size: int) -> List:
    """The container as a list of bytes-like parts (index first); frames stay zero-copy views."""
    B, H, W = shape
    index: Dict = {"crs": str(crs), "transform": list(transform), "width": W, "height": H, "bands": B,
                   "dtype": str(np.dtype(dtype)), "tile_size": tile_size, "frames": []}
    parts: List = []
    total = 0
    for fid, ((r, c, h, w), ts) in enumerate(zip(tiles, streams)):
        head, body, tt = tile_flac_parts(ts, transform, crs, r, c, h, w, dtype)
        size = len(head) + len(body)
        xmin, ymax = tt.c, tt.f
        index["frames"].append({
            "frame_id": fid,
            "bbox": [xmin, ymax + h * tt.e, xmin + w * tt.a, ymax],
            "window": {"col_off": c, "row_off": r, "width": w, "height": h},
            "byte_offset": total,
            "byte_size": size,
        })
        parts += [head, body]
        total += size
    head = json.dumps(index, separators=(",", ":")).encode("utf-8")
    return [len(head).to_bytes(4, "big") + head] + parts


def assemble_streaming(tiles: Sequence[Tuple[int, int, int, int]], streams: Sequence[TileStream], shape,
                       dtype, transform: Affine, crs: Optional[str], tile_size: int) -> bytes:
    """Container bytes from encoded tile streams (tile order = ``calculate_tiles`` order)."""
    return b"".join(bytes(p) if isinstance(p, memoryview) else p
                    for p in streaming_parts(tiles, streams, shape, dtype, transform, crs, tile_size))


def build_streaming(raster: np.ndarray, transform: Affine, crs: Optional[str], tile_size: int,
                    compression_level: int = 5, devices: Optional[Sequence[int]] = None) -> bytes:
    """Container bytes for a band-planar ``(B, H, W)`` raster (all tiles on the GPU(s))."""
    a = raster if raster.ndim == 3 else raster[None]
    tiles = calculate_tiles(a.shape[1], a.shape[2], tile_size)
    streams = encode_tiles(a, tiles, compression_level, devices)
    return assemble_streaming(tiles, streams, a.shape, a.dtype, transform, crs, tile_size)


def decode_while_encoding(g: GeoTIFF, tile_size: int):
    """Start decoding a GeoTIFF into page-locked memory on a producer thread, top to bottom in row bands
    (one tile row, rounded up to whole TIFF strips/tiles): returns ``(raster, rows_ready, thread)``;
    ``rows_ready[0]`` = rows decoded so far (-1 on failure).  The encoder's host pipeline copies a band
    H2D as soon as its rows are published (``fra_plan_encode_host_progress``), so the decode of band b+1
    overlaps the PCIe copies and kernels of band b."""
    from .tiff import _alloc

    info = g.info
    raster = _alloc((info.count, info.height, info.width), info.dtype, True)
    rows_ready = np.zeros(1, np.int64)
    step = decode_step(g, tile_size)
    errors: list = []

    def run():
        try:
            for r0 in range(0, info.height, step):
                r1 = min(info.height, r0 + step)
                g.read_window_into(raster[:, r0:r1, :], r0, 0, r1 - r0, info.width)
                rows_ready[0] = r1
        except BaseException as e:  # reported to the encoder (rows_ready = -1) and re-raised by the caller
            errors.append(e)
            rows_ready[0] = -1

    th = threading.Thread(target=run, name="geotiff-decode", daemon=True)
    th.errors = errors  # type: ignore[attr-defined]
    th.start()
    return raster, rows_ready, th


def decode_step(g: GeoTIFF, tile_size: int) -> int:
    """Rows per producer step: one tile row, rounded up to whole TIFF strips / tiles."""
    info = g.info
    step = max(tile_size, g.ch)
    return ((step + g.ch - 1) // g.ch) * g.ch if g.ch < info.height else info.height


def encode_geotiff_ring(g: GeoTIFF, tiles, compression_level: int = 5, device: int = 0, tile_size: int = 512,
                        ring_rows: int = 0):
    """GeoTIFF -> tile streams with bounded host memory: the file's row bands are decoded into a
    page-locked ring (``tiles.encode_tiles_ring``) that the pipelined encoder copies from and recycles, so
    the raster is never held whole -- as the reference, which reads one tile window at a time
    (``cli.py:553-559``).  Returns ``(streams, ring_rows)``."""
    info = g.info

    def fill(dst, r0, r1):
        g.read_window_into(dst, r0, 0, r1 - r0, info.width)

    return encode_tiles_ring((info.count, info.height, info.width), info.dtype, tiles, fill, compression_level,
                             device, step=decode_step(g, tile_size), ring_rows=ring_rows)


def encode_geotiff_streaming(input_path: Path, tile_size: int = 512, compression_level: int = 5,
                             devices: Optional[Sequence[int]] = None, ring: bool = True):
    """GeoTIFF file -> (tiles, streams, raster info): decode and encode overlapped.  One device: through
    the bounded ring (``encode_geotiff_ring``); several: the whole raster is decoded into page-locked
    memory (``decode_while_encoding``) and split over the devices."""
    g = GeoTIFF(input_path)
    if ring and (not devices or len(devices) == 1):
        try:
            info = g.info
            tiles = calculate_tiles(info.height, info.width, tile_size)
            streams, _ = encode_geotiff_ring(g, tiles, compression_level, devices[0] if devices else 0, tile_size)
            return tiles, streams, (info.count, info.height, info.width), np.dtype(info.dtype), info
        finally:
            g.close()
    raster, rows_ready, th = decode_while_encoding(g, tile_size)
    try:
        tiles = calculate_tiles(raster.shape[1], raster.shape[2], tile_size)
        try:
            streams = encode_tiles(raster, tiles, compression_level, devices, rows_ready=rows_ready, producer=th)
        finally:
            th.join()
        if th.errors:  # type: ignore[attr-defined]
            raise th.errors[0]  # type: ignore[attr-defined]
        return tiles, streams, raster.shape, raster.dtype, g.info
    finally:
        g.close()


def create_streaming_flac(input_path: Path, output_path: Path, tile_size: int = 512, compression_level: int = 5,
                          devices: Optional[Sequence[int]] = None) -> Dict:
    """Write the streaming container for a GeoTIFF; returns the index.

    The raster is decoded into page-locked memory by a producer thread, row band by row band, while the
    pipelined host path encodes the bands already decoded (H2D, kernels and D2H of band b overlap the
    decode of band b+1); the container is written from zero-copy views of the page-locked frames."""
    tiles, streams, shape, dtype, info = encode_geotiff_streaming(input_path, tile_size, compression_level, devices)
    parts = streaming_parts(tiles, streams, shape, dtype, Affine(*info.transform), info.crs, tile_size)
    with open(output_path, "wb") as f:
        for p in parts:
            f.write(p)
    n = struct.unpack(">I", parts[0][:4])[0]
    return json.loads(parts[0][4:4 + n].decode("utf-8"))


@dataclass
class StreamingFile:
    """Parsed container: index + absolute byte range of every tile."""

    index: Dict
    header_size: int

    def tile_range(self, frame: Dict) -> Tuple[int, int]:
        start = self.header_size + frame["byte_offset"]
        return start, start + frame["byte_size"]


def read_index_bytes(data: bytes) -> Tuple[Dict, int]:
    n = struct.unpack(">I", data[:4])[0]
    return json.loads(data[4:4 + n].decode("utf-8")), 4 + n


def open_streaming(path: Path) -> StreamingFile:
    with open(path, "rb") as f:
        n = struct.unpack(">I", f.read(4))[0]
        idx = json.loads(f.read(n).decode("utf-8"))
    return StreamingFile(idx, 4 + n)


def select_frame(frames: List[Dict], tile_id: Optional[int] = None, bbox: Optional[Sequence[float]] = None,
                 center: bool = False, last: bool = False) -> Dict:
    """Tile choice of ``cli.extract`` (``cli.py:245-296``)."""
    if tile_id is not None:
        fr = next((f for f in frames if f["frame_id"] == tile_id), None)
        if fr is None:
            raise KeyError(f"Tile ID {tile_id} not found")
        return fr
    if last:
        return max(frames, key=lambda f: f["frame_id"])
    if center:
        boxes = [f["bbox"] for f in frames]
        cx = (min(b[0] for b in boxes) + max(b[2] for b in boxes)) / 2
        cy = (min(b[1] for b in boxes) + max(b[3] for b in boxes)) / 2
        return min(frames, key=lambda f: ((f["bbox"][0] + f["bbox"][2]) / 2 - cx) ** 2
                   + ((f["bbox"][1] + f["bbox"][3]) / 2 - cy) ** 2)
    if bbox is not None:
        if len(bbox) != 4:
            raise ValueError("Bbox must have 4 coordinates")
        hit = [f for f in frames if bbox[0] < f["bbox"][2] and bbox[2] > f["bbox"][0] and bbox[1] < f["bbox"][3]
               and bbox[3] > f["bbox"][1]]
        if not hit:
            raise LookupError("No tiles intersect bbox")
        return hit[0]
    raise ValueError("Specify tile_id, bbox, center or last")


def read_tile_bytes(path: Path, frame: Dict, header_size: int) -> bytes:
    with open(path, "rb") as f:
        f.seek(header_size + frame["byte_offset"])
        return f.read(frame["byte_size"])
