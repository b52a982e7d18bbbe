"""Minimal GeoTIFF reader/writer (numpy only) standing in for the rasterio calls on the encode path.

The reference reads rasters with ``rasterio.open(...).read()`` (``converter.py:73-79``) and
``src.read(window=...)`` (``cli.py:559``, ``spatial_encoder.py:205-206``) and writes tile GeoTIFFs
(``cli.py:577-591``).  rasterio/GDAL are not part of this image, so this module implements the
subset the encode path needs:

* baseline TIFF + BigTIFF, II/MM byte order, strips or tiles, PlanarConfiguration 1 or 2,
  Compression 1 (none), 5 (LZW), 8 (Adobe deflate), 32946 (deflate); Predictor 1, 2 (integers),
  3 (floating point) -- decoded natively (``csrc/fra_tiff.cpp``), any other value is rejected;
* SampleFormat uint / int / IEEE float, 8/16/32/64 bits;
* GeoTIFF ModelPixelScale + ModelTiepoint or ModelTransformation -> affine transform
  (GDAL order ``(a, b, c, d, e, f)`` as ``list(rasterio.Affine)[:6]``), GeoKeyDirectory -> ``EPSG:n``.

Arrays are returned band-planar ``(bands, height, width)`` like ``rasterio.read()``.
"""

from __future__ import annotations

import mmap
import os
import struct
from dataclasses import dataclass, field
from pathlib import Path
from typing import Optional

import numpy as np

_TYPE_SIZES = {1: 1, 2: 1, 3: 2, 4: 4, 5: 8, 6: 1, 7: 1, 8: 2, 9: 4, 10: 8, 11: 4, 12: 8, 16: 8, 17: 8, 18: 8}
_TYPE_FMT = {1: "B", 2: "c", 3: "H", 4: "I", 5: "II", 6: "b", 7: "B", 8: "h", 9: "i", 10: "ii", 11: "f",
             12: "d", 16: "Q", 17: "q", 18: "Q"}


@dataclass
class RasterInfo:
    width: int
    height: int
    count: int
    dtype: np.dtype
    transform: tuple = (1.0, 0.0, 0.0, 0.0, 1.0, 0.0)  # a, b, c, d, e, f
    crs: Optional[str] = None
    nodata: Optional[float] = None
    tags: dict = field(default_factory=dict)

    @property
    def bounds(self):
        a, b, c, d, e, f = self.transform
        xs = [c, c + a * self.width]
        ys = [f, f + e * self.height]
        return (min(xs), min(ys), max(xs), max(ys))  # left, bottom, right, top

    def window_transform(self, col_off: int, row_off: int):
        a, b, c, d, e, f = self.transform
        return (a, b, c + a * col_off + b * row_off, d, e, f + d * col_off + e * row_off)


def _dtype_from(fmt: int, bits: int) -> np.dtype:
    kind = {1: "u", 2: "i", 3: "f"}.get(fmt, "u")
    return np.dtype(f"{kind}{bits // 8}")


class GeoTIFF:
    """Read-only GeoTIFF.  ``read()`` -> (bands, H, W); ``read_window(r, c, h, w)``.

    The file is memory-mapped; only the IFD is parsed in Python.  Strips/tiles are decoded by the
    native multi-threaded decoder (``fra_tiff_decode``: none / LZW / deflate, predictors 1-3) straight
    into the destination array -- page-locked memory when ``pinned=True`` (the layout the pipelined
    encode ``fra_plan_encode_host`` copies at full PCIe rate).  A window read decodes only the chunks
    that overlap the window (rasterio ``read(window=...)``, ``cli.py:559``).
    """

    def __init__(self, path):
        self.path = Path(path)
        with open(self.path, "rb") as f:
            size = os.fstat(f.fileno()).st_size
            if size < 8:
                raise ValueError(f"not a TIFF: {path}")
            self._buf = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
        b = self._buf
        if b[:2] == b"II":
            self.bo = "<"
        elif b[:2] == b"MM":
            self.bo = ">"
        else:
            raise ValueError(f"not a TIFF: {path}")
        magic = struct.unpack(self.bo + "H", b[2:4])[0]
        self.big = magic == 43
        if self.big:
            off = struct.unpack(self.bo + "Q", b[8:16])[0]
        elif magic == 42:
            off = struct.unpack(self.bo + "I", b[4:8])[0]
        else:
            raise ValueError("bad TIFF magic")
        self.tags = self._read_ifd(off)
        t = self.tags
        W, H = int(t[256][0]), int(t[257][0])
        spp = int(t.get(277, [1])[0])
        bits = t.get(258, [8] * spp)
        fmt = int(t.get(339, [1])[0])
        if any(int(x) != int(bits[0]) for x in bits) or int(bits[0]) not in (8, 16, 32, 64):
            raise NotImplementedError(f"TIFF BitsPerSample {bits} not supported")
        self.dtype = _dtype_from(fmt, int(bits[0])).newbyteorder(self.bo)
        self.planar = int(t.get(284, [1])[0])
        self.compression = int(t.get(259, [1])[0])
        self.predictor = int(t.get(317, [1])[0])
        if self.compression not in (1, 5, 8, 32946):
            raise NotImplementedError(f"TIFF compression {self.compression} not supported (none, LZW, deflate)")
        if self.predictor not in (1, 2, 3) or (self.predictor == 2 and fmt == 3) or (self.predictor == 3 and fmt != 3):
            raise NotImplementedError(f"TIFF predictor {self.predictor} not supported for SampleFormat {fmt}")
        transform = (1.0, 0.0, 0.0, 0.0, 1.0, 0.0)
        if 34264 in t:
            m = t[34264]
            transform = (m[0], m[1], m[3], m[4], m[5], m[7])
        elif 33550 in t and 33922 in t:
            sx, sy = t[33550][0], t[33550][1]
            tp = t[33922]
            i, j, x, y = tp[0], tp[1], tp[3], tp[4]
            transform = (sx, 0.0, x - i * sx, 0.0, -sy, y + j * sy)
        crs = None
        if 34735 in t:
            keys = t[34735]
            for k in range(4, len(keys), 4):
                kid, loc, cnt, val = keys[k:k + 4]
                if kid in (2048, 3072) and loc == 0:
                    crs = f"EPSG:{val}"
                    if kid == 3072:
                        break
        nodata = None
        if 42113 in t:
            try:
                nodata = float(t[42113].strip("\x00"))
            except ValueError:
                nodata = None
        self.info = RasterInfo(W, H, spp, np.dtype(self.dtype.newbyteorder("=")), transform, crs, nodata, {})
        self._data = None
        # chunk grid
        self.tiled = 322 in t
        self._offs = t[324] if self.tiled else t[273]
        self._cnts = t[325] if self.tiled else t[279]
        if self.tiled:
            self.cw, self.ch = int(t[322][0]), int(t[323][0])
        else:
            self.cw, self.ch = W, min(int(t.get(278, [H])[0]), H)  # RowsPerStrip 2^32-1 = one strip
        # chunk geometry comes from untrusted tags: positive and at most 2^20 on a side (the native decoder
        # re-checks every chunk's decoded size with overflow-safe arithmetic against its stored bytes)
        if not (0 < self.cw <= (1 << 20) and 0 < self.ch <= (1 << 20)):
            raise ValueError(f"TIFF chunk geometry {self.cw} x {self.ch} is not supported")
        self.nx = (W + self.cw - 1) // self.cw
        self.ny = (H + self.ch - 1) // self.ch

    def close(self):
        if self._buf is not None:
            try:
                self._buf.close()
            except BufferError:  # still exported to a live array
                pass

    # -- IFD parsing
    def _read_ifd(self, off: int) -> dict:
        b, bo = self._buf, self.bo
        if self.big:
            n = struct.unpack(bo + "Q", b[off:off + 8])[0]
            esz, p, inl = 20, off + 8, 8
        else:
            n = struct.unpack(bo + "H", b[off:off + 2])[0]
            esz, p, inl = 12, off + 2, 4
        tags = {}
        for i in range(n):
            e = b[p + i * esz:p + (i + 1) * esz]
            tag, typ = struct.unpack(bo + "HH", e[:4])
            if self.big:
                cnt = struct.unpack(bo + "Q", e[4:12])[0]
                raw = e[12:20]
            else:
                cnt = struct.unpack(bo + "I", e[4:8])[0]
                raw = e[8:12]
            size = _TYPE_SIZES.get(typ, 1) * cnt
            if size > inl:
                vo = struct.unpack(bo + ("Q" if self.big else "I"), raw)[0]
                data = b[vo:vo + size]
            else:
                data = raw[:size]
            if typ == 2:
                tags[tag] = data.decode("latin-1")
            elif typ in (5, 10):
                v = struct.unpack(bo + _TYPE_FMT[typ][0] * (2 * cnt), data)
                tags[tag] = [v[2 * k] / v[2 * k + 1] if v[2 * k + 1] else 0.0 for k in range(cnt)]
            else:
                tags[tag] = list(struct.unpack(bo + _TYPE_FMT.get(typ, "B") * cnt, data))
        return tags

    def _chunks(self, row_off: int, col_off: int, height: int, width: int):
        """Strips/tiles overlapping the window, as ``fra_tiff_chunk`` records."""
        from . import _native as N

        H = self.info.height
        cy0, cy1 = row_off // self.ch, (row_off + height - 1) // self.ch
        cx0, cx1 = col_off // self.cw, (col_off + width - 1) // self.cw
        planes = self.info.count if self.planar == 2 else 1
        per_plane = self.nx * self.ny
        out = []
        for pl in range(planes):
            for cy in range(cy0, cy1 + 1):
                for cx in range(cx0, cx1 + 1):
                    idx = pl * per_plane + cy * self.nx + cx
                    rows = self.ch if self.tiled else min(self.ch, H - cy * self.ch)
                    out.append(N.TiffChunk(int(self._offs[idx]), int(self._cnts[idx]), cy * self.ch, cx * self.cw,
                                           rows, self.cw, pl, 0))
        return out

    def read_window_into(self, out: np.ndarray, row_off: int, col_off: int, height: int, width: int,
                         threads: int = 0) -> np.ndarray:
        """Decode a window into ``out`` (band-planar ``(bands, height, width)`` view, native byte order,
        unit column stride; e.g. a page-locked array from ``_native.pinned_empty``)."""
        import ctypes as C

        from . import _native as N

        info = self.info
        if out.shape != (info.count, height, width) or out.dtype != info.dtype:
            raise ValueError(f"out must be {(info.count, height, width)} {info.dtype}, got {out.shape} {out.dtype}")
        es = info.dtype.itemsize
        if out.strides[2] != es or out.strides[0] % es or out.strides[1] % es:
            raise ValueError("out needs unit column stride")
        if not (0 <= row_off and 0 <= col_off and row_off + height <= info.height and col_off + width <= info.width):
            raise ValueError("window outside the raster")
        if height == 0 or width == 0:
            return out
        chunks = self._chunks(row_off, col_off, height, width)
        arr = (N.TiffChunk * len(chunks))(*chunks)
        lay = N.TiffLayout(self.compression, self.predictor, es, 1 if self.planar == 2 else info.count,
                           1 if info.dtype.kind == "f" else 0, 1 if self.bo == ">" else 0, info.count, row_off,
                           col_off, height, width, 0, out.strides[0] // es, out.strides[1] // es)
        src = np.frombuffer(self._buf, dtype=np.uint8)
        N._check(N.load().fra_tiff_decode(src.ctypes.data_as(C.c_void_p), len(self._buf), C.byref(lay), arr,
                                          len(chunks), out.ctypes.data_as(C.c_void_p), threads or _threads()))
        del src
        return out

    def read(self, out: Optional[np.ndarray] = None, pinned: bool = False) -> np.ndarray:
        """All bands, (count, H, W) native-endian -- rasterio ``read()`` equivalent."""
        info = self.info
        if out is None:
            if self._data is not None and not pinned:
                return self._data
            out = _alloc((info.count, info.height, info.width), info.dtype, pinned)
            self.read_window_into(out, 0, 0, info.height, info.width)
            if not pinned:
                self._data = out
            return out
        return self.read_window_into(out, 0, 0, info.height, info.width)

    def read_window(self, row_off: int, col_off: int, height: int, width: int, pinned: bool = False) -> np.ndarray:
        """rasterio ``read(window=Window(col_off, row_off, width, height))``: only the overlapping chunks
        are decoded."""
        out = _alloc((self.info.count, height, width), self.info.dtype, pinned)
        return self.read_window_into(out, row_off, col_off, height, width)


def _threads() -> int:
    """Decoder threads: the process's CPU share (OMP_NUM_THREADS, set to the share on the GPU boxes), else
    at most 16 -- os.cpu_count() reports the whole machine there."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return max(1, min(16, os.cpu_count() or 1))


def _alloc(shape, dtype, pinned: bool) -> np.ndarray:
    if pinned:
        from . import _native as N

        return N.pinned_empty(shape, dtype)
    return np.empty(shape, dtype=dtype)


def read_geotiff(path, pinned: bool = False):
    g = GeoTIFF(path)
    return g.read(pinned=pinned), g.info


def _geo_entries(S, H, W, dt, transform, crs, nodata):
    fmt = 3 if dt.kind == "f" else (2 if dt.kind == "i" else 1)
    bits = dt.itemsize * 8
    entries = []  # (tag, type, values)
    entries.append((256, 3 if W < 65536 else 4, [W]))
    entries.append((257, 3 if H < 65536 else 4, [H]))
    entries.append((258, 3, [bits] * S))
    entries.append((262, 3, [2 if S == 3 and dt == np.uint8 else 1]))
    entries.append((277, 3, [S]))
    entries.append((284, 3, [1]))
    entries.append((339, 3, [fmt] * S))
    if transform is not None:
        a, b, c, d, e, f = [float(v) for v in list(transform)[:6]]
        if b == 0.0 and d == 0.0:
            entries.append((33550, 12, [a, -e, 0.0]))
            entries.append((33922, 12, [0.0, 0.0, 0.0, c, f, 0.0]))
        else:
            entries.append((34264, 12, [a, b, 0.0, c, d, e, 0.0, f, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0]))
    if crs and str(crs).upper().startswith("EPSG:"):
        code = int(str(crs).split(":")[1])
        geographic = 4000 <= code < 5000
        keys = [1, 1, 0, 3, 1024, 0, 1, 2 if geographic else 1, 1025, 0, 1, 1,
                2048 if geographic else 3072, 0, 1, code]
        entries.append((34735, 3, keys))
    if nodata is not None:
        entries.append((42113, 2, (str(nodata) + "\x00").encode("latin-1")))
    return entries


def _write_tiff(path, entries, chunks, offsets_tag: int):
    """Classic little-endian TIFF: header | IFD | external tag values | chunks (offsets patched)."""
    entries = sorted(entries, key=lambda x: x[0])
    n = len(entries)
    ifd_size = 2 + 12 * n + 4
    ext = bytearray()
    ext_base = 8 + ifd_size
    packed = []
    fmtmap = {3: "H", 4: "I", 12: "d"}
    for tag, typ, vals in entries:
        if typ == 2:
            raw = bytes(vals)
            cnt = len(raw)
        else:
            raw = struct.pack("<" + fmtmap[typ] * len(vals), *vals)
            cnt = len(vals)
        packed.append([tag, typ, cnt, raw])
    for it in packed:
        if len(it[3]) > 4:
            it.append(ext_base + len(ext))
            ext += it[3]
            if len(ext) % 2:
                ext += b"\x00"
        else:
            it.append(None)
    offsets, pos = [], ext_base + len(ext)
    for c in chunks:
        offsets.append(pos)
        pos += len(c)
    if pos >= (1 << 32):
        raise ValueError("file larger than 4 GiB needs BigTIFF, which this writer does not produce")
    for it in packed:  # patch the chunk offsets
        if it[0] == offsets_tag:
            raw = struct.pack("<" + "I" * len(offsets), *offsets)
            it[3] = raw
            if it[4] is not None:
                ext[it[4] - ext_base:it[4] - ext_base + len(raw)] = raw
    head = bytearray(b"II*\x00" + struct.pack("<I", 8))
    head += struct.pack("<H", n)
    for tag, typ, cnt, raw, loc in packed:
        head += struct.pack("<HHI", tag, typ, cnt)
        head += struct.pack("<I", loc) if loc is not None else raw.ljust(4, b"\x00")
    head += struct.pack("<I", 0)
    head += ext
    with open(path, "wb") as f:
        f.write(head)
        for c in chunks:
            f.write(c)


def write_geotiff(path, data: np.ndarray, transform=None, crs: Optional[str] = None, nodata=None,
                  compression: Optional[str] = None, tile: Optional[int] = None, predictor: int = 1,
                  level: int = 6):
    """Write a pixel-interleaved little-endian GeoTIFF: uncompressed strips by default (the layout the
    tests' fixtures use), or ``tile`` x ``tile`` tiles compressed with ``compression`` = "lzw" / "deflate"
    (native thread pool, ``fra_tiff_compress``) and ``predictor`` 2 (horizontal differencing, integer
    samples) -- the tiled GeoTIFFs rasterio writes for the tile files of ``cli.py:577-591``."""
    data = np.asarray(data)
    if data.ndim == 2:
        data = data[None]
    S, H, W = data.shape
    dt = data.dtype
    entries = _geo_entries(S, H, W, dt, transform, crs, nodata)
    if compression is None and tile is None:
        pix = np.ascontiguousarray(np.moveaxis(data, 0, 2)).astype(dt.newbyteorder("<"), copy=False)
        rows_per_strip = max(1, min(H, (1 << 16) // max(1, W * S * dt.itemsize)))
        strips = [pix[r:r + rows_per_strip].tobytes() for r in range(0, H, rows_per_strip)]
        entries += [(259, 3, [1]), (273, 4, [0] * len(strips)), (278, 4, [rows_per_strip]),
                    (279, 4, [len(x) for x in strips])]
        _write_tiff(path, entries, strips, 273)
        return
    comp = {None: 1, "none": 1, "lzw": 5, "deflate": 8}[compression]
    T = int(tile or 256)
    if T % 16:
        raise ValueError("TIFF tile size must be a multiple of 16")
    if predictor not in (1, 2) or (predictor == 2 and dt.kind == "f"):
        raise ValueError("predictor 1, or 2 on integer samples")
    nx, ny = (W + T - 1) // T, (H + T - 1) // T
    pix = np.zeros((ny * T, nx * T, S), dt.newbyteorder("<"))
    pix[:H, :W] = np.moveaxis(data, 0, 2)
    tiles = pix.reshape(ny, T, nx, T, S).transpose(0, 2, 1, 3, 4)  # (ny, nx, T rows, T cols, S)
    if predictor == 2:  # horizontal differencing per tile row, stride = samples per pixel (modular)
        u = tiles.view(np.dtype(f"<u{dt.itemsize}"))
        d = u.copy()
        d[:, :, :, 1:, :] = u[:, :, :, 1:, :] - u[:, :, :, :-1, :]
        tiles = d
    raw = np.ascontiguousarray(tiles).reshape(ny * nx, T * T * S).view(np.uint8)
    if comp == 1:
        chunks = [raw[i].tobytes() for i in range(raw.shape[0])]
    else:
        from . import _native as N

        chunks = N.tiff_compress(comp, raw, level=level)
    entries += [(259, 3, [comp]), (317, 3, [predictor]), (322, 3, [T]), (323, 3, [T]),
                (324, 4, [0] * len(chunks)), (325, 4, [len(x) for x in chunks])]
    _write_tiff(path, entries, chunks, 324)
