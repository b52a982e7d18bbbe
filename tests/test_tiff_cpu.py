"""GeoTIFF reader (raster I/O ahead of the encode path) on the CPU: the native chunk
decoder (fra_tiff_decode: none / LZW / deflate, predictors 1-3, strips and tiles, chunky and planar,
II and MM) against independent encoders -- Pillow's libtiff (LZW / deflate, predictor 2 and the
floating-point predictor 3) and a small spec-level TIFF writer below -- and against the reference's own
test rasters.  Window reads decode only the overlapping chunks and equal the slice of a full read
(rasterio ``read(window=...)``, reference ``cli.py:559``)."""
import struct
import zlib

import numpy as np
import pytest

from flac_raster.tiff import GeoTIFF, read_geotiff

PIL = pytest.importorskip("PIL.Image")


def lzw_encode(data: bytes) -> bytes:
    """TIFF 6.0 LZW (MSB-first, 9..12-bit codes, early change), for fixtures only."""
    out, acc, nbits = bytearray(), 0, 0
    width = 9

    def put(code):
        nonlocal acc, nbits
        acc = (acc << width) | code
        nbits += width
        while nbits >= 8:
            out.append((acc >> (nbits - 8)) & 0xFF)
            nbits -= 8

    table = {bytes([i]): i for i in range(256)}
    nxt = 258
    put(256)
    w = b""
    for byte in data:
        wc = w + bytes([byte])
        if wc in table:
            w = wc
            continue
        put(table[w])
        table[wc] = nxt
        nxt += 1
        if nxt >= (1 << width) and width < 12:  # encoder side of the early change (decoder lags one entry)
            width += 1
        if nxt >= 4094:
            put(256)
            table = {bytes([i]): i for i in range(256)}
            nxt, width = 258, 9
        w = bytes([byte])
    if w:
        put(table[w])
        nxt += 1
        if nxt >= (1 << width) and width < 12:  # encoder side of the early change (decoder lags one entry)
            width += 1
    put(257)
    if nbits:
        out.append((acc << (8 - nbits)) & 0xFF)
    return bytes(out)


def write_tiff(path, data, tile=None, planar=1, compression=1, predictor=1, bo="<", rows_per_strip=None):
    """Spec-level TIFF writer: strips or tiles, chunky or planar, none / LZW / deflate, predictor 1/2/3."""
    B, H, W = data.shape
    dt = data.dtype
    fmt = 3 if dt.kind == "f" else (2 if dt.kind == "i" else 1)
    es = dt.itemsize

    def encode_chunk(block):  # block: (rows, cols, spp) native
        rows, cols, spp = block.shape
        if predictor == 2:
            d = block.copy()
            d[:, 1:, :] = block[:, 1:, :] - block[:, :-1, :]
            raw = d.astype(dt.newbyteorder(bo)).tobytes()
        elif predictor == 3:
            be = block.astype(dt.newbyteorder(">")).reshape(rows, cols * spp).view(np.uint8).reshape(rows, cols * spp, es)
            planes = np.ascontiguousarray(np.transpose(be, (0, 2, 1))).reshape(rows, -1)
            diff = planes.copy()
            diff[:, spp:] = planes[:, spp:] - planes[:, :-spp]
            raw = diff.tobytes()
        else:
            raw = block.astype(dt.newbyteorder(bo)).tobytes()
        if compression == 5:
            return lzw_encode(raw)
        if compression == 8:
            return zlib.compress(raw)
        return raw

    chunks = []
    planes = range(B) if planar == 2 else [None]
    if tile:
        tw, th = tile
        for pl in planes:
            for r in range(0, H, th):
                for c in range(0, W, tw):
                    blk = np.zeros((th, tw, 1 if pl is not None else B), dt)
                    src = data[pl:pl + 1] if pl is not None else data
                    part = np.moveaxis(src[:, r:r + th, c:c + tw], 0, 2)
                    blk[:part.shape[0], :part.shape[1]] = part
                    chunks.append(encode_chunk(blk))
    else:
        rps = rows_per_strip or max(1, 7)
        for pl in planes:
            src = data[pl:pl + 1] if pl is not None else data
            for r in range(0, H, rps):
                chunks.append(encode_chunk(np.ascontiguousarray(np.moveaxis(src[:, r:r + rps, :], 0, 2))))
    entries = [(256, 4, [W]), (257, 4, [H]), (258, 3, [es * 8] * B), (259, 3, [compression]), (262, 3, [1]),
               (277, 3, [B]), (284, 3, [planar]), (317, 3, [predictor]), (339, 3, [fmt] * B)]
    if tile:
        entries += [(322, 3, [tile[0]]), (323, 3, [tile[1]]), (324, 4, [0] * len(chunks)),
                    (325, 4, [len(c) for c in chunks])]
    else:
        entries += [(273, 4, [0] * len(chunks)), (278, 4, [rps]), (279, 4, [len(c) for c in chunks])]
    entries.sort()
    n = len(entries)
    head = 8 + 2 + 12 * n + 4
    ext = bytearray()
    locs = {}
    for tag, typ, vals in entries:
        raw = struct.pack(bo + ("H" if typ == 3 else "I") * len(vals), *vals)
        if len(raw) > 4:
            locs[tag] = head + len(ext)
            ext += raw
    data_base = head + len(ext)
    offs, pos = [], data_base
    for c in chunks:
        offs.append(pos)
        pos += len(c)
    off_tag = 324 if tile else 273
    entries = [(t, ty, offs if t == off_tag else v) for t, ty, v in entries]
    ext = bytearray()
    out = bytearray((b"II" if bo == "<" else b"MM") + struct.pack(bo + "HI", 42, 8) + struct.pack(bo + "H", n))
    for tag, typ, vals in entries:
        raw = struct.pack(bo + ("H" if typ == 3 else "I") * len(vals), *vals)
        if len(raw) > 4:
            out += struct.pack(bo + "HHII", tag, typ, len(vals), head + len(ext))
            ext += raw
        else:
            out += struct.pack(bo + "HHI", tag, typ, len(vals)) + raw.ljust(4, b"\0")
    out += struct.pack(bo + "I", 0) + ext
    assert len(out) == data_base
    for c in chunks:
        out += c
    open(path, "wb").write(bytes(out))


def _rand(shape, dtype, seed=0):
    rng = np.random.default_rng(seed)
    if np.dtype(dtype).kind == "f":
        return (rng.standard_normal(shape) * 100).astype(dtype)
    info = np.iinfo(dtype)
    base = np.cumsum(rng.integers(-20, 21, size=shape), axis=-1)  # smooth rows: predictors matter
    return np.clip(base + (info.min + info.max) // 2, info.min, info.max).astype(dtype)


@pytest.mark.parametrize("compression", ["tiff_lzw", "tiff_adobe_deflate", None])
@pytest.mark.parametrize("dtype,pred", [(np.uint16, 1), (np.uint16, 2), (np.uint8, 2),
                                        (np.float32, 3), (np.float32, 1)])
def test_pillow_written_strips(tmp_path, compression, dtype, pred):
    if pred != 1 and compression is None:
        pytest.skip("predictor needs compression in Pillow's libtiff writer")
    a = _rand((77, 131), dtype, seed=int(pred) + (compression or "x").__len__())
    f = tmp_path / "p.tif"
    kw = {"compression": compression} if compression else {}
    if pred != 1:
        kw["tiffinfo"] = {317: pred}
    PIL.fromarray(a).save(f, **kw)
    g = GeoTIFF(f)
    assert g.predictor == pred
    full = g.read()
    assert full.dtype == np.dtype(dtype) and np.array_equal(full[0], a)
    assert np.array_equal(np.asarray(PIL.open(f)), a)
    assert np.array_equal(g.read_window(5, 9, 40, 100)[0], a[5:45, 9:109])


def test_pillow_rgb_lzw(tmp_path):
    a = _rand((3, 64, 90), np.uint8, 5)
    f = tmp_path / "rgb.tif"
    PIL.fromarray(np.moveaxis(a, 0, 2), "RGB").save(f, compression="tiff_lzw", tiffinfo={317: 2})
    assert np.array_equal(read_geotiff(f)[0], a)


@pytest.mark.parametrize("compression", [1, 5, 8])
@pytest.mark.parametrize("planar", [1, 2])
@pytest.mark.parametrize("tile", [None, (32, 16)])
@pytest.mark.parametrize("bo", ["<", ">"])
def test_spec_writer_matrix(tmp_path, compression, planar, tile, bo):
    a = _rand((3, 50, 70), np.int16, 11)
    f = tmp_path / "m.tif"
    write_tiff(f, a, tile=tile, planar=planar, compression=compression, predictor=2 if compression != 1 else 1, bo=bo)
    g = GeoTIFF(f)
    assert np.array_equal(g.read(), a)
    for (r, c, h, w) in [(0, 0, 50, 70), (3, 5, 20, 33), (49, 69, 1, 1), (16, 32, 16, 32)]:
        assert np.array_equal(g.read_window(r, c, h, w), a[:, r:r + h, c:c + w])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("bo", ["<", ">"])
def test_float_predictor3(tmp_path, dtype, bo):
    a = _rand((2, 21, 37), dtype, 3)
    a[0, 3, 4] = np.nan
    f = tmp_path / "f.tif"
    write_tiff(f, a, tile=(16, 16), planar=1, compression=8, predictor=3, bo=bo)
    got = GeoTIFF(f).read()
    assert got.dtype == np.dtype(dtype)
    assert np.array_equal(got, a, equal_nan=True)


def test_reference_rasters_match_pillow():
    from pathlib import Path

    gold = Path(__file__).resolve().parent / "golden"
    for name in ("sample_dem.tif", "sample_rgb.tif"):
        a, _ = read_geotiff(gold / name)
        p = np.asarray(PIL.open(gold / name))
        p = p[None] if p.ndim == 2 else np.moveaxis(p, 2, 0)
        assert np.array_equal(a, p)


def test_rejects_invalid(tmp_path):
    a = _rand((1, 8, 8), np.uint16, 1)
    f = tmp_path / "bad.tif"
    write_tiff(f, a, compression=8, predictor=1)
    raw = bytearray(f.read_bytes())
    g = GeoTIFF(f)
    off = int(g._offs[0])
    raw[off:off + 4] = b"\xff\xff\xff\xff"  # corrupt the first deflate stream
    bad = tmp_path / "bad2.tif"
    bad.write_bytes(bytes(raw))
    from flac_raster._native import NativeError

    with pytest.raises(NativeError):
        GeoTIFF(bad).read()
    fl = tmp_path / "p2f.tif"
    write_tiff(fl, _rand((1, 8, 8), np.float32, 2), compression=8, predictor=3)
    raw = bytearray(fl.read_bytes())
    i = raw.find(struct.pack("<HHI", 317, 3, 1))
    raw[i + 8:i + 10] = struct.pack("<H", 2)  # predictor 2 on float data is invalid
    (tmp_path / "p2f_bad.tif").write_bytes(bytes(raw))
    with pytest.raises(NotImplementedError):
        GeoTIFF(tmp_path / "p2f_bad.tif")


@pytest.mark.parametrize("compression,pred", [(5, 2), (8, 2), (5, 1)])
def test_spec_writer_cross_checked_by_pillow(tmp_path, compression, pred):
    """The fixture writer itself is checked by an independent reader (Pillow's libtiff)."""
    a = _rand((1, 40, 52), np.uint16, 9)
    f = tmp_path / "x.tif"
    write_tiff(f, a, tile=(16, 16), compression=compression, predictor=pred)
    assert np.array_equal(np.asarray(PIL.open(f)), a[0])
    assert np.array_equal(GeoTIFF(f).read(), a)


@pytest.mark.parametrize("compression", ["lzw", "deflate"])
@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.int16, np.float32])
@pytest.mark.parametrize("pred", [1, 2])
def test_native_tile_writer_round_trip_and_pillow(tmp_path, compression, dtype, pred):
    """write_geotiff(compression=, tile=, predictor=) -- the native LZW / deflate chunk encoder
    (fra_tiff_compress) -- reads back bit-exactly through fra_tiff_decode, and Pillow (libtiff) decodes
    the single-band files identically (independent LZW decoder: early change, Clear/EOI placement)."""
    if dtype == np.float32 and pred == 2:
        pytest.skip("predictor 2 is for integer samples")
    from flac_raster.tiff import write_geotiff

    rng = np.random.default_rng(11)
    base = np.cumsum(rng.integers(-3, 4, size=(3, 300, 333)), axis=2)
    a = (base - base.min()).astype(dtype) if dtype != np.float32 else (base * 0.5).astype(dtype)
    f = tmp_path / "t.tif"
    write_geotiff(f, a, compression=compression, tile=128, predictor=pred)
    b, _ = read_geotiff(f)
    assert b.dtype == a.dtype and np.array_equal(a, b)
    if dtype in (np.uint8, np.uint16):
        write_geotiff(f, a[:1], compression=compression, tile=64, predictor=pred)
        assert np.array_equal(np.asarray(PIL.open(f)).astype(dtype), a[0])


def test_native_lzw_table_resets(tmp_path):
    """Incompressible and constant tiles: the LZW table fills and restarts (Clear at 4093 entries)."""
    from flac_raster.tiff import write_geotiff

    rng = np.random.default_rng(3)
    for a in (rng.integers(0, 256, size=(1, 700, 700)).astype(np.uint8), np.zeros((1, 512, 512), np.uint8)):
        f = tmp_path / "r.tif"
        write_geotiff(f, a, compression="lzw", tile=512)
        assert np.array_equal(read_geotiff(f)[0], a)
        assert np.array_equal(np.asarray(PIL.open(f)), a[0])
