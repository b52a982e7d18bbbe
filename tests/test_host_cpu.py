"""CPU tests of the product's host side (no GPU needed).

* C ABI: ``libflac_raster_amd.so`` loads and exports every ``FRA_API`` symbol of include/*.h.
* native decoder (``fra_decode``, host C++ in the product library): libFLAC golden KAT, oracle
  streams of every level / edge case, concatenated streams, corruption.
* mutagen-equivalent tag writer: rebuilds ``sample_dem.flac`` byte for byte and its
  spatial index JSON (F6).
* geometry (tiles, LPT/contiguous splits, window transforms, bboxes), streaming container layout
  and per-tile tags assembled from encoded streams (oracle stand-in), extract tile selection.
* normalization host functions vs golden vectors generated from the reference's normalization.py.
* no silent fallback: encode calls raise NativeUnavailable without a device.
"""
import base64
import gzip
import hashlib
import json
import re
from pathlib import Path

import numpy as np
import pytest

import oracle as O
from flac_raster import _native as N
from flac_raster import flac_meta, normalization
from flac_raster.converter import RasterFLACConverter, raster_metadata, raster_tags
from flac_raster.geo import Affine, Window, bounds, window_transform
from flac_raster.spatial_encoder import SpatialFrame, SpatialIndex, tile_bbox
from flac_raster.streaming import assemble_streaming, open_streaming, read_index_bytes, read_tile_bytes, select_frame
from flac_raster.tiff import read_geotiff, write_geotiff
from flac_raster.tiles import calculate_tiles, lpt_assign, split_contiguous
from oracle_tiles import oracle_encode_tiles

ROOT = Path(__file__).resolve().parents[1]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ----------------------------------------------------------------------------------- C ABI
def test_abi_exports_every_declared_symbol():
    decl = set()
    for h in (ROOT / "include").glob("*.h"):
        decl |= set(re.findall(r"FRA_API\s+[^;(]*?\b(fra_\w+)\s*\(", h.read_text()))
    assert len(decl) >= 26
    L = N.load()
    missing = [s for s in sorted(decl) if not hasattr(L, s)]
    assert not missing, missing
    assert set(N.EXPORTS) == decl
    assert L.fra_abi_version() == 3


def test_abi_errors_without_device():
    if N.device_count() > 0:
        pytest.skip("a GPU is visible; this checks the no-device error path")
    with pytest.raises(N.NativeUnavailable):
        N.Context(0)
    with pytest.raises(N.NativeUnavailable):
        normalization.normalize_to_audio(np.arange(10, dtype=np.uint8).reshape(-1, 1), 16)


def test_stream_header_matches_oracle():
    for ch, bps, sr, bs in [(1, 16, 44100, 4096), (4, 16, 48000, 4096), (8, 32, 44100, 4096), (3, 16, 96000, 1152)]:
        assert N.stream_header(ch, bps, sr, bs) == O.stream_header(ch, bps, sr, bs)


# ----------------------------------------------------------------------------------- decoder
def test_decoder_libflac_golden(golden_dir):
    g = json.loads((golden_dir / "golden.json").read_text())
    x, info = N.decode((golden_dir / "sample_rgb.flac").read_bytes())
    assert (info.sample_rate, info.channels, info.bps, info.nframes, info.nstreams) == (44100, 3, 16, 16, 1)
    assert sha(x.astype(np.int16)) == g["tiffs"]["sample_rgb.tif"]["audio_sha256"]


def test_decoder_rejects_corruption_and_truncation(golden_dir):
    d = bytearray((golden_dir / "sample_rgb.flac").read_bytes())
    for pos in (200, 50000, len(d) - 3):
        e = bytearray(d)
        e[pos] ^= 0x04
        with pytest.raises(N.NativeError):
            N.decode(bytes(e))
    with pytest.raises(N.NativeError):
        N.decode(bytes(d[:-100]))
    with pytest.raises(N.NativeError):
        N.decode(b"RIFF0000")


def test_decoder_rejects_id3_past_end():
    """an ID3v2 size pointing past the buffer must fail cleanly, not read out of bounds."""
    with pytest.raises(N.NativeError):
        N.decode(b"ID3\x04\x00\x00\x7f\x7f\x7f\x7f" + b"fLaC")
    with pytest.raises(N.NativeError):
        N.decode(b"ID3\x04\x00\x00\x00\x00\x00\x05fL")


def _crc(data, poly, width):
    c = 0
    top = 1 << (width - 1)
    mask = (1 << width) - 1
    for b in data:
        c ^= b << (width - 8)
        for _ in range(8):
            c = ((c << 1) ^ poly) & mask if c & top else (c << 1) & mask
    return c


def test_decoder_rejects_out_of_range_prediction():
    """a CRC-valid frame whose FIXED reconstruction leaves the 16-bit sample range is
    rejected (libFLAC does too) instead of overflowing / truncating."""
    hdr = N.stream_header(1, 16, 44100, 16)
    bits = []

    def put(v, n):
        bits.extend((v >> (n - 1 - i)) & 1 for i in range(n))
    # frame header: sync, fixed blocksize, bs code 6 (8-bit bs-1), sr 44.1k, mono, 16 bit, frame 0
    put(0xFFF8, 16); put(6, 4); put(9, 4); put(0, 4); put(4, 3); put(0, 1); put(0, 8); put(15, 8)
    fh = bytes(int("".join(map(str, bits[i:i + 8])), 2) for i in range(0, len(bits), 8))
    bits.clear()
    # FIXED order 1, warm-up 32767, residual partition order 0 escaped to 17-bit raw residuals of 65535
    put(0, 1); put(9, 6); put(0, 1); put(32767, 16)
    put(0, 2); put(0, 4); put(15, 4); put(17, 5)
    for _ in range(15):
        put(65535, 17)
    while len(bits) % 8:
        bits.append(0)
    body = bytes(int("".join(map(str, bits[i:i + 8])), 2) for i in range(0, len(bits), 8))
    frame = fh + bytes([_crc(fh, 0x07, 8)]) + body
    frame += _crc(frame, 0x8005, 16).to_bytes(2, "big")
    with pytest.raises(N.NativeError):
        N.decode(hdr + frame)


def test_decoder_concatenated_streams(golden_dir):
    d = (golden_dir / "sample_dem.flac").read_bytes()
    with pytest.raises(N.NativeError):
        N.decode(d)
    x, info = N.decode(d, concat=True)
    assert info.nstreams == 4 and info.bps == 32 and x.shape == (262144, 1)
    assert not x.any()  # F12: legacy artefact, every sample 0


@pytest.mark.parametrize("level", [0, 2, 5, 8])
def test_decoder_oracle_streams(golden_dir, level):
    data, _ = read_geotiff(golden_dir / "sample_multispectral.tif")
    audio, _, _ = O.normalize(data.transpose(1, 2, 0).reshape(-1, data.shape[0]), 16)
    bs = 1152 if level <= 2 else 4096
    x, info = N.decode(O.encode(audio, 44100, level=level, blocksize=bs))
    assert np.array_equal(x, audio.astype(np.int32)) and info.blocksize == bs


def test_decoder_edge_cases():
    rng = np.random.default_rng(5)
    for n, ch in [(1, 1), (15, 3), (4096, 2), (4097, 8), (9000, 1)]:
        a = rng.integers(-32768, 32767, size=(n, ch)).astype(np.int16)
        assert np.array_equal(N.decode(O.encode(a, 44100))[0], a.astype(np.int32))
    b = rng.integers(-2**31, 2**31 - 1, size=(5000, 2), dtype=np.int64).astype(np.int32)
    for lvl in (0, 5, 8):
        x, info = N.decode(O.encode(b, 44100, level=lvl))
        assert info.bps == 32 and np.array_equal(x, b)
    c = np.full((5000, 2), -32767, np.int16)
    assert np.array_equal(N.decode(O.encode(c, 44100))[0], c.astype(np.int32))
    w = (rng.integers(-100, 100, size=(9000, 1)) * 64).astype(np.int16)
    assert np.array_equal(N.decode(O.encode(w, 44100))[0], w.astype(np.int32))
    # > 1 MiB stream: multi-threaded pass 1 / pass 2
    big = np.cumsum(rng.integers(-300, 300, size=(700_000, 2)), axis=0).clip(-32768, 32767).astype(np.int16)
    x, info = N.decode(O.encode(big, 44100, level=1, blocksize=1152))
    assert np.array_equal(x, big.astype(np.int32)) and info.nframes == (700_000 + 1151) // 1152


def test_pcm16_float_semantics():
    from flac_raster.decoder import pcm16_float

    a = np.array([[-32768], [-1], [0], [32767]], np.int16)
    assert np.array_equal(pcm16_float(a), a / 32768.0)
    b = np.array([[-8388607], [8388607], [65535], [65536], [-65537]], np.int32)
    assert np.array_equal(pcm16_float(b), (b >> 16) / 32768.0)


# ----------------------------------------------------------------------------------- tags
def _pre_mutagen(d: bytes):
    blocks, off = flac_meta.parse_blocks(d)
    vc = flac_meta.VorbisComment.parse(blocks[1][1])
    orig = (b"fLaC" + flac_meta.render_block(0, blocks[0][1], False)
            + flac_meta.render_block(4, flac_meta.VorbisComment(vc.vendor).render(), True) + d[off:])
    return orig, vc


def test_mutagen_layout_sample_dem(golden_dir):
    """F5: STREAMINFO, VORBIS_COMMENT (vendor kept, tags in order), PADDING 1024 + audio//1000."""
    d = (golden_dir / "sample_dem.flac").read_bytes()
    orig, vc = _pre_mutagen(d)
    assert len(orig) == 86 + 33730
    assert flac_meta.rewrite_header(orig, vc.comments) == d
    assert flac_meta.rewrite_header(d, vc.comments) == d  # re-save keeps the padding (available >= 0)
    blocks, off = flac_meta.parse_blocks(d)
    assert [(t, len(b)) for t, b in blocks] == [(0, 34), (4, 951), (1, 1057)]


def test_padding_rules():
    assert flac_meta.default_padding(-5, 33730) == 1057
    assert flac_meta.default_padding(100, 0) == 100
    assert flac_meta.default_padding(20000, 0) == 1024
    vc = flac_meta.VorbisComment("v", [("TITLE", "a")])
    vc["title"] = "b"
    assert vc.comments == [("title", "b")] and "TITLE" in vc and vc["Title"] == ["b"]
    with pytest.raises(flac_meta.FLACMetaError):
        flac_meta.VorbisComment("v", [("BAD=KEY", "x")]).render()


def test_spatial_index_json_matches_reference(golden_dir):
    """The compact JSON of SpatialIndex.to_dict equals the one the reference embedded (F6)."""
    f = flac_meta.FLACFile(golden_dir / "sample_dem.flac")
    ref_json = gzip.decompress(base64.b64decode(f["GEOSPATIAL_SPATIAL_INDEX"][0])).decode()
    d = json.loads(ref_json)
    frames = [SpatialFrame(x["frame_id"], tuple(x["bbox"]), Window(x["window"]["col_off"], x["window"]["row_off"],
                                                                   x["window"]["width"], x["window"]["height"]),
                           x["byte_offset"], x["byte_size"]) for x in d["frames"]]
    T = Affine(*d["transform"][:6])
    for fr in frames:  # bboxes recomputed through the affine equal the reference's
        w = fr.window
        assert fr.bbox == tile_bbox(T, w.row_off, w.col_off, w.height, w.width)
    idx = SpatialIndex(frames, d["crs"], T)
    assert json.dumps(idx.to_dict(), separators=(",", ":")) == ref_json
    # stale offsets (F6): index says tile 1 at 8,454; the file has its fLaC at 10,426
    raw = (golden_dir / "sample_dem.flac").read_bytes()
    assert frames[1].byte_offset == 8454 and raw[10426:10430] == b"fLaC"


# ----------------------------------------------------------------------------------- geometry
def test_tiles_c4_geometry():
    t = calculate_tiles(10980, 10980, 1024)
    assert len(t) == 121
    sizes = sorted({(h, w) for _, _, h, w in t})
    assert sizes == [(740, 740), (740, 1024), (1024, 740), (1024, 1024)]
    assert sum(h * w for _, _, h, w in t) == 10980 * 10980
    assert t[0] == (0, 0, 1024, 1024) and t[10] == (0, 10240, 1024, 740) and t[-1] == (10240, 10240, 740, 740)
    assert len(calculate_tiles(16384, 16384, 512)) == 1024 and len(calculate_tiles(32768, 32768, 512)) == 4096


def test_splits():
    w = [h * ww for _, _, h, ww in calculate_tiles(10980, 10980, 1024)]
    for parts in (1, 2, 4, 8):
        runs = split_contiguous(w, parts)
        assert runs[0][0] == 0 and runs[-1][1] == len(w) and len(runs) == parts
        assert all(a[1] == b[0] for a, b in zip(runs, runs[1:]))
        loads = [sum(w[s:e]) for s, e in runs]
        assert max(loads) / (sum(w) / parts) < 1.1
        g = lpt_assign(w, parts)
        assert sorted(i for x in g for i in x) == list(range(len(w)))
        assert max(sum(w[i] for i in x) for x in g) / (sum(w) / parts) < 1.05


def test_affine_and_window_transform():
    T = Affine(10.0, 0.0, 300000.0, 0.0, -10.0, 5000040.0)
    assert list(T) == [10.0, 0.0, 300000.0, 0.0, -10.0, 5000040.0, 0.0, 0.0, 1.0]
    assert T * (3, 4) == (300030.0, 5000000.0)
    tt = window_transform(T, 1024, 2048)
    assert tuple(tt)[:6] == (10.0, 0.0, 310240.0, 0.0, -10.0, 4979560.0)
    assert bounds(tt, 740, 1024) == (310240.0, 4979560.0 - 10240.0, 310240.0 + 7400.0, 4979560.0)
    # rasterio's windows.transform: translation(x - c, y - f) * T, not T.c + a*col
    G = Affine(0.1, 0.0, 0.3, 0.0, -0.1, 0.7)
    x, y = G * (3.0, 7.0)
    assert window_transform(G, 3, 7).c == 0.3 + (x - 0.3)


# ----------------------------------------------------------------------------------- containers
def _small_raster():
    rng = np.random.default_rng(11)
    base = np.cumsum(np.cumsum(rng.integers(-3, 4, size=(2, 300, 260)), axis=1), axis=2)
    return (base - base.min() + 100).astype(np.uint16)


def test_streaming_container_layout():
    r = _small_raster()
    T = Affine(20.0, 0.0, 500000.0, 0.0, -20.0, 4200000.0)
    tiles = calculate_tiles(300, 260, 128)
    streams = oracle_encode_tiles(r, tiles, 5)
    blob = assemble_streaming(tiles, streams, r.shape, r.dtype, T, "EPSG:32633", 128)
    idx, hs = read_index_bytes(blob)
    assert list(idx) == ["crs", "transform", "width", "height", "bands", "dtype", "tile_size", "frames"]
    assert blob[4:hs] == json.dumps(idx, separators=(",", ":")).encode()
    assert (idx["crs"], idx["width"], idx["height"], idx["bands"], idx["dtype"]) == ("EPSG:32633", 260, 300, 2, "uint16")
    off = 0
    for fr, (row, col, h, w), ts in zip(idx["frames"], tiles, streams):
        assert list(fr) == ["frame_id", "bbox", "window", "byte_offset", "byte_size"]
        assert fr["byte_offset"] == off
        tile = blob[hs + off: hs + off + fr["byte_size"]]
        off += fr["byte_size"]
        f = flac_meta.FLACFile(tile)
        tags = [k for k, _ in f.tags.comments]
        assert tags == [k for k, _ in raster_tags({})]
        assert f["GEOSPATIAL_WIDTH"] == [str(w)] and f["GEOSPATIAL_HEIGHT"] == [str(h)]
        assert f["GEOSPATIAL_NODATA"] == ["None"] and f["GEOSPATIAL_SPATIAL_TILING"] == ["False"]
        assert f["GEOSPATIAL_DATA_MIN"] == [str(ts.data_min)]
        tt = json.loads(f["GEOSPATIAL_TRANSFORM"][0])
        assert tt == list(window_transform(T, col, row))
        assert fr["bbox"] == [tt[2], tt[5] + h * tt[4], tt[2] + w * tt[0], tt[5]]
        # the tile decodes to the normalised tile (interleave = pixel-major, channel = band)
        x, info = N.decode(tile)
        inter = r[:, row:row + h, col:col + w].transpose(1, 2, 0).reshape(-1, 2)
        assert np.array_equal(x, O.normalize(inter, 16)[0].astype(np.int32))
        blocks, aoff = flac_meta.parse_blocks(tile)
        assert blocks[-1][0] == flac_meta.PADDING and len(blocks[-1][1]) == 1024 + (len(tile) - aoff) // 1000
    assert hs + off == len(blob)


def test_extract_selection_and_converter_metadata(tmp_path):
    r = _small_raster()
    T = Affine(20.0, 0.0, 500000.0, 0.0, -20.0, 4200000.0)
    tiles = calculate_tiles(300, 260, 128)
    blob = assemble_streaming(tiles, oracle_encode_tiles(r, tiles, 5), r.shape, r.dtype, T, "EPSG:32633", 128)
    p = tmp_path / "s.flac"
    p.write_bytes(blob)
    sf = open_streaming(p)
    fr = sf.index["frames"]
    assert select_frame(fr, tile_id=4)["frame_id"] == 4
    assert select_frame(fr, last=True)["frame_id"] == len(tiles) - 1
    c = select_frame(fr, center=True)
    assert c["window"]["row_off"] == 128 and c["window"]["col_off"] == 128
    b = fr[7]["bbox"]
    assert select_frame(fr, bbox=[b[0] + 1, b[1] + 1, b[0] + 2, b[1] + 2])["frame_id"] == 7
    with pytest.raises(LookupError):
        select_frame(fr, bbox=[0, 0, 1, 1])
    tile = read_tile_bytes(p, fr[5], sf.header_size)
    tp = tmp_path / "t.flac"
    tp.write_bytes(tile)
    md = RasterFLACConverter()._read_embedded_metadata(tp)
    (row, col, h, w) = tiles[5]
    assert (md["width"], md["height"], md["count"], md["dtype"], md["crs"]) == (w, h, 2, "uint16", "EPSG:32633")
    assert md["nodata"] is None and md["spatial_tiling"] is False
    assert md["bounds"] == dict(zip(["left", "bottom", "right", "top"], bounds(window_transform(T, col, row), w, h)))


def test_raster_tags_order_and_values():
    T = Affine(1.0, 0.0, 0.0, 0.0, -1.0, 256.0)
    md = raster_metadata(256, 256, 3, np.uint8, "EPSG:4326", T, 1.0, 255.0, None)
    tags = raster_tags(md)
    assert [k for k, _ in tags] == [
        "TITLE", "DESCRIPTION", "ENCODER", "GEOSPATIAL_CRS", "GEOSPATIAL_WIDTH", "GEOSPATIAL_HEIGHT",
        "GEOSPATIAL_COUNT", "GEOSPATIAL_DTYPE", "GEOSPATIAL_NODATA", "GEOSPATIAL_DATA_MIN", "GEOSPATIAL_DATA_MAX",
        "GEOSPATIAL_TRANSFORM", "GEOSPATIAL_BOUNDS", "GEOSPATIAL_SPATIAL_TILING"]
    d = dict(tags)
    assert d["GEOSPATIAL_TRANSFORM"] == "[1.0, 0.0, 0.0, 0.0, -1.0, 256.0, 0.0, 0.0, 1.0]"
    assert d["GEOSPATIAL_BOUNDS"] == '{"left": 0.0, "bottom": 0.0, "right": 256.0, "top": 256.0}'
    assert d["GEOSPATIAL_DATA_MIN"] == "1.0" and d["GEOSPATIAL_NODATA"] == "None"


def test_geotiff_roundtrip(tmp_path, golden_dir):
    for name in ("sample_rgb.tif", "sample_dem.tif", "sample_multispectral.tif"):
        data, info = read_geotiff(golden_dir / name)
        out = tmp_path / name
        write_geotiff(out, data, transform=info.transform, crs=info.crs, nodata=info.nodata)
        d2, i2 = read_geotiff(out)
        assert np.array_equal(d2, data) and i2.transform == info.transform and i2.crs == info.crs
    for dt in (np.int8, np.uint32, np.int32, np.float32, np.float64):
        a = (np.arange(2 * 33 * 17) % 251).astype(dt).reshape(2, 33, 17)
        write_geotiff(tmp_path / "x.tif", a)
        assert np.array_equal(read_geotiff(tmp_path / "x.tif")[0], a)


# ----------------------------------------------------------------------------------- normalization host side
def test_denormalize_and_precision_loss_match_reference(golden_dir):
    v = np.load(golden_dir / "normalize_extra.npz")
    n = 0
    for k in v.files:
        if not (k.startswith("denorm__") and k.endswith("__in")):
            continue
        base = k[:-4]
        lo, hi, bps, scale = v[base + "__params"]
        p = normalization.NormalizationParams(float(lo), float(hi), str(v[base + "__dtype"]), int(bps), int(scale))
        out = normalization.denormalize_from_audio(v[k], p)
        assert out.dtype == v[base + "__out"].dtype and np.array_equal(out, v[base + "__out"]), base
        n += 1
    assert n == 6
    for row in json.loads((golden_dir / "precision_loss.json").read_text()):
        got = normalization.estimate_precision_loss(row["dtype"], row["min"], row["max"], row["bps"])
        assert got == row["out"], row


def test_audio_params_host(golden_dir):
    g = json.loads((golden_dir / "golden.json").read_text())
    for row in g["audio_params"]:
        class S:  # shape-only stand-in
            shape = tuple(row["shape"])
            ndim = 3
        assert normalization.calculate_audio_params(S, row["dtype"]) == (row["sample_rate"], row["bps"])
    assert normalization.get_dtype_info(np.uint16) == (0.0, 65535.0, True)
    assert normalization.get_dtype_info(np.float32) == (None, None, False)


def test_bench_gpus_flag_fails_loudly_without_enough_gpus():
    """``bench.py --gpus N`` starts its own ranks only onto visible GPUs: with none here it must
    exit non-zero before any rank starts, instead of timing one process and printing an ``n_gpus: 1`` line."""
    import os
    import subprocess
    import sys
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "FRA_DIST_BACKEND"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--config", "c3"], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode != 0 and "GPU(s) visible" in r.stderr and not r.stdout.strip()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--config", "c3"], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
