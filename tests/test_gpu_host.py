"""GPU tests of the reference-API host layer over the HIP library.

* ``normalize_to_audio`` on the GPU == the reference's normalization.py on every golden vector.
* pyflac-compatible ``StreamEncoder``: callback sequence (fLaC / STREAMINFO / VORBIS_COMMENT, then
  one call per frame with num_samples / current_frame) and bytes == the oracle.
* ``RasterFLACConverter.tiff_to_flac`` / ``flac_to_tiff``, ``create_streaming_flac`` (the north-star
  container, byte-identical to the oracle-assembled one, 1 or 2 device threads),
  ``SpatialFLACEncoder`` (+ stale index offsets, F6), and the CLI end to end.
"""
import json

import numpy as np
import pytest

import oracle as O
from flac_raster import _native as N
from flac_raster import flac_meta, normalization
from flac_raster.converter import RasterFLACConverter
from flac_raster.encoder import EncoderInitException, StreamEncoder, encode_array
from flac_raster.geo import Affine
from flac_raster.spatial_encoder import SpatialFLACEncoder, SpatialFLACStreamer
from flac_raster.streaming import assemble_streaming, create_streaming_flac, open_streaming
from flac_raster.synth import synth_window
from flac_raster.tiff import read_geotiff, write_geotiff
from flac_raster.tiles import calculate_tiles, encode_tiles
from oracle_tiles import oracle_encode_tiles

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    N.load()
    assert N.device_count() > 0, "no HIP device: GPU tests must not pass on a fallback"


def test_normalize_to_audio_golden_vectors(golden_dir):
    v = np.load(golden_dir / "normalize_vectors.npz")
    n = 0
    for k in v.files:
        if not k.endswith("__in"):
            continue
        base = k[:-4]
        bps = int(base.split("__")[1])
        audio, p = normalization.normalize_to_audio(v[k].reshape(-1, 1), bps)
        assert audio.dtype == v[base + "__out"].dtype, base
        assert np.array_equal(audio.reshape(-1), v[base + "__out"]), base
        assert np.array_equal(np.array([p.data_min, p.data_max]), v[base + "__mnmx"], equal_nan=True), base
        assert p.scale_factor == (32767 if bps == 16 else 8388607)
        n += 1
    assert n >= 70


def test_normalize_overrides_and_bps32(golden_dir):
    v = np.load(golden_dir / "normalize_extra.npz")
    n = 0
    for k in v.files:
        if not (k.startswith("norm__") and k.endswith("__in")):
            continue
        base = k[:-4]
        bps, lo, hi, pmin, pmax = v[base + "__args"]
        lo = None if np.isnan(lo) else float(lo)
        hi = None if np.isnan(hi) else float(hi)
        audio, p = normalization.normalize_to_audio(v[k].reshape(-1, 1), int(bps), lo, hi)
        assert np.array_equal(audio.reshape(-1), v[base + "__out"]), base
        assert (p.data_min, p.data_max) == (pmin, pmax), base
        n += 1
    assert n == 6


def test_normalize_sample_tiffs(golden_dir):
    g = json.loads((golden_dir / "golden.json").read_text())
    import hashlib
    for name in ("sample_rgb.tif", "sample_dem.tif", "sample_multispectral.tif"):
        data, _ = read_geotiff(golden_dir / name)
        audio, p = normalization.normalize_to_audio(data.transpose(1, 2, 0).reshape(-1, data.shape[0]), 16)
        assert hashlib.sha256(audio.tobytes()).hexdigest() == g["tiffs"][name]["audio_sha256"]
        assert (p.data_min, p.data_max) == (g["tiffs"][name]["data_min"], g["tiffs"][name]["data_max"])


def _rgb_audio(golden_dir):
    data, _ = read_geotiff(golden_dir / "sample_rgb.tif")
    return O.normalize(data.transpose(1, 2, 0).reshape(-1, 3), 16)[0]


def test_stream_encoder_callback_sequence(golden_dir):
    audio = _rgb_audio(golden_dir)
    calls = []
    enc = StreamEncoder(write_callback=lambda b, n, s, f: calls.append((bytes(b), n, s, f)), sample_rate=44100,
                        compression_level=5, blocksize=4096)
    enc._channels, enc._bits_per_sample = 3, 16  # what the reference sets; overridden by process (F3)
    enc.process(audio)
    # header at init (first process), then every block but the last (libFLAC keeps one sample of look-ahead)
    assert len(calls) == 3 + 15 and [c[1] for c in calls[:3]] == [4, 38, 44]
    assert enc.finish()
    ref, fb, _ = O.encode(audio, 44100, level=5, return_info=True)
    assert [c[1] for c in calls[:3]] == [4, 38, 44] and calls[0][0] == b"fLaC"
    assert all(c[2] == 0 and c[3] == 0 for c in calls[:3])
    fr = calls[3:]
    assert [c[1] for c in fr] == list(fb) and [c[3] for c in fr] == list(range(16))
    assert all(c[2] == 4096 for c in fr) and all(len(c[0]) == c[1] for c in calls)
    assert b"".join(c[0] for c in calls) == ref


def test_stream_encoder_incremental_emission(golden_dir):
    """pyflac/libFLAC call timing: frames are emitted during process() as soon as blocksize + 1 samples
    are buffered, numbered continuously across calls; the tail waits for finish()."""
    audio = _rgb_audio(golden_dir)
    calls = []
    enc = StreamEncoder(44100, lambda b, n, s, f: calls.append((bytes(b), s, f)), compression_level=5, blocksize=4096)
    fed = 0
    for part in np.array_split(audio, 13):  # 5041-5042 samples per call
        enc.process(part)
        fed += len(part)
        assert len(calls) == 3 + max(0, (fed - 1) // 4096)
    assert enc.finish()
    assert [c[2] for c in calls[3:]] == list(range(16)) and all(c[1] == 4096 for c in calls[3:])
    assert b"".join(c[0] for c in calls) == O.encode(audio, 44100, level=5)
    # exact multiples and single-sample calls
    calls.clear()
    enc = StreamEncoder(44100, lambda b, n, s, f: calls.append((bytes(b), s, f)), compression_level=5, blocksize=4096)
    enc.process(audio[:4096])
    assert len(calls) == 3
    enc.process(audio[4096:4097])
    assert len(calls) == 4 and calls[3][2] == 0
    enc.process(audio[4097:])
    enc.finish()
    assert b"".join(c[0] for c in calls) == O.encode(audio, 44100, level=5)


def test_stream_encoder_reused_input_buffer(golden_dir):
    """One caller buffer refilled between process() calls of <= blocksize samples (sf.read(out=buf)
    shape): the look-ahead samples the encoder keeps must be its own copy."""
    audio = _rgb_audio(golden_dir)
    out = bytearray()
    enc = StreamEncoder(44100, lambda b, n, s, f: out.extend(b), compression_level=5, blocksize=4096)
    buf = np.empty((3000, 3), np.int16)
    for a in range(0, len(audio), len(buf)):
        part = audio[a:a + len(buf)]
        buf[:len(part)] = part
        enc.process(buf[:len(part)])
        buf.fill(0x5A5A)  # the caller reuses its buffer
    enc.finish()
    assert bytes(out) == O.encode(audio, 44100, level=5)


def test_stream_encoder_multi_process_and_defaults(golden_dir):
    audio = _rgb_audio(golden_dir)
    out = bytearray()
    enc = StreamEncoder(44100, lambda b, n, s, f: out.extend(b), compression_level=1)  # blocksize 0 -> 1152
    for part in np.array_split(audio, 7):
        enc.process(part)
    enc.finish()
    assert bytes(out) == O.encode(audio, 44100, level=1, blocksize=1152)
    # int32 audio -> 32-bps FLAC (F3); last partial block
    x = np.random.default_rng(2).integers(-8388607, 8388607, size=(10000, 2)).astype(np.int32)
    assert encode_array(x, 48000, 8) == O.encode(x, 48000, level=8)
    with pytest.raises(EncoderInitException):
        StreamEncoder(44100, lambda *a: None).process(np.zeros((10, 1), np.int8))
    with pytest.raises(TypeError):
        StreamEncoder(44100, lambda *a: None).process([1, 2, 3])


def test_tiff_to_flac_and_back(tmp_path, golden_dir):
    conv = RasterFLACConverter()
    for name in ("sample_rgb.tif", "sample_dem.tif", "sample_multispectral.tif"):
        src = golden_dir / name
        out = tmp_path / (name + ".flac")
        conv.tiff_to_flac(src, out, 5)
        raw = out.read_bytes()
        data, info = read_geotiff(src)
        f = flac_meta.FLACFile(raw)
        assert f["GEOSPATIAL_WIDTH"] == [str(info.width)] and f["GEOSPATIAL_COUNT"] == [str(info.count)]
        assert f["GEOSPATIAL_CRS"] == [str(info.crs)] and f["GEOSPATIAL_DTYPE"] == [str(data.dtype)]
        audio, mn, mx = O.normalize(data.transpose(1, 2, 0).reshape(-1, info.count), 16)
        assert f["GEOSPATIAL_DATA_MIN"] == [str(float(mn))] and f["GEOSPATIAL_DATA_MAX"] == [str(float(mx))]
        ref = O.encode(audio, O.sample_rate_for_pixels(info.width * info.height), level=5)
        assert raw[f.audio_offset:] == ref[86:]  # frames identical to the oracle
        blocks, _ = flac_meta.parse_blocks(raw)
        assert blocks[-1][0] == flac_meta.PADDING and len(blocks[-1][1]) == 1024 + len(ref[86:]) // 1000
        back = tmp_path / (name + ".back.tif")
        conv.flac_to_tiff(out, back)
        d2, i2 = read_geotiff(back)
        assert d2.dtype == data.dtype and d2.shape == data.shape and i2.transform == info.transform
        assert np.array_equal(d2, data)  # ranges <= 16451: lossless through PCM_16 (F8)


def _synthetic_tif(tmp_path, kind=4, bands=4, H=1300, W=1100, dtype=np.uint16):
    r = synth_window(kind, 20260227, bands, H, W, 0, 0, H, W).astype(dtype)
    p = tmp_path / f"synth{kind}.tif"
    write_geotiff(p, r, transform=(10.0, 0.0, 300000.0, 0.0, -10.0, 5000040.0), crs="EPSG:32633")
    return p, r


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_streaming_container_equals_oracle(tmp_path, devices):
    p, r = _synthetic_tif(tmp_path)
    out = tmp_path / "s.flac"
    idx = create_streaming_flac(p, out, 512, 5, devices)
    tiles = calculate_tiles(r.shape[1], r.shape[2], 512)
    ref = assemble_streaming(tiles, oracle_encode_tiles(r, tiles, 5), r.shape, r.dtype,
                             Affine(10.0, 0.0, 300000.0, 0.0, -10.0, 5000040.0), "EPSG:32633", 512)
    assert out.read_bytes() == ref
    assert len(idx["frames"]) == len(tiles) == 9


def test_streaming_float32_32bps(tmp_path):
    p, r = _synthetic_tif(tmp_path, kind=5, bands=2, H=600, W=700, dtype=np.float32)
    out = tmp_path / "f.flac"
    create_streaming_flac(p, out, 256, 8)
    tiles = calculate_tiles(600, 700, 256)
    ref = assemble_streaming(tiles, oracle_encode_tiles(r, tiles, 8), r.shape, r.dtype,
                             Affine(10.0, 0.0, 300000.0, 0.0, -10.0, 5000040.0), "EPSG:32633", 256)
    assert out.read_bytes() == ref


def test_spatial_format(tmp_path):
    p, r = _synthetic_tif(tmp_path, H=900, W=700)
    out = tmp_path / "sp.flac"
    idx = SpatialFLACEncoder(tile_size=256).encode_spatial_flac(p, out, 5)
    raw = out.read_bytes()
    tiles = calculate_tiles(900, 700, 256)
    streams = oracle_encode_tiles(r, tiles, 5)
    # index offsets are pre-rewrite (F6): shift by the growth of the first header
    growth = len(raw) - sum(len(s.data) for s in streams)
    for fr, ts in zip(idx.frames, streams):
        start = fr.byte_offset + (growth if fr.frame_id > 0 else 0)
        if fr.frame_id == 0:
            assert raw[flac_meta.FLACFile(raw).audio_offset:fr.byte_size + growth] == ts.data[86:]
        else:
            assert raw[start:start + fr.byte_size] == ts.data
    f = flac_meta.FLACFile(raw)
    assert f["GEOSPATIAL_NUM_TILES"] == [str(len(tiles))] and f["GEOSPATIAL_DATA_MIN"] == [str(float(r.min()))]
    st = SpatialFLACStreamer(out)
    assert [x.to_dict() for x in st.spatial_index.frames] == [x.to_dict() for x in idx.frames]
    b = idx.frames[4].bbox
    assert st.get_byte_ranges_for_bbox((b[0] + 1, b[1] + 1, b[0] + 2, b[1] + 2)) == [
        (idx.frames[4].byte_offset, idx.frames[4].byte_offset + idx.frames[4].byte_size - 1)]


def test_cli_end_to_end(tmp_path):
    from typer.testing import CliRunner

    from flac_raster.cli import app

    p, r = _synthetic_tif(tmp_path, H=700, W=650)
    run = CliRunner().invoke
    s = tmp_path / "out_streaming.flac"
    res = run(app, ["convert", str(p), "-o", str(s), "--streaming", "--tile-size", "256"])
    assert res.exit_code == 0, res.output
    t = tmp_path / "tile.tif"
    res = run(app, ["extract", str(s), "-o", str(t), "--tile-id", "4"])
    assert res.exit_code == 0, res.output
    d, _ = read_geotiff(t)
    assert np.array_equal(d, r[:, 256:512, 256:512])  # range <= 16451 -> lossless (F8)
    assert open_streaming(s).index["frames"][4]["window"] == {"col_off": 256, "row_off": 256, "width": 256,
                                                              "height": 256}
    f = tmp_path / "std.flac"
    assert run(app, ["convert", str(p), "-o", str(f)]).exit_code == 0
    back = tmp_path / "back.tif"
    assert run(app, ["convert", str(f), "-o", str(back)]).exit_code == 0
    assert np.array_equal(read_geotiff(back)[0], r)
    assert run(app, ["info", str(f)]).exit_code == 0
    assert run(app, ["compare", str(p), str(back)]).exit_code == 0


def test_encode_tiles_device_split_identical():
    r = synth_window(3, 7, 1, 2048, 1536, 0, 0, 2048, 1536)
    tiles = calculate_tiles(2048, 1536, 512)
    a = encode_tiles(r, tiles, 5, [0])
    b = encode_tiles(r, tiles, 5, [0, 0, 0])
    assert [x.data for x in a] == [x.data for x in b]
