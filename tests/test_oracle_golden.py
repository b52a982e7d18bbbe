"""CPU tests: the oracle (oracle/fr_oracle.c) pinned against the reference's golden artefacts.

* normalize_to_audio: every vector generated from the reference's own normalization.py
  (tests/golden/make_golden.py) must match bit for bit, plus the three sample TIFFs' hashes.
* decoder KAT: the committed libFLAC 1.4.3 output test_data/sample_rgb.flac decodes to exactly
  normalize_to_audio(sample_rgb.tif) (F10), with every CRC-8/CRC-16 verified.
* encoder: every encoded stream decodes bit-exactly; -c 5 size within 2 % of libFLAC's golden.
* calculate_audio_params: sample rate / bps rule vs the reference outputs.
"""
import hashlib
import json

import numpy as np
import pytest

import oracle as O
from flac_raster.tiff import read_geotiff


@pytest.fixture(scope="module")
def golden(golden_dir):
    return json.loads((golden_dir / "golden.json").read_text())


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_normalize_vectors_match_reference(golden_dir):
    v = np.load(golden_dir / "normalize_vectors.npz")
    n = 0
    for k in v.files:
        if not k.endswith("__in"):
            continue
        base = k[:-4]
        bps = int(base.split("__")[1])
        out, mn, mx = O.normalize(v[k], bps)
        exp = v[base + "__out"]
        assert out.dtype == exp.dtype, base
        assert np.array_equal(out, exp), base
        assert np.array_equal(np.array([mn, mx]), v[base + "__mnmx"], equal_nan=True), base
        n += 1
    assert n >= 70


@pytest.mark.parametrize("name", ["sample_rgb.tif", "sample_dem.tif", "sample_multispectral.tif"])
def test_sample_tiffs_normalize(golden_dir, golden, name):
    g = golden["tiffs"][name]
    data, info = read_geotiff(golden_dir / name)
    assert list(data.shape) == g["shape"] and str(data.dtype) == g["dtype"]
    assert sha(data) == g["raw_sha256"]
    inter = data.transpose(1, 2, 0).reshape(-1, data.shape[0])
    audio, mn, mx = O.normalize(inter, g["bps"])
    assert (mn, mx) == (g["data_min"], g["data_max"])
    assert sha(audio) == g["audio_sha256"]
    assert O.sample_rate_for_pixels(data.shape[1] * data.shape[2]) == g["sample_rate"]
    assert list(info.transform[:6]) == g["transform"][:6]
    assert info.crs == g["crs"]


def test_decode_libflac_golden(golden_dir, golden):
    flac = (golden_dir / "sample_rgb.flac").read_bytes()
    dec, sr, bps, nframes = O.decode(flac)
    assert (sr, bps, nframes, dec.shape) == (44100, 16, 16, (65536, 3))
    assert sha(dec.astype(np.int16)) == golden["tiffs"]["sample_rgb.tif"]["audio_sha256"]


def test_decoder_rejects_corruption(golden_dir):
    flac = bytearray((golden_dir / "sample_rgb.flac").read_bytes())
    flac[5000] ^= 0x10
    with pytest.raises(ValueError):
        O.decode(bytes(flac))


def test_golden_header_layout(golden_dir):
    """F4: fLaC + STREAMINFO(min=max 4096, sizes 0, total 0, MD5 0) + VORBIS_COMMENT = 86 bytes."""
    flac = (golden_dir / "sample_rgb.flac").read_bytes()
    ours = O.stream_header(3, 16, 44100, 4096)
    assert len(ours) == 86
    assert ours[:42] == flac[:42]          # identical STREAMINFO
    assert ours[42:46] == flac[42:46]      # VC block header: last flag, type 4, length 40
    assert flac[46:50] == b"\x20\x00\x00\x00"  # 32-byte vendor string in both


@pytest.mark.parametrize("level", range(9))
def test_encode_roundtrip_all_levels(golden_dir, level):
    data, _ = read_geotiff(golden_dir / "sample_multispectral.tif")
    inter = data.transpose(1, 2, 0).reshape(-1, data.shape[0])
    audio, _, _ = O.normalize(inter, 16)
    enc = O.encode(audio, 44100, level=level)
    dec, sr, bps, _ = O.decode(enc)
    assert np.array_equal(dec, audio.astype(np.int32)) and sr == 44100 and bps == 16


def test_size_vs_libflac_c2(golden_dir):
    data, _ = read_geotiff(golden_dir / "sample_rgb.tif")
    audio, _, _ = O.normalize(data.transpose(1, 2, 0).reshape(-1, 3), 16)
    frames = O.encode(audio, 44100, level=5, with_header=False)
    golden_frames = len((golden_dir / "sample_rgb.flac").read_bytes()) - 86
    assert golden_frames == 178857
    assert len(frames) / golden_frames <= 1.02


def test_encode_edge_cases():
    rng = np.random.default_rng(1)
    for n, ch in [(1, 1), (2, 2), (15, 3), (16, 1), (17, 8), (4095, 2), (4096, 1), (4097, 4), (12289, 1)]:
        x = rng.integers(-32768, 32767, size=(n, ch)).astype(np.int16)
        dec, *_ = O.decode(O.encode(x, 44100, level=5))
        assert np.array_equal(dec, x.astype(np.int32)), (n, ch)
    # 32-bps: full int32 range (fixed predictors overflow -> other models / verbatim)
    x = rng.integers(-2**31, 2**31 - 1, size=(5000, 2), dtype=np.int64).astype(np.int32)
    for lvl in (0, 5, 8):
        dec, _, bps, _ = O.decode(O.encode(x, 44100, level=lvl))
        assert bps == 32 and np.array_equal(dec, x)
    # constant and wasted bits
    c = np.full((5000, 2), -32767, np.int16)
    assert np.array_equal(O.decode(O.encode(c, 44100))[0], c.astype(np.int32))
    wb = (rng.integers(-100, 100, size=(9000, 1)) * 64).astype(np.int16)
    assert np.array_equal(O.decode(O.encode(wb, 44100))[0], wb.astype(np.int32))


def test_audio_params_match_reference(golden):
    for row in golden["audio_params"]:
        shape = row["shape"]
        assert O.sample_rate_for_pixels(shape[1] * shape[2]) == row["sample_rate"]
        bps = 16 if row["dtype"] in ("uint8", "int8", "uint16", "int16") else 24
        assert bps == row["bps"]


def test_window_and_lpc_primitives():
    w = O.window_set(4096, 3)
    assert w.shape == (6, 4096)
    assert w[0, 0] == 0.0 and w[0, 2048] == 1.0 and w[1, 2048:].max() == 0.0
    rng = np.random.default_rng(3)
    x = np.cumsum(rng.normal(size=4096)).astype(np.float32)
    ac = O.autocorr(x, 8)
    assert ac[0] > 0 and np.all(np.abs(ac[1:]) <= ac[0])
    # FRA-1 3.5b: integer windowed samples, exact sums (= numpy int64), extremes included
    v = np.clip(np.rint(x * 3000.0), -32768, 32767).astype(np.int32)
    v[:3] = [-32768, 32767, -32768]
    ai = O.autocorr_int(v, 8)
    ref = [int(np.dot(v[: 4096 - l].astype(np.int64), v[l:].astype(np.int64))) for l in range(9)]
    assert [int(t) for t in ai] == ref and ai.dtype == np.float64
    lp, err, n = O.levinson(ac, 8)
    assert n == 8 and np.all(np.diff(err) <= 0)
    q, sh = O.quantize(lp[1], 2, 12)
    assert 0 <= sh <= 15 and np.all(np.abs(q) < 2048)


def test_oracle_mid_side_round_trip_and_gain(golden_dir):
    """FRA-1 3.1b on the CPU: 2-channel 16-bps streams decode bit-exactly (oracle and product decoders)
    and are never larger than independent coding (the side/mid choice is a per-frame minimum)."""
    import numpy as np

    import oracle as O
    from flac_raster import _native as N
    from flac_raster.tiff import read_geotiff

    rgb, _ = read_geotiff(golden_dir / "sample_rgb.tif")
    for bands in ((0, 1), (1, 2)):
        a, _, _ = O.normalize(rgb[list(bands)].transpose(1, 2, 0).reshape(-1, 2), 16)
        for level in (1, 5, 8):
            ms = O.encode(a, 44100, level=level)
            O.set_stereo(False)
            try:
                ind = O.encode(a, 44100, level=level)
            finally:
                O.set_stereo(True)
            assert len(ms) <= len(ind)
            assert np.array_equal(O.decode(ms)[0], a.astype(np.int32))
            assert np.array_equal(N.decode(ms)[0], a.astype(np.int32))


def test_lpc_window_pruning_costs_little(golden_dir):
    """FRA-1 3.7b (r06): at levels 7-8 only the LPC window with the best window score gets residual sums and a
    partition search (the GPU's k_analyze then sums 1 model instead of up to 6).  On the reference's rasters the
    rule costs at most 0.1 % of the frame bytes against evaluating every window, the streams decode bit-exactly,
    and levels <= 6 are unchanged (their level-table entry keeps every window)."""
    from flac_raster.synth import synth_window

    cases = []
    for name in ("sample_rgb.tif", "sample_dem.tif", "sample_multispectral.tif"):
        d, _ = read_geotiff(golden_dir / name)
        cases.append((O.normalize(d.transpose(1, 2, 0).reshape(-1, d.shape[0]), 16)[0], 16))
    t = synth_window(5, 20260227, 8, 32768, 32768, 4096, 8192, 256, 512).astype(np.float32)  # C5-like, 32 bps
    cases.append((O.normalize(t.transpose(1, 2, 0).reshape(-1, 8), 24)[0], 32))
    try:
        for a, bps in cases:
            for level in (6, 7, 8):
                rule = O.encode(a, 44100, level=level, with_header=False)
                O.set_lpc_keep(0)
                every = O.encode(a, 44100, level=level, with_header=False)
                O.set_lpc_keep(-1)
                if level == 6:
                    assert rule == every
                else:
                    assert len(rule) <= 1.001 * len(every), (level, bps, len(rule), len(every))
                dec = O.decode(O.stream_header(a.shape[1], bps, 44100) + rule)[0]
                assert np.array_equal(dec, a.astype(np.int32))
    finally:
        O.set_lpc_keep(-1)
