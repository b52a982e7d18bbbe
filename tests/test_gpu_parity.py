"""GPU parity: the HIP encoder's FLAC frames must be byte-identical to the CPU oracle's
(oracle/fr_oracle.c, FRA-1 rule) on the same inputs, and must decode bit-exactly to
normalize_to_audio(input) -- the reference's compare_tiffs round-trip criterion at codec level.

Inputs: the reference's own test rasters (tests/golden/*.tif), synthetic windows of the benchmark
configurations (flac_raster.synth, identical on CPU and GPU), and edge cases (constant, NaN, inf,
tiny/ragged windows, partial last frames, every compression level, 16- and 32-bps paths).
"""
import json

import numpy as np
import pytest

import oracle as O
from flac_raster import _native as N
from flac_raster.synth import synth_window
from flac_raster.tiff import read_geotiff

pytestmark = pytest.mark.gpu


def _diag(got: bytes, exp: bytes, fb):
    n = min(len(got), len(exp))
    i = next((k for k in range(n) if got[k] != exp[k]), n)
    f, acc = 0, 0
    for f, b in enumerate(fb):
        if acc + b > i:
            break
        acc += b
    return f"len got {len(got)} exp {len(exp)}; first diff byte {i} (frame {f}, +{i - acc})"


def check_windows(raster, windows, level, norm, blocksize=4096):
    """Encode windows on the GPU and compare each stream with the oracle."""
    infos, frames = N.encode_windows(raster, windows, level=level, norm=norm, blocksize=blocksize)
    bps = 16 if norm == 16 else 24
    total = 0
    for (r0, c0, h, w), info in zip(windows, infos):
        tile = raster[:, r0:r0 + h, c0:c0 + w]
        inter = tile.transpose(1, 2, 0).reshape(-1, tile.shape[0])
        audio, mn, mx = O.normalize(inter, bps)
        sr = O.sample_rate_for_pixels(h * w)
        assert info.sample_rate == sr
        assert np.array_equal(np.array([info.data_min, info.data_max]), np.array([mn, mx]), equal_nan=True)
        exp, fb, _ = O.encode(audio, sr, level=level, blocksize=blocksize, with_header=False, return_info=True)
        got = frames[info.offset: info.offset + info.frame_bytes]
        assert got == exp, f"window {(r0, c0, h, w)} level {level}: " + _diag(got, exp, fb)
        if h * w:
            hdr = O.stream_header(tile.shape[0], 16 if norm == 16 else 32, sr, blocksize)
            dec, _, _, _ = O.decode(hdr + got)
            assert np.array_equal(dec, audio.astype(np.int32))
        total += len(got)
    return total


def tiles(H, W, t):
    return [(r, c, min(t, H - r), min(t, W - c)) for r in range(0, H, t) for c in range(0, W, t)]


def test_device_visible():
    assert N.device_count() >= 1


def test_stream_header_matches_oracle():
    for ch, bps, sr in [(1, 16, 44100), (3, 16, 44100), (4, 16, 48000), (8, 32, 44100), (2, 32, 192000)]:
        assert N.stream_header(ch, bps, sr, 4096) == O.stream_header(ch, bps, sr, 4096)


@pytest.mark.parametrize("name", ["sample_rgb.tif", "sample_dem.tif", "sample_multispectral.tif"])
@pytest.mark.parametrize("level", [0, 1, 3, 5, 6, 8])
def test_reference_rasters_standard_format(golden_dir, name, level):
    data, _ = read_geotiff(golden_dir / name)
    B, H, W = data.shape
    check_windows(data, [(0, 0, H, W)], level, 16)


def test_sample_rgb_size_vs_libflac(golden_dir):
    """-c 5 size vs the committed libFLAC 1.4.3 golden (178,857 frame bytes)."""
    data, _ = read_geotiff(golden_dir / "sample_rgb.tif")
    infos, frames = N.encode_windows(data, [(0, 0, 256, 256)], level=5, norm=16)
    golden = (golden_dir / "sample_rgb.flac").read_bytes()
    ratio = len(frames) / (len(golden) - 86)
    assert ratio <= 1.02, ratio


@pytest.mark.parametrize("level", [5])
def test_sample_dem_spatial_tiles(golden_dir, level):
    data, _ = read_geotiff(golden_dir / "sample_dem.tif")
    check_windows(data, tiles(512, 512, 256), level, 16)


def test_synthetic_s2_tiles_level5():
    """C4-like: 4-band uint16, tile 1024 incl. ragged edge tiles (2832-sample last frame)."""
    H = W = 1764  # 1024 + 740 -> full, 1024x740, 740x1024, 740x740 tiles
    r = synth_window(4, 20260227, 4, H, W)
    check_windows(r, tiles(H, W, 1024), 5, 16)


@pytest.mark.parametrize("level", [0, 2, 4, 7])
def test_synthetic_s2_levels(level):
    r = synth_window(4, 7, 4, 300, 700)
    check_windows(r, tiles(300, 700, 256), level, 16)


def test_synthetic_dem_tiles():
    r = synth_window(3, 11, 1, 1024, 1024)
    check_windows(r, tiles(1024, 1024, 512), 5, 16)


@pytest.mark.parametrize("level", [5, 8])
def test_float32_24bit_path(level):
    """C5-like: 8-band float32 -> int32 audio -> 32-bps FLAC."""
    r = synth_window(5, 3, 8, 512, 512)
    check_windows(r, tiles(512, 512, 256), level, 24)


@pytest.mark.parametrize("dtype", ["uint8", "int8", "uint16", "int16", "uint32", "int32", "float32", "float64"])
def test_all_dtypes(dtype):
    rng = np.random.default_rng(abs(hash(dtype)) % 1000)
    base = synth_window(4, 5, 3, 200, 300).astype(np.float64)
    if dtype.startswith("float"):
        r = (base / 1000.0).astype(dtype)
    else:
        info = np.iinfo(dtype)
        r = np.clip(base - 1000 + (info.min + info.max) // 2, info.min, info.max).astype(dtype)
    for norm in (16, 24):
        check_windows(r, tiles(200, 300, 128), 5, norm)


def test_edge_cases():
    z = np.zeros((2, 64, 64), np.uint16)
    check_windows(z, [(0, 0, 64, 64)], 5, 16)  # constant -> all -32767, CONSTANT subframes
    r = synth_window(4, 9, 2, 97, 131)
    wins = [(0, 0, 1, 1), (0, 0, 3, 5), (5, 7, 1, 131 - 7), (10, 0, 87, 1), (0, 0, 97, 131), (40, 50, 57, 81)]
    check_windows(r, wins, 5, 16)
    f = synth_window(5, 9, 3, 64, 80)
    f[0, ::7, ::3] = np.nan
    f[1, 5, 5] = np.inf
    check_windows(f, [(0, 0, 64, 80), (0, 0, 32, 40)], 5, 16)
    check_windows(f, [(0, 0, 64, 80)], 8, 24)
    allnan = np.full((1, 40, 40), np.nan, np.float32)
    check_windows(allnan, [(0, 0, 40, 40)], 5, 16)
    # r06 (float32 quotient by Markstein's correction, IEEE division only for an infinite range): -inf in one tile,
    # a one-ulp range, subnormal and huge values, against the oracle's IEEE division
    g = synth_window(5, 10, 2, 64, 96)
    g[0, 3, 70] = -np.inf
    g[1, 40:, :48] = np.float32(1e-40)  # subnormal float32
    g[1, 40:, 48:] = np.float32(3e38)
    check_windows(g, [(0, 0, 64, 48), (0, 48, 64, 48), (32, 0, 32, 96)], 5, 24)
    ulp = np.full((1, 32, 64), np.float32(0.15), np.float32)
    ulp[0, ::3, ::5] = np.nextafter(np.float32(0.15), np.float32(1))
    check_windows(ulp, [(0, 0, 32, 64)], 8, 24)
    check_windows(ulp, [(0, 0, 32, 64)], 5, 16)


def test_small_blocksizes():
    r = synth_window(4, 2, 2, 100, 100)
    for bs in (16, 192, 1000, 1152, 4096):
        check_windows(r, [(0, 0, 100, 100)], 5, 16, blocksize=bs)


def test_interleaved_pyflac_path(golden_dir):
    """pyflac StreamEncoder semantics: pre-normalised int16/int32 audio in."""
    data, _ = read_geotiff(golden_dir / "sample_rgb.tif")
    inter = data.transpose(1, 2, 0).reshape(-1, 3)
    audio, _, _ = O.normalize(inter, 16)
    info, frames = N.encode_interleaved(audio, 44100, level=5)
    assert frames == O.encode(audio, 44100, level=5, with_header=False)
    a32 = (audio.astype(np.int32) * 255)
    info, frames = N.encode_interleaved(a32, 44100, level=5)
    assert frames == O.encode(a32, 44100, level=5, with_header=False)
    assert info.bps == 32


def test_synth_matches_numpy_mirror():
    ctx = N.default_context(0)
    for kind, bands, dt in [(3, 1, np.int16), (4, 4, np.uint16), (5, 8, np.float32)]:
        H, W = 300, 520
        dev = ctx.alloc(bands * H * W * np.dtype(dt).itemsize)
        try:
            ctx.synth(kind, 99, bands, H, W, dev)
            got = np.empty((bands, H, W), dt)
            ctx.d2h(got, dev)
        finally:
            ctx.free(dev)
        exp = synth_window(kind, 99, bands, H, W)
        assert np.array_equal(got, exp), kind


@pytest.mark.parametrize("groups", [2, 3, 8])
def test_frame_groups_pipelined_equal_serial(monkeypatch, groups):
    """fra_plan_execute with FRA_GROUPS > 1 (window runs on their own streams, per-group scans joined by
    k_group_offsets) must give the same stream table and bytes as the serial plan; a few streams are
    also checked against the oracle.  >= 4096 frames so the plan really splits."""
    H, W = 2048, 8200
    r = synth_window(3, 21, 1, H, W)
    wins = tiles(H, W, 512) + [(0, 0, 0, 0)]  # an empty window in the last group
    monkeypatch.setenv("FRA_GROUPS", "1")
    i1, f1 = N.encode_windows(r, wins, level=5, norm=16, path="device")
    monkeypatch.setenv("FRA_GROUPS", str(groups))
    ig, fg = N.encode_windows(r, wins, level=5, norm=16, path="device")
    assert fg == f1
    assert [(a.offset, a.frame_bytes, a.nframes) for a in ig] == [(a.offset, a.frame_bytes, a.nframes) for a in i1]
    check_windows(r, [wins[0], wins[len(wins) // 2], wins[-2]], 5, 16)


def test_minmax_one_vector_wide_windows():
    """Windows exactly one load vector wide (8 int16 / 16 uint8 / 4 float32 columns) take the vectorised
    min/max path with one vector per row (regression: its row divisor wrapped to 0)."""
    for dt, w in ((np.int16, 8), (np.uint8, 16), (np.float32, 4)):
        r = synth_window(3, 5, 2, 96, 64).astype(dt)
        wins = [(0, 0, 96, 32), (0, 64 - w, 96, w), (32, 32, 64, w)]
        check_windows(r, wins, 5, 16)


@pytest.mark.parametrize("blocksize", [4096, 1000])
def test_32bps_verbatim_and_wasted_bits(blocksize):
    """32-bps VERBATIM subframes (full-range noise, also with wasted bits) and partial frames: the
    32-bps encoder writes VERBATIM words straight from the sample buffer (its bit buffer aliases it)."""
    rng = np.random.default_rng(blocksize)
    n = 3 * 4096 + 1234
    full = rng.integers(-2**31, 2**31, size=(n, 2), dtype=np.int64).astype(np.int32)
    wasted = (rng.integers(-2**26, 2**26, size=(n, 2)) << 5).astype(np.int32)
    mixed = rng.integers(-3000, 3000, size=(n, 2)).astype(np.int32)
    mixed[::97] = rng.integers(-2**30, 2**30, size=mixed[::97].shape)
    for a in (full, wasted, mixed):
        info, frames = N.encode_interleaved(a, 44100, level=8, blocksize=blocksize)
        assert frames == O.encode(a, 44100, level=8, blocksize=blocksize, with_header=False)
        dec, _, _, _ = O.decode(O.stream_header(2, 32, 44100, blocksize) + frames)
        assert np.array_equal(dec, a)


@pytest.mark.parametrize("level", [0, 1, 3, 5, 8])
def test_two_band_mid_side(golden_dir, level):
    """FRA-1 3.1b: 2-band rasters (16-bps streams) choose among L/R, L/S, S/R, M/S per frame at the
    levels whose libFLAC preset enables mid-side; the side channel (17-bit samples) runs on the 32-bit
    instance.  Ragged tiles cover partial frames."""
    data, _ = read_geotiff(golden_dir / "sample_rgb.tif")
    check_windows(np.ascontiguousarray(data[:2]), [(0, 0, 256, 256), (7, 3, 100, 91)], level, 16)
    r = synth_window(4, 31, 2, 700, 900)
    check_windows(r, tiles(700, 900, 512), level, 16)
    c = r.copy()
    c[1] = c[0]  # identical bands: the side channel is all zeros (CONSTANT)
    check_windows(c, [(0, 0, 300, 900)], level, 16)


def test_two_channel_pyflac_path_mid_side():
    rng = np.random.default_rng(5)
    base = np.cumsum(rng.integers(-40, 41, size=(30000, 1)), axis=0)
    a = np.clip(np.concatenate([base, base + rng.integers(-9, 10, size=(30000, 1))], axis=1), -32768, 32767)
    a = a.astype(np.int16)
    for level in (2, 5, 8):
        info, frames = N.encode_interleaved(a, 44100, level=level)
        assert frames == O.encode(a, 44100, level=level, with_header=False)
        dec, _, _, _ = O.decode(O.stream_header(2, 16, 44100, 4096) + frames)
        assert np.array_equal(dec, a.astype(np.int32))
    a32 = a.astype(np.int32) * 97  # 32-bps: independent channels only
    info, frames = N.encode_interleaved(a32, 44100, level=5)
    assert frames == O.encode(a32, 44100, level=5, with_header=False)


# ---- k_analyze_w (one subframe per wave: full frames of <= 16-bit LUT rasters, levels 3-6, 8-byte sample vectors)
@pytest.fixture(params=["1", "0"], ids=["keep17", "keep16"])
def require_wave(monkeypatch, request):
    """The plan must take k_analyze_w (FRA_REQUIRE_WAVE=1: the library fails a plan that would not), once with each
    instance of it (FRA_KEEP17=1: kept residuals up to 17 bits; 0: up to 16, the rest through the sample path)."""
    monkeypatch.setenv("FRA_REQUIRE_WAVE", "1")
    monkeypatch.setenv("FRA_KEEP17", request.param)


@pytest.mark.parametrize("level", [3, 4, 5, 6])
@pytest.mark.parametrize("dtype", ["uint8", "int16"])
def test_wave_kernel_levels_dtypes(require_wave, level, dtype):
    """Every level the wave kernel takes, both LUT widths, full + partial frames (partial ones go to
    k_analyze through the frame list) against the oracle.  Window columns and widths keep every 8-byte
    sample vector inside a row (the wave path's condition), which FRA_REQUIRE_WAVE checks."""
    r = synth_window(4 if dtype == "uint8" else 3, 7 + level, 2, 300, 704).astype(np.float64)
    info = np.iinfo(dtype)
    r = np.clip(r / r.max() * (info.max - info.min) + info.min, info.min, info.max).astype(dtype)
    check_windows(r, [(0, 0, 300, 704), (0, 0, 64, 64), (17, 8, 131, 256)], level, 16)


def test_require_wave_rejects_other_paths(monkeypatch):
    """FRA_REQUIRE_WAVE=1 fails a plan outside the wave kernel's scope (level 8), so the tests above prove the
    wave kernel ran."""
    monkeypatch.setenv("FRA_REQUIRE_WAVE", "1")
    r = synth_window(4, 3, 1, 64, 256)
    with pytest.raises(N.NativeError):
        N.encode_windows(r, [(0, 0, 64, 256)], level=8, norm=16)


@pytest.mark.parametrize("keep17", ["1", "0"])
@pytest.mark.parametrize("kind,bands,tile", [(4, 4, 1024), (3, 1, 512)])
def test_wave_kernel_equals_workgroup_kernel(monkeypatch, kind, bands, tile, keep17):
    """k_analyze_w (both instances: kept residuals up to 17 or 16 bits) and k_analyze (FRA_ANALYZE_WG=1) produce the
    same bytes on a C4-like scene and on a C3-like int16 DEM (whose LPC residuals often pass 2^16: 17-bit kept
    residuals, or the sample path with codes in the LDS bit buffer)."""
    H = W = 1300
    r = synth_window(kind, 99, bands, H, W)
    wins = tiles(H, W, tile)
    monkeypatch.setenv("FRA_KEEP17", keep17)
    _, wave = N.encode_windows(r, wins, level=5, norm=16)
    monkeypatch.setenv("FRA_ANALYZE_WG", "1")
    _, wg = N.encode_windows(r, wins, level=5, norm=16)
    assert wave == wg
    if kind == 3:  # and against the oracle on a few tiles
        check_windows(r, wins[:2] + wins[-1:], 5, 16)


def _noise_then_smooth(n_frames=3, seed=5):
    """1-band uint16 rows whose frames start with 1024 samples of full-range noise followed by a slow ramp:
    the first quarter costs ~17 bits/sample, so the encoded bits of chunks 0-63 run past their own sample
    words in the LDS bit buffer (k_analyze_w encodes such a subframe straight into the slot)."""
    rng = np.random.default_rng(seed)
    x = np.empty(4096 * n_frames, np.uint16)
    for f in range(n_frames):
        blk = x[4096 * f: 4096 * (f + 1)]
        blk[:1024] = rng.integers(0, 65536, 1024)
        blk[1024:] = (np.arange(3072) * 3 + 1000 * f).astype(np.uint16)
    return x.reshape(1, -1, 4096)


@pytest.mark.parametrize("level", [3, 5])
def test_wave_kernel_noise_verbatim(require_wave, level):
    """Full-range noise: k_analyze_w's kept LPC winner is not smaller than VERBATIM, so the wave reloads the
    samples and writes VERBATIM from them (no hand-back); mixed with smooth bands in the same frames."""
    rng = np.random.default_rng(11 + level)
    r = synth_window(4, 5, 3, 256, 512)
    r[1] = rng.integers(0, 65536, size=r[1].shape, dtype=np.uint16)
    r[2, :64] = rng.integers(0, 65536, size=(64, 512), dtype=np.uint16)
    check_windows(r, [(0, 0, 256, 512), (0, 0, 100, 300)], level, 16)


@pytest.mark.parametrize("level", [0, 5, 6])
def test_wave_kernel_incompressible_start(level):
    r = _noise_then_smooth()
    check_windows(r, [(0, 0, r.shape[1], 4096)], level, 16)


@pytest.mark.parametrize("amp", [2000, 9000, 15000, 24000])
def test_wave_kernel_large_rice_parameters(require_wave, amp):
    """Noisy rasters whose kept LPC residuals still fit 16 bits but need Rice parameters up to 15-16: the packed
    u16 shift-and-dot2 sums of the exact pass (shift counts capped, pairs weighted 0 past 15) against the oracle."""
    rng = np.random.default_rng(amp)
    base = synth_window(4, 23, 2, 128, 512).astype(np.int64)
    r = np.clip(base // 4 + rng.integers(-amp, amp + 1, size=base.shape), 0, 65535).astype(np.uint16)
    check_windows(r, [(0, 0, 128, 512), (0, 0, 64, 256)], 5, 16)


# ---- 32-bps full + partial frames at levels 7-8 (k_analyze<true, 12>; r05's opt-in one-wave k_analyze_w32, which
# these cases pinned, lost to it and was removed in r06)
@pytest.mark.parametrize("level", [7, 8])
def test_32bps_levels_full_and_partial_frames(level):
    """Both high levels of the 32-bps path (3 / 6 apodization windows, lag 12), full and partial frames."""
    r = synth_window(5, 9 + level, 3, 300, 704).astype(np.float32)
    check_windows(r, [(0, 0, 300, 704), (0, 0, 64, 64), (17, 8, 131, 256)], level, 24)


def test_32bps_noise_constant_and_overrun():
    """Full-range noise bands (VERBATIM), constant frames, and frames whose first quarter is noise before a smooth
    rest (encoded bits overrun the samples they alias)."""
    rng = np.random.default_rng(31)
    r = synth_window(5, 5, 3, 256, 512).astype(np.float32)
    r[1] = rng.standard_normal(r[1].shape).astype(np.float32)
    r[2, :64] = 7.25
    x = np.empty((1, 48, 1024), np.float32)
    for f in range(3):
        blk = x[0, 16 * f:16 * (f + 1)].reshape(-1)
        blk[:1024] = rng.standard_normal(1024)
        blk[1024:] = np.linspace(0.0, 1.0 + f, blk.size - 1024)
    check_windows(r, [(0, 0, 256, 512), (0, 0, 64, 512)], 8, 24)
    check_windows(x, [(0, 0, 48, 1024)], 8, 24)


def test_wave_kernel_constant_and_two_valued(require_wave):
    """Constant frames (CONSTANT subframes), two-valued frames and their mix in one stream."""
    base = synth_window(3, 11, 1, 64, 192)[0].astype(np.int64)
    x = np.empty((1, 64 * 3, 192), np.int16)
    x[0, :64] = ((base % 4000) * 8 - 16000).astype(np.int16)
    x[0, 64:128] = 1234
    x[0, 128:] = np.where(base % 2 == 0, -5, 7).astype(np.int16)
    check_windows(x, [(0, 0, 64, 192), (64, 0, 64, 192), (128, 0, 64, 192), (0, 0, 192, 192)], 5, 16)


@pytest.mark.parametrize("level", [3, 5, 6])
def test_integer_autocorrelation_full_scale(level):
    """FRA-1 3.5b at the int16 extremes (pyflac path, pre-normalised audio): full-scale square waves (-32768 /
    32767: signed high bytes -128 / 127, low bytes 0 / 255), a full-range ramp and a slow sine with the extremes
    in the plateau and the tapers of the windows (level 6: the two partial tukeys, zero blocks of the matrix-core
    sums), 4,096-sample frames plus a partial last frame."""
    n = 4096 * 6 + 1000
    i = np.arange(n)
    sq = np.where((i // 37) % 2 == 0, -32768, 32767)
    ramp = ((i * 16) % 65536) - 32768
    sine = np.round(32767 * np.sin(i / 300.0))
    mix = np.where(i < n // 2, sq, sine)
    for sig in (sq, ramp, sine, mix):
        audio = sig.astype(np.int16).reshape(-1, 1)
        _, frames = N.encode_interleaved(audio, 44100, level=level)
        assert frames == O.encode(audio, 44100, level=level, with_header=False)
    stereo = np.stack([sq, sine], axis=1).astype(np.int16)  # two channels: mid / side at levels 5-6
    _, frames = N.encode_interleaved(stereo, 44100, level=level)
    assert frames == O.encode(stereo, 44100, level=level, with_header=False)
