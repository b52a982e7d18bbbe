"""GPU tests of the PCIe-inclusive path: fra_plan_encode_host (row bands: H2D of band
b+1 || kernels of band b || D2H of band b-1) must give exactly the bytes and stream table of the
device-resident path, for page-locked and pageable buffers, strided raster views, non-monotone window
orders (single-band fallback) and a too-small output buffer; and GeoTIFFs in the compressions GDAL
writes (LZW, deflate, predictors 2 and 3) must reach the same container bytes as the oracle."""
import numpy as np
import pytest

from flac_raster import _native as N
from flac_raster.geo import Affine
from flac_raster.streaming import assemble_streaming, create_streaming_flac
from flac_raster.synth import synth_window
from flac_raster.tiles import calculate_tiles
from oracle_tiles import oracle_encode_tiles

pytestmark = pytest.mark.gpu


def _device_path(r, wins, level, norm):
    return N.encode_windows(r, wins, level=level, norm=norm, path="device")


def _table(infos):
    return [(i.offset, i.frame_bytes, i.nframes, i.sample_rate, i.data_min, i.data_max) for i in infos]


@pytest.mark.parametrize("kind,bands,H,W,tile,dtype,level,norm", [
    (3, 1, 4096, 4096, 512, np.int16, 5, 16),      # C3-like: 8 row bands
    (4, 4, 3600, 3600, 1024, np.uint16, 5, 16),    # C4-like: ragged edge tiles
    (5, 3, 3072, 3072, 512, np.float32, 8, 24),    # C5-like: 32-bps
])
def test_encode_host_equals_device_path(kind, bands, H, W, tile, dtype, level, norm):
    r = synth_window(kind, 41, bands, H, W).astype(dtype)
    wins = calculate_tiles(H, W, tile)
    di, df = _device_path(r, wins, level, norm)
    plan = N.Plan(N.default_context(0), None, False, r.dtype, bands, (H * W, W, 1), wins, level, 4096, norm)
    try:
        cap, nbands = plan.capacity()
        assert nbands > 1
        pin = N.pinned_empty(r.shape, r.dtype)
        pin[...] = r
        out = N.pinned_empty(cap, np.uint8)
        total = plan.encode_host(pin, out)
        infos, _ = plan.result()
        assert bytes(out[:total]) == df and _table(infos) == _table(di)
        page = np.empty(cap, np.uint8)  # pageable raster and output
        assert plan.encode_host(r, page) == total and bytes(page[:total]) == df
        small = np.empty(total // 2, np.uint8)  # too small: FRA_E_SPACE, frames stay on the device
        with pytest.raises(N.OutputTooSmall) as e:
            plan.encode_host(pin, small)
        assert e.value.needed == total
        assert plan.download()[1] == df
    finally:
        plan.close()


def test_encode_host_strided_view_and_window_orders():
    r = synth_window(4, 8, 3, 2600, 2200)
    view = r[:, 300:2600, :]  # a row band of a larger raster: strides stay those of r
    wins = calculate_tiles(2300, 2200, 512)
    exp_i, exp_f = _device_path(np.ascontiguousarray(view), wins, 5, 16)
    gi, gf = N.encode_windows_buffer(view, wins, 5, 4096, 16)
    assert bytes(gf) == exp_f and _table(gi) == _table(exp_i)
    rev = wins[::-1]  # non-monotone row order -> one band covering every row
    ri, rf = N.encode_windows(view, rev, 5, 4096, 16)
    di, df = _device_path(np.ascontiguousarray(view), rev, 5, 16)
    assert rf == df and _table(ri) == _table(di)


def _gdal_like_tiff(path, a, compression, predictor):
    """Strip GeoTIFF written by an independent libtiff (Pillow) -- single band, as Pillow supports."""
    from PIL import Image

    kw = {"compression": compression}
    if predictor != 1:
        kw["tiffinfo"] = {317: predictor}
    Image.fromarray(a[0]).save(path, **kw)


@pytest.mark.parametrize("compression,predictor,dtype,level,tile", [
    ("tiff_lzw", 2, np.uint16, 5, 512),
    ("tiff_lzw", 1, np.uint16, 5, 384),
    ("tiff_adobe_deflate", 2, np.uint16, 5, 512),
    ("tiff_adobe_deflate", 3, np.float32, 8, 256),
])
def test_compressed_geotiff_to_streaming_container(tmp_path, compression, predictor, dtype, level, tile):
    pytest.importorskip("PIL")
    r = synth_window(4 if dtype == np.uint16 else 5, 3, 1, 1100, 1300).astype(dtype)
    p = tmp_path / "in.tif"
    _gdal_like_tiff(p, r, compression, predictor)
    out = tmp_path / "s.flac"
    create_streaming_flac(p, out, tile, level)
    tiles = calculate_tiles(1100, 1300, tile)
    ref = assemble_streaming(tiles, oracle_encode_tiles(r, tiles, level), r.shape, r.dtype,
                             Affine(1.0, 0.0, 0.0, 0.0, 1.0, 0.0), None, tile)
    assert out.read_bytes() == ref


@pytest.mark.parametrize("compression,tile", [("deflate", 256), ("lzw", 512)])
def test_native_tiled_geotiff_decode_overlapped_with_encode(tmp_path, compression, tile):
    """4-band tiled GeoTIFF from the native writer (predictor 2): create_streaming_flac decodes it on a
    producer thread while the host pipeline encodes the rows already published
    (fra_plan_encode_host_progress) -- the container equals the oracle's."""
    from flac_raster.tiff import write_geotiff

    r = synth_window(4, 9, 4, 1500, 1200).astype(np.uint16)
    p = tmp_path / "in.tif"
    write_geotiff(p, r, compression=compression, tile=256, predictor=2)
    out = tmp_path / "s.flac"
    create_streaming_flac(p, out, tile, 5)
    tiles = calculate_tiles(1500, 1200, tile)
    ref = assemble_streaming(tiles, oracle_encode_tiles(r, tiles, 5), r.shape, r.dtype,
                             Affine(1.0, 0.0, 0.0, 0.0, 1.0, 0.0), None, tile)
    assert out.read_bytes() == ref


def test_corrupt_geotiff_fails_cleanly_while_encoding(tmp_path):
    """A chunk that fails to decode mid-file: the producer publishes -1, the host pipeline stops waiting
    and reports the error (no hang, no partial container)."""
    from flac_raster.tiff import GeoTIFF, write_geotiff

    r = synth_window(4, 9, 1, 2048, 1024).astype(np.uint16)
    p = tmp_path / "bad.tif"
    write_geotiff(p, r, compression="deflate", tile=256, predictor=2)
    g = GeoTIFF(p)
    off = int(g._offs[len(g._offs) - 3])
    g.close()
    raw = bytearray(p.read_bytes())
    raw[off:off + 64] = b"\xff" * 64  # not a deflate stream any more
    p.write_bytes(bytes(raw))
    with pytest.raises(Exception):
        create_streaming_flac(p, tmp_path / "x.flac", 512, 5)
    assert not (tmp_path / "x.flac").exists()


def _band_rows(r, wins, level, norm):
    plan = N.Plan(N.default_context(0), None, False, r.dtype, r.shape[0], (r.shape[1] * r.shape[2], r.shape[2], 1),
                  wins, level, 4096, norm)
    try:
        return plan.host_band_rows()
    finally:
        plan.close()


@pytest.mark.parametrize("kind,bands,H,W,tile,dtype,level,norm,step,extra", [
    (4, 4, 4608, 2048, 512, np.uint16, 5, 16, 512, 0),     # minimum ring (one band + one step): wraps every band
    (4, 2, 4608, 1900, 256, np.uint16, 5, 16, 96, 37),     # steps that straddle band edges, odd ring size
    (5, 3, 4096, 2048, 512, np.float32, 8, 24, 0, 0),      # 32-bps, default ring (two bands + a step)
])
def test_ring_encode_equals_device_path(kind, bands, H, W, tile, dtype, level, norm, step, extra):
    """fra_plan_encode_ring: the raster only ever exists as a ring of a few row bands (the producer writes
    image row r at ring row r % R once the encoder's H2D copies released it); frames and stream table equal
    the device-resident path's, so no ring row was overwritten before its copy completed."""
    from flac_raster.tiles import encode_tiles_ring, streams_from  # noqa: F401

    r = synth_window(kind, 77, bands, H, W).astype(dtype)
    wins = calculate_tiles(H, W, tile)
    di, df = _device_path(r, wins, level, norm)
    band = _band_rows(r, wins, level, norm)
    st = step or band
    R = band + st + extra if extra or step else 0
    calls = []

    def fill(dst, r0, r1):
        calls.append((r0, r1))
        dst[...] = r[:, r0:r1, :]

    infos, frames, ring_rows = N.encode_windows_ring(r.shape, r.dtype, wins, fill, level, 4096, norm, step=st,
                                                     ring_rows=R)
    assert ring_rows < H  # the raster was never whole in host memory
    assert bytes(frames) == df and _table(infos) == _table(di)
    assert calls[0][0] == 0 and calls[-1][1] == H and all(a[1] == b[0] for a, b in zip(calls, calls[1:]))


def test_ring_geotiff_larger_than_ring_equals_device_path(tmp_path):
    """The user path: create_streaming_flac on a GeoTIFF much taller than the ring (single device: the ring
    path) -- container bytes equal the device-resident path's container."""
    from flac_raster.streaming import encode_geotiff_ring
    from flac_raster.tiff import GeoTIFF, write_geotiff

    H, W, tile = 6144, 1536, 512  # >= 2,048 frames: one tile row per host band
    r = synth_window(4, 21, 3, H, W).astype(np.uint16)
    p = tmp_path / "big.tif"
    write_geotiff(p, r, compression="deflate", tile=256, predictor=2)
    tiles = calculate_tiles(H, W, tile)
    g = GeoTIFF(p)
    try:
        streams, R = encode_geotiff_ring(g, tiles, 5, 0, tile, ring_rows=_band_rows(r, tiles, 5, 16) + 512)
    finally:
        g.close()
    assert R < H / 3
    di, df = _device_path(r, tiles, 5, 16)
    assert b"".join(bytes(s.body) for s in streams) == df
    out = tmp_path / "s.flac"
    create_streaming_flac(p, out, tile, 5)
    ref = assemble_streaming(tiles, streams, r.shape, r.dtype, Affine(1.0, 0.0, 0.0, 0.0, 1.0, 0.0), None, tile)
    assert out.read_bytes() == ref


def test_ring_producer_failure_is_reported():
    r = synth_window(4, 5, 1, 3000, 1024).astype(np.uint16)
    wins = calculate_tiles(3000, 1024, 512)

    def fill(dst, r0, r1):
        if r0 >= 1500:
            raise OSError("decode failed")
        dst[...] = r[:, r0:r1, :]

    with pytest.raises(OSError):
        N.encode_windows_ring(r.shape, r.dtype, wins, fill, 5, 4096, 16, step=256)


def test_pinned_pool_reuse():
    a = N.pinned_empty(1 << 20, np.uint8)
    p = a.ctypes.data
    del a
    b = N.pinned_empty((1 << 20) - 100, np.uint8)
    assert b.ctypes.data == p and N.is_pinned(b)
    N.release_pinned_pool()


def test_cross_execute_pipelining_buffers():
    """A plan large enough for cross-execute pipelining (>= 4096 frames: k_assemble of execute k on its own
    stream while execute k+1 analyses into the other buffer set) gives the same bytes on every execute,
    after a drain into the timing mode and into the host pipeline, and after set_raster."""
    H, W = 4096, 4096
    r = synth_window(3, 77, 1, H, W)
    wins = calculate_tiles(H, W, 512)
    ctx = N.default_context(0)
    dev = ctx.alloc(r.nbytes)
    try:
        ctx.h2d(dev, r)
        plan = N.Plan(ctx, dev, True, r.dtype, 1, (H * W, W, 1), wins, 5, 4096, 16)
        try:
            outs = []
            for _ in range(3):  # buffer sets 0, 1, 0
                plan.execute()
                plan.sync()
                outs.append(plan.download())
            assert all(o[1] == outs[0][1] for o in outs)
            assert all(_table(o[0]) == _table(outs[0][0]) for o in outs)
            plan.execute()
            plan.execute()  # two in flight, then the timing mode drains them
            plan.enable_timing(True)
            plan.execute()
            plan.sync()
            assert plan.download()[1] == outs[0][1]
            plan.enable_timing(False)
            plan.execute()
            cap, _ = plan.capacity()
            out = np.empty(cap, np.uint8)
            total = plan.encode_host(r, out)  # drains the pipelined execute, then the host bands
            assert bytes(out[:total]) == outs[0][1]
            assert plan.frame_offsets(sum(i.nframes for i in outs[0][0]))[-1] == total
            # pipelined -> serial (timing) -> pipelined with no host sync anywhere (the first
            # pipelined norm stage after serial work must wait for the plan's stream)
            plan.execute()
            plan.enable_timing(True)
            plan.execute()
            plan.enable_timing(False)
            plan.execute()
            plan.execute()
            plan.sync()
            assert plan.download()[1] == outs[0][1]
        finally:
            plan.close()
    finally:
        ctx.free(dev)


@pytest.mark.parametrize("kind,bands,H,W,tile,dtype,level,norm", [
    (4, 4, 4500, 4500, 1024, np.uint16, 5, 16),    # 4 channels, ragged edge tiles (k_analyze<16-bit, lag 8>)
    (4, 2, 4500, 4096, 1000, np.uint16, 5, 16),    # 2 channels: mid-side slot map, odd tile width
    (3, 1, 4096, 4096, 512, np.int16, 8, 16),      # lag-12 16-bit instance
    (5, 2, 4096, 4096, 512, np.float32, 8, 24),    # 32-bps
])
def test_pipelined_assembly_equals_serial(kind, bands, H, W, tile, dtype, level, norm):
    """Pipelined executes run the frame-size chain and the assembly of execute k on the pack stream beside
    execute k+1's analysis (k_frame_scan + k_assemble4).  The output of
    execute 2, written into an output buffer poisoned after execute 1 and read after a device-wide barrier,
    must be byte-identical to the serial (timing-mode) execute's; so must the plan's own download; and
    sampled tiles must equal the oracle's frames."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")  # the HIP runtime the product library runs on (one per process)

    def device_barrier():  # hipDeviceSynchronize: every stream of the device, independent of the plan's sync
        assert hip.hipDeviceSynchronize() == 0

    r = synth_window(kind, 91, bands, H, W).astype(dtype, copy=False)
    wins = calculate_tiles(H, W, tile)
    ctx = N.default_context(0)
    dev = ctx.alloc(r.nbytes)
    try:
        ctx.h2d(dev, r)
        plan = N.Plan(ctx, dev, True, r.dtype, bands, (H * W, W, 1), wins, level, 4096, norm)
        try:
            assert plan.flags() & 2, "plan too small for the pipelined execute (FRA_PLAN_PIPELINED)"
            out_ptr, out_cap = plan.device_output()
            plan.enable_timing(True)
            plan.execute()
            plan.sync()
            infos_s, serial = plan.download()
            plan.enable_timing(False)
            plan.execute()  # execute 1
            device_barrier()
            ctx.h2d(out_ptr, np.full(min(out_cap, len(serial) + 256), 0xA5, np.uint8))
            plan.execute()  # execute 2, beside execute 1's assembly; its own assembly rewrites the buffer
            device_barrier()
            fused = np.empty(len(serial), np.uint8)
            ctx.d2h(fused, out_ptr)
            plan.sync()
            infos_p, piped = plan.download()
        finally:
            plan.close()
    finally:
        ctx.free(dev)
    assert fused.tobytes() == serial
    assert _table(infos_p) == _table(infos_s)
    assert piped == serial
    exp = oracle_encode_tiles(r, [wins[0], wins[-1]], level=level)
    for k, i in enumerate((0, len(wins) - 1)):
        s = infos_p[i]
        assert piped[s.offset:s.offset + s.frame_bytes] == bytes(exp[k].body)


def test_host_raster_swap_between_pipelined_executes():
    """A host raster set between pipelined executes (no sync) is copied into the plan's device buffer on the
    plan's stream; with each buffer set's analysis on its own stream, the copy must wait for the analyses
    still reading the old rows.  Outputs after the swap equal a fresh plan's on the new raster, and the
    executes before it a fresh plan's on the old one."""
    H, W = 4096, 4096
    a = synth_window(4, 5, 1, H, W).astype(np.uint16)
    b = synth_window(4, 6, 1, H, W).astype(np.uint16)
    wins = calculate_tiles(H, W, 1024)
    ctx = N.default_context(0)

    def fresh(r):
        p = N.Plan(ctx, r.ctypes.data, False, r.dtype, 1, (H * W, W, 1), wins, 5, 4096, 16, keepalive=r)
        try:
            p.execute()
            return p.download()[1]
        finally:
            p.close()

    exp_a, exp_b = fresh(a), fresh(b)
    assert exp_a != exp_b
    plan = N.Plan(ctx, a.ctypes.data, False, a.dtype, 1, (H * W, W, 1), wins, 5, 4096, 16, keepalive=a)
    try:
        assert plan.flags() & 2
        plan.execute()
        plan.execute()
        plan.sync()
        assert plan.download()[1] == exp_a
        plan.execute()
        plan.execute()  # two analyses in flight (one per buffer set) when the copy of b is queued
        plan.set_raster(b.ctypes.data, False, keepalive=b)
        plan.execute()
        plan.execute()
        plan.sync()
        assert plan.download()[1] == exp_b
    finally:
        plan.close()


@pytest.mark.parametrize("items", ["1", "4", "16"])
def test_frame_scan_forms_equal(monkeypatch, items):
    """k_frame_scan's three forms (1, 4 or 16 frames per thread: the decoupled look-back over 1,024 / 256 / 64
    workgroups of this plan) give the same offsets and bytes; FRA_SCAN_ITEMS is read when the plan is made."""
    H, W = 9000, 8192  # 18,000 frames of one band: 71 / 18 / 5 workgroups (two look-back windows at 1)
    r = synth_window(3, 17, 1, H, W)
    wins = calculate_tiles(H, W, 512)
    _, ref = N.encode_windows(r, wins, level=5, norm=16)
    monkeypatch.setenv("FRA_SCAN_ITEMS", items)
    infos, got = N.encode_windows(r, wins, level=5, norm=16)
    assert got == ref


@pytest.mark.parametrize("kind,dtype,level,norm", [(4, np.uint16, 5, 16), (5, np.float32, 8, 24)])
def test_ranged_plan_frames_equal_stream_slices(kind, dtype, level, norm):
    """fra_plan_create_ranged (the (tile, frame range) work items of the multi-GPU split): each window's
    frames [f0, f0 + n) equal that slice of the whole-stream encode -- same normalisation (whole window),
    same frame numbers -- including ranges that start mid-stream and end at the partial last frame."""
    r = synth_window(kind, 13, 3, 1500, 1300).astype(dtype)
    wins = calculate_tiles(1500, 1300, 512)
    ctx = N.default_context(0)
    full = N.Plan(ctx, None, False, r.dtype, 3, (1500 * 1300, 1300, 1), wins, level, 4096, norm)
    try:
        cap, _ = full.capacity()
        out = np.empty(cap, np.uint8)
        full.encode_host(r, out)
        fi, _ = full.result()
        offs = full.frame_offsets(sum(i.nframes for i in fi))
    finally:
        full.close()
    nfr = [i.nframes for i in fi]
    ranges = [((k * 7) % n, -1 if k % 3 == 0 else max(1, n // 3)) for k, n in enumerate(nfr)]
    ri, rf = N.encode_windows_buffer(r, wins, level, 4096, norm, frame_ranges=ranges)
    base = 0
    for k, ((f0, n), info) in enumerate(zip(ranges, ri)):
        n = nfr[k] - f0 if n < 0 else min(n, nfr[k] - f0)
        g0 = base + f0
        exp = bytes(out[offs[g0]:offs[g0 + n]])
        assert bytes(rf[info.offset:info.offset + info.frame_bytes]) == exp, f"window {k} range {(f0, n)}"
        assert info.nframes == n and info.sample_rate == fi[k].sample_rate
        assert (info.data_min, info.data_max) == (fi[k].data_min, fi[k].data_max)
        base += nfr[k]


def test_ranged_plan_rejects_ranges_outside_the_stream():
    """a (tile, frame range) work item outside its window's stream -- a first frame past the stream's
    frame count or a count below -1 -- is rejected at plan creation instead of silently dropping or duplicating
    frames of the multi-GPU split (a count past the end is clipped to it)."""
    ctx = N.default_context(0)
    wins = calculate_tiles(512, 512, 256)  # 16 frames per window
    ok = [(0, -1), (15, 1), (16, 0), (10, 7)]
    plan = N.Plan(ctx, None, False, np.uint16, 1, (512 * 512, 512, 1), wins, 5, 4096, 16, frame_ranges=ok)
    plan.close()
    for bad in [(17, -1), (0, -5), (20, 1), (-1, 2)]:
        with pytest.raises(N.NativeError, match="frame range|first frame"):
            N.Plan(ctx, None, False, np.uint16, 1, (512 * 512, 512, 1), wins, 5, 4096, 16,
                   frame_ranges=[bad] + ok[1:])


def test_plan_rejects_bad_strides():
    """Strides are validated at plan creation (negative strides, col_stride < 1, row_stride >= 2^32 elements:
    the per-frame analysis descriptors hold the row stride in 32 bits)."""
    ctx = N.default_context(0)
    wins = calculate_tiles(16, 16, 16)
    for strides in [(256, 2 ** 32, 1), (256, -16, 1), (256, 16, 0), (-256, 16, 1)]:
        with pytest.raises(N.NativeError, match="strides"):
            N.Plan(ctx, None, False, np.uint16, 1, strides, wins, 5, 4096, 16)


@pytest.mark.parametrize("dtype,level,norm,wave", [
    (np.uint16, 5, 16, True), (np.int16, 6, 16, True), (np.uint8, 3, 16, True),   # k_analyze_w: levels 3-6
    (np.uint16, 8, 16, False), (np.uint16, 2, 16, False),                         # lag 12 / no LPC: k_analyze
    (np.float32, 8, 24, False), (np.int32, 5, 24, False),                         # 32-bps: k_analyze
])
def test_plan_reports_analysis_path(dtype, level, norm, wave):
    """fra_plan_flags reports FRA_PLAN_WAVE exactly when full frames take the per-wave analysis kernel (bench.py
    names the dominant kernel from it)."""
    wins = calculate_tiles(512, 512, 256)
    plan = N.Plan(N.default_context(0), None, False, np.dtype(dtype), 1, (512 * 512, 512, 1), wins, level, 4096, norm)
    try:
        assert bool(plan.flags() & 4) == wave
    finally:
        plan.close()


@pytest.mark.parametrize("threads", [1, 7])
def test_encode_host_pageable_output_worker_counts(threads, monkeypatch):
    """A pageable output is filled by the context's D2H workers through page-locked staging (FRA_D2H_THREADS,
    read when a context first needs them): one worker and an odd count give the device path's bytes, into a
    fresh (lazily committed) buffer and into one already written."""
    monkeypatch.setenv("FRA_D2H_THREADS", str(threads))
    r = synth_window(4, 5, 4, 3600, 3600)
    wins = calculate_tiles(3600, 3600, 1024)
    di, df = _device_path(r, wins, 5, 16)
    ctx = N.Context(0)
    plan = N.Plan(ctx, None, False, r.dtype, 4, (3600 * 3600, 3600, 1), wins, 5, 4096, 16)
    try:
        cap, nbands = plan.capacity()
        assert nbands > 1
        for _ in range(2):
            out = np.empty(cap, np.uint8)
            total = plan.encode_host(r, out)
            assert bytes(out[:total]) == df
        assert plan.encode_host(r, out) == total and bytes(out[:total]) == df  # pages already committed
    finally:
        plan.close()
        ctx.close()


@pytest.mark.parametrize("kind,bands,n,tile,want17", [(3, 1, 2048, 512, True), (0, 4, 2100, 1024, False)])
def test_keep17_instance_follows_the_data(monkeypatch, kind, bands, n, tile, want17):
    """A pipelined wave-path plan starts on the 17-bit k_analyze_w instance and then takes the one an earlier
    execute's count of waves that needed bit 16 calls for (FRA_PLAN_KEEP17): the C3-like int16 DEM (a third of its
    waves) keeps 17 bits, a smooth 4-band ramp with small noise (LPC residuals far below 2^16) drops to 16.  Every
    execute's bytes are the same whichever instance ran, and equal the oracle's on sampled tiles."""
    monkeypatch.delenv("FRA_KEEP17", raising=False)
    if kind:
        r = synth_window(kind, 7, bands, n, n)
    else:
        yy, xx = np.mgrid[0:n, 0:n]
        noise = np.random.default_rng(3).integers(0, 4, size=(bands, n, n))
        r = (3 * yy + 2 * xx + 100 * np.arange(bands)[:, None, None] + noise).astype(np.uint16)
    wins = calculate_tiles(n, n, tile)
    ctx = N.default_context(0)
    dev = ctx.alloc(r.nbytes)
    try:
        ctx.h2d(dev, r)
        plan = N.Plan(ctx, dev, True, r.dtype, bands, (n * n, n, 1), wins, 5, 4096, 16)
        try:
            assert plan.flags() & 2 and plan.flags() & 4, "needs a pipelined wave-path plan"
            assert plan.flags() & 8  # no count yet: 17 bits
            outs = []
            for _ in range(3):
                plan.execute()
                plan.sync()
                outs.append(plan.download()[1])
            assert bool(plan.flags() & 8) == want17
            plan.execute()  # on the chosen instance
            plan.sync()
            outs.append(plan.download()[1])
        finally:
            plan.close()
    finally:
        ctx.free(dev)
    assert all(o == outs[0] for o in outs[1:])
    exp = oracle_encode_tiles(r, [wins[0], wins[-1]], level=5)
    assert bytes(exp[0].body) in outs[-1] and bytes(exp[1].body) in outs[-1]


def test_keep17_instance_on_a_subset_of_the_c4_bench_scene(monkeypatch):
    """the bench's C4 scene settles on the 16-bit k_analyze_w instance; a plan over a subset of
    that same scene's 1024^2 tiles (tile rows 4-5, 22 tiles incl. two 740-wide edge tiles, generated on the device
    exactly as bench.py does) must settle on it too, so the instance the bench line reports is not a property of
    re-encoding the whole scene only.  Bytes are the same on either instance."""
    monkeypatch.delenv("FRA_KEEP17", raising=False)
    H = W = 10980
    ctx = N.default_context(0)
    dev = ctx.alloc(4 * H * W * 2)
    try:
        ctx.synth(4, 20260227, 4, H, W, dev)
        wins = [w for w in calculate_tiles(H, W, 1024) if w[0] in (4096, 5120)]
        assert len(wins) == 22
        plan = N.Plan(ctx, dev, True, np.uint16, 4, (H * W, W, 1), wins, 5, 4096, 16)
        try:
            assert plan.flags() & 2 and plan.flags() & 4 and plan.flags() & 8
            outs = []
            for _ in range(3):
                plan.execute()
                plan.sync()
                outs.append(plan.download()[1])
            assert not plan.flags() & 8, "the C4 subset stayed on the 17-bit instance"
            plan.execute()
            plan.sync()
            outs.append(plan.download()[1])
        finally:
            plan.close()
    finally:
        ctx.free(dev)
    assert all(o == outs[0] for o in outs[1:])
