"""Full-size BASELINE configurations (C3, C4, C5) on the GPU, checked through size-independent
properties: the whole scene is encoded on the device exactly as `bench.py` does, then sampled tiles --
the first, one past 2 GiB and one past 4 GiB of output (C5: 22 GB of frames), the middle and the last --
are copied back and must (a) equal the CPU oracle's frames for the same tile byte for byte and
(b) decode (CRC-8/CRC-16 checked) to normalize_to_audio(tile).  Stream bookkeeping must tile the
output exactly (offsets + sizes == the scan's total).
"""
import numpy as np
import pytest

import bench
import oracle as O
from flac_raster import _native as N
from flac_raster.synth import synth_window

pytestmark = pytest.mark.gpu


def _pick(infos, total):
    """Indices of the sampled streams: first, middle, last, and the first stream starting past 2 GiB / 4 GiB."""
    n = len(infos)
    idx = {0, n // 2, n - 1}
    for edge in (1 << 31, 1 << 32):
        if total > edge:
            idx.add(next(i for i, s in enumerate(infos) if s.offset >= edge))
    return sorted(idx)


@pytest.mark.parametrize("name", ["c3", "c4", "c5"])
def test_full_scene(name):
    cfg = bench.CONFIGS[name]
    B, H, W = cfg["bands"], cfg["H"], cfg["W"]
    dt = np.dtype(cfg["dtype"])
    ctx = N.default_context(0)
    dev = ctx.alloc(B * H * W * dt.itemsize)
    plan = None
    try:
        ctx.synth(cfg["kind"], bench.SEED, B, H, W, dev)
        wins = bench.tiles(H, W, cfg["tile"])
        plan = N.Plan(ctx, dev, True, dt, B, (H * W, W, 1), wins, cfg["level"], 4096, cfg["norm"])
        plan.execute()
        infos, total = plan.result()
        out_ptr, cap = plan.device_output()
        assert total <= cap
        # the streams tile the output exactly
        offs = np.array([s.offset for s in infos], dtype=np.uint64)
        sizes = np.array([s.frame_bytes for s in infos], dtype=np.uint64)
        assert offs[0] == 0 and np.all(offs[1:] == offs[:-1] + sizes[:-1]) and int(offs[-1] + sizes[-1]) == total
        bps = 16 if cfg["norm"] == 16 else 24
        for i in _pick(infos, total):
            r0, c0, h, w = wins[i]
            s = infos[i]
            got = np.empty(s.frame_bytes, np.uint8)
            ctx.d2h(got, out_ptr + s.offset)
            tile = synth_window(cfg["kind"], bench.SEED, B, H, W, r0, c0, h, w)
            inter = tile.transpose(1, 2, 0).reshape(-1, B)
            audio, mn, mx = O.normalize(inter, bps)
            assert s.sample_rate == O.sample_rate_for_pixels(h * w)
            exp = O.encode(audio, s.sample_rate, level=cfg["level"], with_header=False)
            assert got.tobytes() == exp, f"{name} tile {i} at output offset {s.offset}"
            hdr = O.stream_header(B, 16 if bps == 16 else 32, s.sample_rate, 4096)
            dec, _, _, _ = O.decode(hdr + got.tobytes())
            assert np.array_equal(dec, audio.astype(np.int32))
    finally:
        if plan is not None:
            plan.close()
        ctx.free(dev)
