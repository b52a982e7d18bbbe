"""GPU tests of the direct-write path (fra_dw.h): 16-bit k_analyze places every encoded
subframe at its final bit offset (decoupled look-back over the launch), merges the byte shared with its
predecessor, writes frame headers, pad bytes, the CRC-16 combined from per-subframe residues and the frame
offsets.  Its bytes must equal the slot path's (FRA_DW=0: subframe slots + k_frame_bytes + scan +
k_assemble) and the oracle's, for every subframe type the path can emit: CONSTANT (24-bit blobs, several
inside one dword), VERBATIM (noise), FIXED/LPC with wasted bits, 1..8 channels, ragged and 1-sample frames,
and across launch epochs (including the 16-bit epoch wrap)."""
import os

import numpy as np
import pytest

import oracle as O
from flac_raster import _native as N
from flac_raster.synth import synth_window
from flac_raster.tiles import calculate_tiles

pytestmark = pytest.mark.gpu


def _plan_bytes(r, wins, level, norm, dw, blocksize=4096, epoch0=None):
    env = {"FRA_DW": "1" if dw else "0"}
    if epoch0 is not None:
        env["FRA_DW_EPOCH0"] = str(epoch0)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        a = np.ascontiguousarray(r)
        B, H, W = a.shape
        plan = N.Plan(N.default_context(0), a.ctypes.data, False, a.dtype, B, (H * W, W, 1), wins, level,
                      blocksize, norm, 0, keepalive=a)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        assert bool(plan.flags() & 1) == dw
        outs = []
        for _ in range(3 if epoch0 is not None else 1):
            plan.execute()
            plan.sync()
            infos, frames = plan.download()
            outs.append((frames, [(i.offset, i.frame_bytes, i.nframes) for i in infos],
                         plan.frame_offsets(sum(i.nframes for i in infos))))
        assert all(o[0] == outs[0][0] and o[1] == outs[0][1] and list(o[2]) == list(outs[0][2]) for o in outs)
        return outs[0]
    finally:
        plan.close()


def _mixed_raster(bands, H, W, dtype, seed):
    """synthetic terrain + a constant block, a noise block (VERBATIM), a block with 3 wasted bits"""
    rng = np.random.default_rng(seed)
    r = synth_window(4, seed, bands, H, W).astype(np.int64)
    r[:, : H // 3, : W // 3] = 1234 if dtype == np.int16 else 40000
    lo, hi = (-32768, 32767) if dtype == np.int16 else (0, 65535)
    r[:, H // 3: 2 * H // 3, W // 3: 2 * W // 3] = rng.integers(lo, hi + 1, (bands, H - H // 3 - (H - 2 * H // 3),
                                                                          (2 * W // 3) - W // 3))
    blk = r[:, 2 * H // 3:, 2 * W // 3:]
    r[:, 2 * H // 3:, 2 * W // 3:] = (blk // 8) * 8
    if dtype == np.int16:
        r = np.clip(r - 20000, -32768, 32767)
    return r.astype(dtype)


@pytest.mark.parametrize("bands,dtype,norm,level,tile", [
    (4, np.uint16, 16, 5, 384),
    (4, np.uint16, 16, 0, 256),
    (3, np.uint16, 16, 8, 300),
    (1, np.int16, 0, 5, 333),
    (2, np.int16, 0, 3, 200),   # 2 channels at level 3: no mid-side, direct write
    (8, np.int16, 0, 6, 128),
    (5, np.uint16, 16, 7, 256),
])
def test_direct_write_equals_slot_path_and_oracle(bands, dtype, norm, level, tile):
    H, W = 900, 1000
    r = _mixed_raster(bands, H, W, dtype, 7 + bands)
    wins = calculate_tiles(H, W, tile)
    dwb = _plan_bytes(r, wins, level, norm, True)
    slot = _plan_bytes(r, wins, level, norm, False)
    assert dwb[1] == slot[1] and list(dwb[2]) == list(slot[2])
    assert dwb[0] == slot[0]
    # oracle on a few windows: the constant corner, the noise block, the wasted-bits corner, a ragged edge
    for wi in {0, len(wins) // 2, len(wins) - 1, len(wins) // 3}:
        r0, c0, h, w = wins[wi]
        tl = r[:, r0:r0 + h, c0:c0 + w]
        inter = tl.transpose(1, 2, 0).reshape(-1, bands)
        if norm:
            audio, _, _ = O.normalize(inter, 16)
        else:
            audio = inter.astype(np.int16)
        exp = O.encode(audio, O.sample_rate_for_pixels(h * w), level=level, blocksize=4096, with_header=False)
        off, fb, _ = dwb[1][wi]
        assert dwb[0][off:off + fb] == exp, f"window {wi}"


@pytest.mark.parametrize("blocksize", [16, 1152, 4095])
def test_direct_write_small_and_odd_blocks(blocksize):
    r = _mixed_raster(3, 160, 170, np.int16, 3)
    wins = calculate_tiles(160, 170, 64) + [(0, 0, 1, 1), (5, 7, 1, 3)]
    dwb = _plan_bytes(r, wins, 5, 0, True, blocksize=blocksize)
    slot = _plan_bytes(r, wins, 5, 0, False, blocksize=blocksize)
    assert dwb[0] == slot[0] and dwb[1] == slot[1]


def test_direct_write_epoch_wrap():
    """the look-back words carry a 16-bit launch epoch: executes across the wrap give identical bytes"""
    r = _mixed_raster(3, 700, 600, np.int16, 11)
    wins = calculate_tiles(700, 600, 256)
    a = _plan_bytes(r, wins, 5, 0, True, epoch0=0xFFFE)
    b = _plan_bytes(r, wins, 5, 0, False)
    assert a[0] == b[0]
