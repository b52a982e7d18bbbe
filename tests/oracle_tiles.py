"""Test-only stand-in for ``flac_raster.tiles.encode_tiles`` built on the CPU oracle.

Used by the CPU tests of the host layer (container assembly, tags, distributed gather): the
oracle is byte-identical to the GPU encoder (GPU parity tests), so host logic verified with this
stand-in is the host logic the GPU path runs.  Never imported by the package.
"""
import numpy as np

import oracle as O
from flac_raster.tiles import TileStream, norm_bits


def oracle_encode_tiles(raster, tiles, level=5, devices=None, frame_ranges=None):
    """``frame_ranges``: (first frame, count) per tile -- that slice of each stream's frames (the oracle
    encodes the whole stream and cuts it at its frame boundaries)."""
    a = np.asarray(raster)
    if a.ndim == 2:
        a = a[None]
    B = a.shape[0]
    bps_norm = norm_bits(a.dtype)
    out = []
    for k, (r, c, h, w) in enumerate(tiles):
        inter = a[:, r:r + h, c:c + w].transpose(1, 2, 0).reshape(-1, B)
        audio, mn, mx = O.normalize(inter, bps_norm)
        sr = O.sample_rate_for_pixels(h * w)
        data, fb, _ = O.encode(audio, sr, level=level, return_info=True)
        nfr = (h * w + 4095) // 4096
        body = data[86:]
        if frame_ranges is not None:
            f0, n = frame_ranges[k]
            n = nfr - f0 if n < 0 else min(n, nfr - f0)
            off = np.concatenate([[0], np.cumsum(fb)]).astype(np.int64)
            body, nfr = body[off[f0]:off[f0 + n]], n
        out.append(TileStream(data[:86], body, float(mn), float(mx), sr, 16 if bps_norm == 16 else 32, B, nfr))
    return out
