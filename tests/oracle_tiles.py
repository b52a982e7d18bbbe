"""Test-only stand-in for ``flac_raster.tiles.encode_tiles`` built on the CPU oracle.

Used by the CPU tests of the host layer (container assembly, tags, distributed gather): the
oracle is byte-identical to the GPU encoder (GPU parity tests), so host logic verified with this
stand-in is the host logic the GPU path runs.  Never imported by the package.
"""
import numpy as np

import oracle as O
from flac_raster.tiles import TileStream, norm_bits


def oracle_encode_tiles(raster, tiles, level=5, devices=None):
    a = np.asarray(raster)
    if a.ndim == 2:
        a = a[None]
    B = a.shape[0]
    bps_norm = norm_bits(a.dtype)
    out = []
    for (r, c, h, w) in tiles:
        inter = a[:, r:r + h, c:c + w].transpose(1, 2, 0).reshape(-1, B)
        audio, mn, mx = O.normalize(inter, bps_norm)
        sr = O.sample_rate_for_pixels(h * w)
        data = O.encode(audio, sr, level=level)
        out.append(TileStream(data[:86], data[86:], float(mn), float(mx), sr, 16 if bps_norm == 16 else 32, B,
                              (h * w + 4095) // 4096))
    return out
