"""Synthetic benchmark rasters, numpy mirror of ``csrc/fra_synth.hip``.

Integer-exact: any window computed here equals the same window generated on the GPU by
``fra_synth_raster`` bit for bit (C5 float32 = one double division then a cast, same on both).

Deviation from Appendix C, stated: the C3 DEM uses integer value noise (scales 1024/256 px plus a
0..50 uniform term, range 550..1500) instead of the ``sin``/``cos`` formula of
``examples/create_test_data.py:18-28``, because libm and the GPU's trig functions round
differently and the CPU baseline sample must be the same data as the GPU run.
"""

from __future__ import annotations

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
KIND_DEM, KIND_S2, KIND_REFL = 3, 4, 5
S2_MEANS = (1200, 1100, 1000, 2500)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _lattice(seed, b, octv, ix, iy):
    key = (np.uint64(seed) ^ (np.uint64(b) << np.uint64(56)) ^ (np.uint64(octv) << np.uint64(48))
           ^ (iy.astype(np.uint64) << np.uint64(24)) ^ ix.astype(np.uint64))
    return splitmix64(key) & np.uint64(0xFFFF)


def _vnoise(seed, b, octv, ls, row, col):
    s = np.uint64(1 << ls)
    ix, iy = col >> np.uint64(ls), row >> np.uint64(ls)
    fx, fy = col & (s - np.uint64(1)), row & (s - np.uint64(1))
    one = np.uint64(1)
    v00 = _lattice(seed, b, octv, ix, iy)
    v10 = _lattice(seed, b, octv, ix + one, iy)
    v01 = _lattice(seed, b, octv, ix, iy + one)
    v11 = _lattice(seed, b, octv, ix + one, iy + one)
    top = v00 * (s - fx) + v10 * fx
    bot = v01 * (s - fx) + v11 * fx
    return (top * (s - fy) + bot * fy) >> np.uint64(2 * ls)


def _ih4(seed, b, row, col):
    h = splitmix64(np.uint64(seed) ^ np.uint64(0xA5A5A5A5A5A5A5A5) ^ (np.uint64(b) << np.uint64(56))
                   ^ (row << np.uint64(28)) ^ col)
    m = np.uint64(0xFF)
    s = (h & m) + ((h >> np.uint64(8)) & m) + ((h >> np.uint64(16)) & m) + ((h >> np.uint64(24)) & m)
    return s.astype(np.int64) - 510


def _tdiv(a, b):
    """C integer division (truncation toward zero)."""
    q = np.abs(a) // abs(b)
    return np.where((a < 0) != (b < 0), -q, q)


def synth_window(kind: int, seed: int, bands: int, H: int, W: int, row_off=0, col_off=0, height=None,
                 width=None) -> np.ndarray:
    """Window (bands, height, width) of the full (bands, H, W) synthetic raster."""
    height = H - row_off if height is None else height
    width = W - col_off if width is None else width
    rows = np.arange(row_off, row_off + height, dtype=np.uint64)[:, None]
    cols = np.arange(col_off, col_off + width, dtype=np.uint64)[None, :]
    row = np.broadcast_to(rows, (height, width))
    col = np.broadcast_to(cols, (height, width))
    out = []
    for b in range(bands):
        if kind == KIND_DEM:
            n1 = _vnoise(seed, b, 0, 10, row, col).astype(np.int64)
            n2 = _vnoise(seed, b, 1, 8, row, col).astype(np.int64)
            h = splitmix64(np.uint64(seed) ^ np.uint64(0x5151515151515151) ^ (row << np.uint64(28)) ^ col)
            v = 550 + n1 * 600 // 65535 + n2 * 300 // 65535 + (h % np.uint64(51)).astype(np.int64)
            out.append(v.astype(np.int16))
        elif kind == KIND_S2:
            nz = (4 * _vnoise(seed, b, 0, 9, row, col) + 2 * _vnoise(seed, b, 1, 7, row, col)
                  + _vnoise(seed, b, 2, 5, row, col)).astype(np.int64)
            dn = nz * 1200 // 458745 - 600
            g = _tdiv(_ih4(seed, b, row, col) * 15, 148)
            v = np.clip(S2_MEANS[b & 3] + dn + g, 1, 11672)
            tri = ((H + W) * 158) // 1000
            v = np.where((row.astype(np.int64) + col.astype(np.int64)) < tri, 0, v)
            out.append(v.astype(np.uint16))
        elif kind == KIND_REFL:
            nz = (2 * _vnoise(seed, b, 0, 9, row, col).astype(np.int64)
                  + _vnoise(seed, b, 1, 6, row, col).astype(np.int64) - 3 * 32767)
            g = _tdiv(_ih4(seed, b, row, col) * 200, 148)
            v = np.clip(15000 + _tdiv(nz * 10000, 3 * 65535) + g, 0, 120000)
            out.append((v.astype(np.float64) / 100000.0).astype(np.float32))
        else:
            raise ValueError(f"unknown synthetic kind {kind}")
    return np.stack(out)
