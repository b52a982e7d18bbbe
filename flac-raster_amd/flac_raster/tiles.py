"""Tile geometry and the batched GPU tile encoder shared by the streaming / spatial / standard paths.

The reference encodes its units one at a time (``cli.py:553-622``: temp GeoTIFF per tile,
``converter.tiff_to_flac``, mutagen; ``spatial_encoder.py:196-245``: ``_encode_tile_to_flac`` per
tile).  Here every unit of a raster is one window of ONE plan (``fra_plan_*``): per-window
nanmin/nanmax, normalisation, analysis, bit packing and CRCs run as a handful of kernel launches
over all tiles at once.  With several devices, the tiles are split into contiguous runs of
near-equal pixel count (so each device receives only the rows its tiles cover) and the devices
run concurrently from host threads (ctypes releases the GIL); there is no exchange between
devices.  Output is identical for any device count.
"""

from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native

BLOCKSIZE = 4096  # converter.py:143, spatial_encoder.py:295


def calculate_tiles(height: int, width: int, tile_size: int) -> List[Tuple[int, int, int, int]]:
    """Row-major ``(row_off, col_off, h, w)`` with clipped edge tiles (``spatial_encoder.py:110-121``,
    ``cli.py:553-556``)."""
    if tile_size <= 0:
        raise ValueError("tile_size must be positive")
    return [(r, c, min(tile_size, height - r), min(tile_size, width - c))
            for r in range(0, height, tile_size) for c in range(0, width, tile_size)]


def split_contiguous(weights: Sequence[int], parts: int) -> List[Tuple[int, int]]:
    """Split ``range(len(weights))`` into ``parts`` contiguous runs of near-equal total weight."""
    n = len(weights)
    parts = max(1, min(parts, n)) if n else 1
    total = float(sum(weights))
    out, start, acc = [], 0, 0.0
    for p in range(parts - 1):
        target = total * (p + 1) / parts
        end = start
        while end < n - (parts - 1 - p) and (acc + weights[end] <= target or end == start):
            acc += weights[end]
            end += 1
        out.append((start, end))
        start = end
    out.append((start, n))
    return out


def frames_of(tile: Tuple[int, int, int, int], blocksize: int = 4096) -> int:
    """FLAC frames of one tile's stream."""
    return -(-(tile[2] * tile[3]) // blocksize)


# What holding partial last frames (n < blocksize) costs a rank, in full frames: those subframes run as ONE separate,
# latency-bound k_analyze launch per execute beside the per-wave analysis of the full frames, whatever their number.
# Measured on the C4 8-way split (r06, profiles/r06_shards_partial_cost.txt): the one rank holding the scene's only
# partial frame (the 740^2 corner tile) stepped ~0.012 ms (~6 %, about 240 frames of analysis) slower than the others;
# after FRA-1 3.5b made the frames cheaper the same launch weighs ~500 frames (256 -> 512: slowest 8-way share 0.200 ->
# 0.190 ms, profiles/r06_shards_final.txt).
PARTIAL_FRAME_COST = 512


def frame_split(tiles: Sequence[Tuple[int, int, int, int]], parts: int,
                blocksize: int = 4096, stride: int = 1,
                partial_cost: int = PARTIAL_FRAME_COST) -> List[List[Tuple[int, int, int]]]:
    """Work items of equal cost for ``parts`` ranks ((tile, frame range) items): the frames of all
    tiles in tile order, cut into ``parts`` contiguous runs; part k gets a list of (tile index, first frame, frame
    count) -- whole tiles, plus at most a partial tile at each end.  The frames of one tile, concatenated over the
    parts in order, are that tile's stream.  A part's cost is its frame count, plus ``partial_cost`` if it holds a
    tile's partial last frame (0: equal frame counts); the cuts are refined over a few passes (the parts holding
    partial frames depend on the cuts) and the pass with the smallest largest cost is kept.

    ``stride`` > 1 visits the tiles as i = 0, s, 2s, ..., then 1, 1 + s, ... (tile index mod s first), so each
    part's run samples the whole scene instead of one band of it: content that varies across the scene (a
    no-data corner, water, cloud) spreads over the parts, while the costs stay equal."""
    counts = [frames_of(t, blocksize) for t in tiles]
    order = sorted(range(len(tiles)), key=lambda j: (j % max(1, stride), j))
    total = sum(counts)
    # the global frame index of every partial last frame, in visiting order
    partial_at, pos = [], 0
    for i in order:
        pos += counts[i]
        if (tiles[i][2] * tiles[i][3]) % blocksize:
            partial_at.append(pos - 1)
    # (bounded by a quarter part's frames: no part can be left empty)
    pc = max(0, min(partial_cost, total // (4 * max(1, parts))))

    def cut(holds):  # cuts giving part k a frame count of (total + pc |P|) / parts - pc [k in P]
        t = total + pc * sum(holds)
        c, acc = [0], 0
        for k in range(parts):
            acc += (t * (k + 1) // parts - t * k // parts) - pc * holds[k]
            c.append(min(total, max(c[-1], acc)))
        c[-1] = total
        return c

    def holders(c):
        return [int(any(c[k] <= f < c[k + 1] for f in partial_at)) for k in range(parts)]

    def worst(c):  # the largest part cost of cuts c
        h = holders(c)
        return max(c[k + 1] - c[k] + pc * h[k] for k in range(parts))

    cuts = [total * k // parts for k in range(parts + 1)]
    if pc and partial_at:
        cands = [cuts]
        for _ in range(4):  # a cut next to a partial frame can flip its holder: keep the best of the passes
            cands.append(cut(holders(cands[-1])))
            if cands[-1] == cands[-2]:
                break
        cuts = min(cands, key=worst)
    out: List[List[Tuple[int, int, int]]] = [[] for _ in range(parts)]
    base = 0
    for i in order:
        n = counts[i]
        for k in range(parts):
            a, b = max(base, cuts[k]), min(base + n, cuts[k + 1])
            if b > a:
                out[k].append((i, a - base, b - a))
        base += n
    return out


def lpt_assign(weights: Sequence[int], parts: int) -> List[List[int]]:
    """Longest-processing-time assignment (used when data already lives on every device)."""
    order = sorted(range(len(weights)), key=lambda i: (-weights[i], i))
    loads = [0] * parts
    groups: List[List[int]] = [[] for _ in range(parts)]
    for i in order:
        g = min(range(parts), key=lambda k: (loads[k], k))
        groups[g].append(i)
        loads[g] += weights[i]
    return [sorted(g) for g in groups]


@dataclass
class TileStream:
    """One encoded unit: a complete FLAC stream (86-byte header + frames) + its normalisation.

    ``header`` is the 86-byte libFLAC-layout header, ``body`` the frames -- a zero-copy view into the
    page-locked output of the pipelined encode (``_native.encode_windows_buffer``); ``data`` joins them."""

    header: bytes
    body: object  # bytes-like (memoryview / bytes)
    data_min: float
    data_max: float
    sample_rate: int
    bps: int        # FLAC bits per sample (16, or 32 for int32 audio: SURVEY.md F3)
    channels: int
    nframes: int

    @property
    def data(self) -> bytes:
        return self.header + bytes(self.body)

    def __len__(self) -> int:
        return len(self.header) + len(self.body)

    def __getstate__(self):  # pickling (multi-process gather) materialises the view
        st = dict(self.__dict__)
        st["body"] = bytes(self.body)
        return st


def norm_bits(dtype) -> int:
    """calculate_audio_params' bit depth: 16 for <=16-bit integers, else 24 (int32 audio)."""
    return 16 if np.dtype(dtype) in (np.uint8, np.int8, np.uint16, np.int16) else 24


def _encode_group(raster: np.ndarray, tiles: Sequence[Tuple[int, int, int, int]], level: int, device: int,
                  norm: int, out: list, errors: list, slot: int, rows_ready=None, frame_ranges=None):
    try:
        r0 = min(t[0] for t in tiles)
        r1 = max(t[0] + t[2] for t in tiles)
        sub = raster[:, r0:r1, :]  # a view: the plan copies only these rows, band by band
        wins = [(t[0] - r0, t[1], t[2], t[3]) for t in tiles]
        if rows_ready is not None and r0 != 0:
            raise ValueError("rows_ready needs the group to start at raster row 0")
        infos, frames = _native.encode_windows_buffer(sub, wins, level=level, blocksize=BLOCKSIZE, norm=norm,
                                                      device=device, rows_ready=rows_ready,
                                                      frame_ranges=frame_ranges)
        out[slot] = streams_from(infos, frames)
    except BaseException as e:  # re-raised on the calling thread
        errors.append(e)


def streams_from(infos, frames) -> List[TileStream]:
    """TileStreams over one plan's output: zero-copy views of ``frames`` at each window's offset."""
    res = []
    mv = memoryview(frames)
    for inf in infos:
        hdr = _native.stream_header(inf.channels, inf.bps, inf.sample_rate, BLOCKSIZE)
        res.append(TileStream(hdr, mv[inf.offset:inf.offset + inf.frame_bytes], float(inf.data_min),
                              float(inf.data_max), inf.sample_rate, inf.bps, inf.channels, inf.nframes))
    return res


def encode_tiles_ring(shape, dtype, tiles: Sequence[Tuple[int, int, int, int]], fill, level: int = 5,
                      device: int = 0, step: int = 0, ring_rows: int = 0) -> Tuple[List[TileStream], int]:
    """:func:`encode_tiles` for a raster that is produced row band by row band and never held whole
    (``_native.encode_windows_ring``): ``fill(dst, r0, r1)`` writes image rows ``[r0, r1)`` of every band
    into ``dst``.  The reference reads each tile's window the same way (``cli.py:553-559``).  Returns the
    streams and the ring's height in rows."""
    if not tiles:
        return [], 0
    infos, frames, R = _native.encode_windows_ring(shape, dtype, tiles, fill, level=level, blocksize=BLOCKSIZE,
                                                   norm=norm_bits(dtype), device=device, step=step,
                                                   ring_rows=ring_rows)
    return streams_from(infos, frames), R


def encode_tiles(raster: np.ndarray, tiles: Sequence[Tuple[int, int, int, int]], level: int = 5,
                 devices: Optional[Sequence[int]] = None, rows_ready=None,
                 producer: Optional[threading.Thread] = None, frame_ranges=None) -> List[TileStream]:
    """Encode every tile of a band-planar ``(B, H, W)`` raster as its own FLAC stream on the GPU(s).

    Each stream equals what ``normalize_to_audio`` + ``pyflac.StreamEncoder(blocksize=4096)``
    produce for ``raster[:, r:r+h, c:c+w]`` interleaved pixel-major (``cli.py:557-597``).
    ``rows_ready`` / ``producer``: the raster is still being decoded by ``producer``, which publishes the
    rows done in ``rows_ready[0]``; one device encodes as the rows land, several wait for the producer.
    ``frame_ranges``: (first frame, count) per tile -- only those frames of each stream (one device; the
    multi-GPU work items of ``frame_split``); the TileStream's body then holds just those frames.
    """
    a = np.asarray(raster)
    if a.ndim == 2:
        a = a[None]
    if not a.dtype.isnative:
        a = a.astype(a.dtype.newbyteorder("="))
    if a.dtype not in _native.DTYPE_CODES:
        raise TypeError(f"unsupported raster dtype {a.dtype}")
    if not tiles:
        return []
    devs = list(devices) if devices else [0]
    norm = norm_bits(a.dtype)
    runs = split_contiguous([t[2] * t[3] for t in tiles], len(devs))
    out: list = [None] * len(runs)
    errors: list = []
    if rows_ready is not None and (len(runs) > 1 or min(t[0] for t in tiles) != 0):
        if producer is not None:
            producer.join()
        if rows_ready[0] < 0:
            raise RuntimeError("raster decode failed")
        rows_ready = None
    if frame_ranges is not None:
        if len(devs) != 1:
            raise ValueError("frame_ranges: one device per call (one rank per GPU)")
        _encode_group(a, tiles, level, devs[0], norm, out, errors, 0, rows_ready, frame_ranges)
    elif len(runs) == 1:
        _encode_group(a, tiles, level, devs[0], norm, out, errors, 0, rows_ready)
    else:
        th = [threading.Thread(target=_encode_group, args=(a, tiles[s:e], level, devs[k], norm, out, errors, k))
              for k, (s, e) in enumerate(runs)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    if errors:
        raise errors[0]
    return [ts for grp in out for ts in grp]
