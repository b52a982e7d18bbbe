"""Multi-process (one process per GPU) driver for the tile encoder.

SURVEY.md 8(e): tiles are independent units, so ranks encode disjoint tile sets with no exchange on
the data path.  The only collective is the final hand-off of the encoded streams to the rank that
writes the container (``gather_streams``), plus barrier / max-time reductions for measurement.
Works with ``torch.distributed`` on ``nccl`` (= RCCL over xGMI on MI355X) or ``gloo`` (CPU tests);
launched by ``torch.distributed.run`` (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR in the env).

The compressed streams never travel through RCCL: each rank copies its frames D2H (the pipelined
``fra_plan_encode_host``) and writes them to a node-local spool file (``/dev/shm``); only a small
manifest (tile ids, lengths, min/max) goes through a gloo group, and the writer rank reads the spool.
Ranks on other hosts (no shared spool) send their bytes through the gloo group instead.
"""

from __future__ import annotations

import os
import socket
import tempfile
from pathlib import Path
from typing import Callable, List, Optional, Sequence, Tuple

from .tiles import TileStream, encode_tiles, frame_split, frames_of, lpt_assign


class Dist:
    """Rank/world plus the few collectives the encoder uses (no-ops when world == 1)."""

    def __init__(self, backend: Optional[str] = None):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        self.host_pg = None  # gloo group for host-side hand-offs (None: the default group is gloo)
        if self.world > 1:
            import torch
            import torch.distributed as td

            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl":
                torch.cuda.set_device(self.local_rank)
            if not td.is_initialized():
                td.init_process_group(backend=backend)
            self.pg = td
            if backend != "gloo":
                self.host_pg = td.new_group(backend="gloo")
        self.backend = backend

    def _dev(self):
        return "cuda" if self.backend == "nccl" else "cpu"

    def barrier(self):
        if self.pg is not None:
            self.pg.barrier()

    def _reduce(self, x: float, op) -> float:
        import torch

        t = torch.tensor([float(x)], dtype=torch.float64, device=self._dev())
        self.pg.all_reduce(t, op=op)
        return float(t.item())

    def allmax(self, x: float) -> float:
        return x if self.pg is None else self._reduce(x, self.pg.ReduceOp.MAX)

    def allsum(self, x: float) -> float:
        return x if self.pg is None else self._reduce(x, self.pg.ReduceOp.SUM)

    def gather_objects(self, obj, dst: int = 0) -> Optional[list]:
        if self.pg is None:
            return [obj]
        out = [None] * self.world if self.rank == dst else None
        self.pg.gather_object(obj, out, dst=dst, group=self.host_pg)
        return out

    def broadcast_object(self, obj, src: int = 0):
        if self.pg is None:
            return obj
        box = [obj]
        self.pg.broadcast_object_list(box, src=src, group=self.host_pg)
        return box[0]

    def gather_streams(self, items: List[Tuple[int, TileStream]], dst: int = 0):
        """Hand every rank's ``(tile id, TileStream)`` list to ``dst`` (others get ``None``) through a
        node-local spool file per rank; only the manifest goes through the (gloo) process group."""
        if self.pg is None:
            return [items]
        host = socket.gethostname()
        spool = None
        if self.rank == dst:
            shm = "/dev/shm" if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK) else None
            spool = tempfile.mkdtemp(prefix="fra_gather_", dir=shm)
        dst_host, spool = self.broadcast_object((host, spool), src=dst)
        meta = [(i, len(ts.header), len(ts.body), ts.data_min, ts.data_max, ts.sample_rate, ts.bps, ts.channels,
                 ts.nframes) for i, ts in items]
        if host == dst_host:
            path = os.path.join(spool, f"rank{self.rank}.bin")
            with open(path, "wb") as f:
                for _, ts in items:
                    f.write(ts.header)
                    f.write(ts.body)
            payload = ("file", path, meta)
        else:  # no shared spool: bytes through the gloo group
            payload = ("inline", b"".join(ts.header + bytes(ts.body) for _, ts in items), meta)
        parts = self.gather_objects(payload, dst)
        if self.rank != dst:
            return None
        out = []
        for kind, where, man in parts:
            if kind == "file":
                buf = Path(where).read_bytes()
                os.unlink(where)
            else:
                buf = where
            mv, pos, lst = memoryview(buf), 0, []
            for (i, hl, bl, mn, mx, sr, bps, ch, nf) in man:
                lst.append((i, TileStream(bytes(mv[pos:pos + hl]), mv[pos + hl:pos + hl + bl], mn, mx, sr, bps, ch, nf)))
                pos += hl + bl
            out.append(lst)
        try:
            os.rmdir(spool)
        except OSError:
            pass
        return out

    def close(self):
        if self.pg is not None:
            self.pg.barrier()
            self.pg.destroy_process_group()
            self.pg = None


def shard(tiles: Sequence[Tuple[int, int, int, int]], world: int, rank: int) -> List[int]:
    """Indices of the tiles this rank encodes (LPT on pixel count, deterministic)."""
    return lpt_assign([t[2] * t[3] for t in tiles], world)[rank]


EncodeFn = Callable[..., List[TileStream]]


def read_rank_mosaic(src, windows: Sequence[Tuple[int, int, int, int]], pinned: bool = False):
    """Decode ONLY ``windows`` of a GeoTIFF (path or open ``GeoTIFF``) into one rank-local band-planar
    mosaic: window k at rows [off_k, off_k + h_k), columns [0, w_k) (stacked top to bottom; page-locked
    when ``pinned``).  Returns ``(mosaic, local_windows)``; every local window holds exactly the pixels of
    its source window, so its FLAC stream is byte-identical (the rasterio ``read(window=...)`` per tile of
    ``cli.py:559``, here one decode per window straight into the rank's buffer)."""
    from .tiff import GeoTIFF, _alloc

    g = src if isinstance(src, GeoTIFF) else GeoTIFF(src)
    try:
        rows = sum(h for (_, _, h, _) in windows)
        width = max((w for (_, _, _, w) in windows), default=0)
        mosaic = _alloc((g.info.count, max(1, rows), max(1, width)), g.info.dtype, pinned)
        local = []
        off = 0
        for (r0, c0, h, w) in windows:
            g.read_window_into(mosaic[:, off:off + h, :w], r0, c0, h, w)
            local.append((off, 0, h, w))
            off += h
        return mosaic, local
    finally:
        if g is not src:
            g.close()


def rank_items(tiles: Sequence[Tuple[int, int, int, int]], world: int, rank: int,
               split: str = "frames") -> List[Tuple[int, int, int]]:
    """This rank's work items (tile index, first frame, frame count): ``split="frames"`` -- equal frame
    counts per rank (``frame_split``: whole tiles plus at most a partial tile at each end, SURVEY.md 8(e)'s
    (tile, frame-range) items); ``"strided"`` -- the same over the tiles in strided order (tile index mod
    world first: every rank samples the whole scene); ``"lpt"`` -- whole tiles by LPT on pixel count."""
    if split in ("frames", "strided"):
        return frame_split(tiles, world, stride=world if split == "strided" else 1)[rank]
    return [(i, 0, frames_of(tiles[i])) for i in shard(tiles, world, rank)]


def encode_tiles_distributed(raster, tiles: Sequence[Tuple[int, int, int, int]], level: int = 5,
                             d: Optional[Dist] = None, encode_fn: EncodeFn = encode_tiles,
                             dst: int = 0, split: str = "frames") -> Optional[List[TileStream]]:
    """Each rank encodes its work items (``rank_items``) on its local GPU; ``dst`` receives every stream in
    tile order (other ranks get ``None``): the frames of a tile split over ranks are concatenated in frame
    order, which is exactly the tile's stream.  Bytes are identical for any world size and split.
    ``raster`` is an in-memory (bands, H, W) array, or a GeoTIFF path / ``GeoTIFF``: then every rank
    decodes only the windows of its own tiles (``read_rank_mosaic``), never the whole scene.  ``encode_fn``
    takes ``frame_ranges=`` when a rank holds part of a tile."""
    d = d or Dist()
    items = rank_items(tiles, d.world, d.rank, split)
    mine = [i for i, _, _ in items]
    whole = all(f0 == 0 and n >= frames_of(tiles[i]) for i, f0, n in items)
    kw = {} if whole else {"frame_ranges": [(f0, n) for _, f0, n in items]}
    if isinstance(raster, (str, os.PathLike)) or type(raster).__name__ == "GeoTIFF":
        mosaic, local = read_rank_mosaic(raster, [tiles[i] for i in mine], pinned=encode_fn is encode_tiles)
        streams = encode_fn(mosaic, local, level, [d.local_rank], **kw) if mine else []
        del mosaic
    else:
        streams = encode_fn(raster, [tiles[i] for i in mine], level, [d.local_rank], **kw) if mine else []
    parts = d.gather_streams([((i, f0), ts) for (i, f0, _), ts in zip(items, streams)], dst)
    if d.rank != dst:
        return None
    pieces: List[List[Tuple[int, TileStream]]] = [[] for _ in tiles]
    for part in parts:
        for (i, f0), ts in part:
            pieces[i].append((f0, ts))
    out: List[TileStream] = []
    for i, ps in enumerate(pieces):
        if not ps:
            raise RuntimeError(f"tile {i} was not encoded by any rank")
        ps.sort(key=lambda x: x[0])
        if len(ps) == 1:
            out.append(ps[0][1])
            continue
        head = ps[0][1]
        body = b"".join(bytes(ts.body) for _, ts in ps)
        out.append(TileStream(head.header, body, head.data_min, head.data_max, head.sample_rate, head.bps,
                              head.channels, sum(ts.nframes for _, ts in ps)))
    return out
