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

from .tiles import TileStream, encode_tiles, lpt_assign


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


def encode_tiles_distributed(raster, tiles: Sequence[Tuple[int, int, int, int]], level: int = 5,
                             d: Optional[Dist] = None, encode_fn: EncodeFn = encode_tiles,
                             dst: int = 0) -> Optional[List[TileStream]]:
    """Each rank encodes its LPT share on its local GPU; ``dst`` receives every stream in tile order
    (other ranks get ``None``).  Bytes are identical for any world size.  ``raster`` is an in-memory
    (bands, H, W) array, or a GeoTIFF path / ``GeoTIFF``: then every rank decodes only its own tiles'
    windows (``read_rank_mosaic``), never the whole scene."""
    d = d or Dist()
    mine = shard(tiles, d.world, d.rank)
    if isinstance(raster, (str, os.PathLike)) or type(raster).__name__ == "GeoTIFF":
        mosaic, local = read_rank_mosaic(raster, [tiles[i] for i in mine], pinned=encode_fn is encode_tiles)
        streams = encode_fn(mosaic, local, level, [d.local_rank]) if mine else []
        del mosaic
    else:
        streams = encode_fn(raster, [tiles[i] for i in mine], level, [d.local_rank]) if mine else []
    parts = d.gather_streams(list(zip(mine, streams)), dst)
    if d.rank != dst:
        return None
    out: List[Optional[TileStream]] = [None] * len(tiles)
    for part in parts:
        for i, ts in part:
            out[i] = ts
    if any(ts is None for ts in out):
        raise RuntimeError("a tile was not encoded by any rank")
    return out  # type: ignore[return-value]
