"""Multi-process (one process per GPU) driver for the tile encoder.

SURVEY.md 8(e): tiles are independent units, so ranks encode disjoint tile sets with no exchange on
the data path.  The only collective is the final hand-off of the encoded streams to the rank that
writes the container (``gather_streams``), plus barrier / max-time reductions for measurement.
Works with ``torch.distributed`` on ``nccl`` (= RCCL over xGMI on MI355X) or ``gloo`` (CPU tests);
launched by ``torch.distributed.run`` (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR in the env).
"""

from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence, Tuple

from .tiles import TileStream, encode_tiles, lpt_assign


class Dist:
    """Rank/world plus the few collectives the encoder uses (no-ops when world == 1)."""

    def __init__(self, backend: Optional[str] = None):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
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
        self.pg.gather_object(obj, out, dst=dst)
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


def encode_tiles_distributed(raster, tiles: Sequence[Tuple[int, int, int, int]], level: int = 5,
                             d: Optional[Dist] = None, encode_fn: EncodeFn = encode_tiles,
                             dst: int = 0) -> Optional[List[TileStream]]:
    """Each rank encodes its LPT share on its local GPU; ``dst`` receives every stream in tile order
    (other ranks get ``None``).  Bytes are identical for any world size."""
    d = d or Dist()
    mine = shard(tiles, d.world, d.rank)
    streams = encode_fn(raster, [tiles[i] for i in mine], level, [d.local_rank]) if mine else []
    parts = d.gather_objects(list(zip(mine, streams)), dst)
    if d.rank != dst:
        return None
    out: List[Optional[TileStream]] = [None] * len(tiles)
    for part in parts:
        for i, ts in part:
            out[i] = ts
    if any(ts is None for ts in out):
        raise RuntimeError("a tile was not encoded by any rank")
    return out  # type: ignore[return-value]
