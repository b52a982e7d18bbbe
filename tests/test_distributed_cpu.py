"""Multi-process path on the CPU (gloo, world_size 2 and 3): tile sharding, the gather to the writer
rank, max/sum reductions, and byte-identical containers for any world size.

The per-rank encoder is the oracle stand-in (tests/oracle_tiles.py), byte-identical to the GPU
encoder; on an MI355X node the same ``encode_tiles_distributed`` runs with ``encode_tiles``."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = Path(__file__).resolve().parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _raster():
    rng = np.random.default_rng(3)
    base = np.cumsum(np.cumsum(rng.integers(-2, 3, size=(3, 200, 333)), axis=1), axis=2)
    return (base - base.min()).astype(np.int16)


def _worker(rank, world, port, out_dir, from_file=False, tile=64, split="frames"):
    for p in (HERE.parent / "flac-raster_amd", HERE.parent / "oracle", HERE):
        sys.path.insert(0, str(p))
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from flac_raster.dist import Dist, encode_tiles_distributed, shard
    from flac_raster.geo import Affine
    from flac_raster.streaming import assemble_streaming
    from flac_raster.tiles import calculate_tiles
    from oracle_tiles import oracle_encode_tiles

    d = Dist(backend="gloo")
    r = _raster()
    tiles = calculate_tiles(200, 333, tile)
    mine = shard(tiles, world, rank)
    assert d.allsum(len(mine)) == len(tiles)
    assert d.allmax(float(rank)) == float(world - 1)
    d.barrier()
    src = Path(out_dir, "scene.tif") if from_file else r  # file: each rank decodes only its own windows
    streams = encode_tiles_distributed(src, tiles, 5, d, encode_fn=oracle_encode_tiles, split=split)
    if rank == 0:
        blob = assemble_streaming(tiles, streams, r.shape, r.dtype, Affine(30.0, 0, 1000.0, 0, -30.0, 9000.0),
                                  "EPSG:3857", tile)
        Path(out_dir, f"w{world}{'f' if from_file else ''}_{tile}_{split}.bin").write_bytes(blob)
    else:
        assert streams is None
    d.close()


@pytest.mark.parametrize("world,tile,split", [(2, 64, "frames"), (3, 64, "lpt"), (3, 128, "frames"),
                                              (2, 160, "frames"), (3, 64, "strided")])
def test_distributed_container_identical(tmp_path, world, tile, split):
    """World 2/3, whole-tile LPT items and (tile, frame range) items: with tiles of 4-7 frames the equal
    frame-count split cuts tiles between ranks, whose frame slices the writer joins back into streams."""
    sys.path.insert(0, str(HERE))
    from flac_raster.geo import Affine
    from flac_raster.streaming import assemble_streaming
    from flac_raster.tiles import calculate_tiles, frame_split
    from oracle_tiles import oracle_encode_tiles

    tiles = calculate_tiles(200, 333, tile)
    if tile > 64 and split == "frames":  # the split really cuts a tile
        assert any(f0 > 0 for part in frame_split(tiles, world) for _, f0, _ in part)
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), False, tile, split), nprocs=world, join=True)
    r = _raster()
    ref = assemble_streaming(tiles, oracle_encode_tiles(r, tiles, 5), r.shape, r.dtype,
                             Affine(30.0, 0, 1000.0, 0, -30.0, 9000.0), "EPSG:3857", tile)
    assert (tmp_path / f"w{world}_{tile}_{split}.bin").read_bytes() == ref


@pytest.mark.parametrize("strided", [False, True])
def test_frame_split_partitions_frames(strided):
    from flac_raster.tiles import PARTIAL_FRAME_COST, calculate_tiles, frame_split, frames_of

    tiles = calculate_tiles(10980, 10980, 1024)
    F = sum(frames_of(t) for t in tiles)
    for world in (1, 2, 3, 8):
        parts = frame_split(tiles, world, stride=world if strided else 1)
        if strided and world == 8:  # every part's run spans the scene (tiles of every row band)
            assert all(max(i for i, _, _ in p) - min(i for i, _, _ in p) > len(tiles) // 2 for p in parts)
        # equal cost: the frames, + PARTIAL_FRAME_COST for the part holding the corner tile's partial last frame
        def cost(p):
            return sum(n for _, _, n in p) + (PARTIAL_FRAME_COST if any(
                f0 + n == frames_of(tiles[i]) and (tiles[i][2] * tiles[i][3]) % 4096 for i, f0, n in p) else 0)
        eq = frame_split(tiles, world, stride=world if strided else 1, partial_cost=0)
        assert max(map(cost, parts)) <= max(map(cost, eq))  # never worse than equal frame counts
        if world > 1 and not strided:  # the part holding the partial frame gets fewer frames
            owner = next(k for k, p in enumerate(parts) if any(i == len(tiles) - 1 for i, _, _ in p))
            assert sum(n for _, _, n in parts[owner]) < min(sum(n for _, _, n in p) for k, p in enumerate(parts)
                                                            if k != owner)
        assert max(sum(n for _, _, n in p) for p in eq) - min(sum(n for _, _, n in p) for p in eq) <= 1
        seen = {}
        for p in parts:
            for i, f0, n in p:
                seen.setdefault(i, []).append((f0, n))
        assert sorted(seen) == list(range(len(tiles)))
        for i, rs in seen.items():  # every tile's frames exactly once, in order
            rs.sort()
            assert rs[0][0] == 0 and all(a + n == b for (a, n), (b, _) in zip(rs, rs[1:]))
            assert rs[-1][0] + rs[-1][1] == frames_of(tiles[i])
        assert sum(n for p in parts for _, _, n in p) == F


def test_distributed_ranks_read_own_windows(tmp_path):
    """World 2 from a GeoTIFF file: each rank decodes only its LPT tiles' windows into a rank-local
    mosaic (read_rank_mosaic) and the container equals the single-process one."""
    sys.path.insert(0, str(HERE))
    from flac_raster.dist import read_rank_mosaic, shard
    from flac_raster.geo import Affine
    from flac_raster.streaming import assemble_streaming
    from flac_raster.tiff import write_geotiff
    from flac_raster.tiles import calculate_tiles
    from oracle_tiles import oracle_encode_tiles

    r = _raster()
    write_geotiff(tmp_path / "scene.tif", r)
    tiles = calculate_tiles(200, 333, 64)
    mine = [tiles[i] for i in shard(tiles, 2, 1)]
    mosaic, local = read_rank_mosaic(tmp_path / "scene.tif", mine)
    assert mosaic.shape[1] == sum(t[2] for t in mine) and mosaic.nbytes < r.nbytes
    for (r0, c0, h, w), (o, _, lh, lw) in zip(mine, local):
        assert np.array_equal(mosaic[:, o:o + lh, :lw], r[:, r0:r0 + h, c0:c0 + w])
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), True), nprocs=2, join=True)
    ref = assemble_streaming(tiles, oracle_encode_tiles(r, tiles, 5), r.shape, r.dtype,
                             Affine(30.0, 0, 1000.0, 0, -30.0, 9000.0), "EPSG:3857", 64)
    assert (tmp_path / "w2f_64_frames.bin").read_bytes() == ref


def test_shards_partition_tiles():
    from flac_raster.dist import shard
    from flac_raster.tiles import calculate_tiles

    tiles = calculate_tiles(10980, 10980, 1024)
    for world in (1, 2, 4, 8):
        got = sorted(i for r in range(world) for i in shard(tiles, world, r))
        assert got == list(range(len(tiles)))
