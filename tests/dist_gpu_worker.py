"""Child process of tests/test_gpu_dist.py: one rank of ``dist.encode_tiles_distributed`` with the REAL
GPU encoder (``tiles.encode_tiles``) on a GeoTIFF, gathered through the node-local spool file; rank 0
writes the container.  Every rank uses device 0 (one-GPU box) and the gloo backend.
usage: dist_gpu_worker.py <rank> <world> <port> <geotiff> <tile> <level> <out>"""
import os
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent / "flac-raster_amd"))


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    src, tile, level, out = Path(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6]), Path(sys.argv[7])
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from flac_raster.dist import Dist, encode_tiles_distributed, shard
    from flac_raster.geo import Affine
    from flac_raster.streaming import assemble_streaming
    from flac_raster.tiff import GeoTIFF
    from flac_raster.tiles import calculate_tiles

    d = Dist(backend="gloo")
    g = GeoTIFF(src)
    info = g.info
    g.close()
    tiles = calculate_tiles(info.height, info.width, tile)
    mine = shard(tiles, world, rank)
    streams = encode_tiles_distributed(src, tiles, level, d)  # encode_fn = tiles.encode_tiles (GPU)
    Path(f"{out}.rank{rank}").write_text(f"{len(mine)}")
    if rank == 0:
        blob = assemble_streaming(tiles, streams, (info.count, info.height, info.width), info.dtype,
                                  Affine(*info.transform), info.crs, tile)
        out.write_bytes(blob)
    else:
        assert streams is None
    d.close()


if __name__ == "__main__":
    main()
