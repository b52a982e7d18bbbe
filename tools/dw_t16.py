import os, sys, time
sys.path.insert(0, "tests"); sys.path.insert(0, "flac-raster_amd"); sys.path.insert(0, "oracle")
import numpy as np
import test_gpu_direct_write as T
from flac_raster.tiles import calculate_tiles
bs = int(sys.argv[1]); dw = sys.argv[2] == "1"; wmode = sys.argv[3]
r = T._mixed_raster(3, 160, 170, np.int16, 3)
wins = calculate_tiles(160, 170, 64)
if wmode == "tiny": wins = wins + [(0, 0, 1, 1), (5, 7, 1, 3)]
if wmode == "only_tiny": wins = [(0, 0, 1, 1), (5, 7, 1, 3)]
t = time.time()
o = T._plan_bytes(r, wins, 5, 0, dw, blocksize=bs)
print("bs", bs, "dw", dw, wmode, "ok", len(o[0]), "%.3fs" % (time.time() - t), flush=True)
