"""The distributed product path on the GPU: two fresh child processes
(started before either touches the GPU), both on device 0 with the gloo backend, each run
``dist.encode_tiles_distributed`` with the real ``tiles.encode_tiles`` on their LPT share of a GeoTIFF (each
decodes only its own windows), gathered through the node-local spool file -- the path one rank per GPU takes
on an 8-GPU node (reference loop being sharded: cli.py:553-630).  The container must equal the
single-process one byte for byte."""
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from flac_raster.streaming import create_streaming_flac
from flac_raster.synth import synth_window
from flac_raster.tiff import write_geotiff

pytestmark = pytest.mark.gpu
HERE = Path(__file__).resolve().parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,dtype,level,tile", [(2, np.uint16, 5, 512), (3, np.float32, 8, 256)])
def test_distributed_gpu_container_equals_single_process(tmp_path, world, dtype, level, tile):
    kind = 4 if dtype == np.uint16 else 5
    r = synth_window(kind, 31, 3, 1800, 1500).astype(dtype)
    src = tmp_path / "scene.tif"
    write_geotiff(src, r, compression="deflate", tile=256, predictor=2 if dtype == np.uint16 else 1,
                  transform=(10.0, 0.0, 300000.0, 0.0, -10.0, 5000040.0), crs="EPSG:32633")
    out = tmp_path / "dist.flac"
    port = _free_port()
    procs = [subprocess.Popen([sys.executable, str(HERE / "dist_gpu_worker.py"), str(k), str(world), str(port),
                               str(src), str(tile), str(level), str(out)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for k in range(world)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=100)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)
    counts = [int(Path(f"{out}.rank{k}").read_text()) for k in range(world)]
    assert all(c > 0 for c in counts)  # every rank encoded a share
    single = tmp_path / "single.flac"
    create_streaming_flac(src, single, tile, level)
    assert out.read_bytes() == single.read_bytes()


def _bench_line(args, env_extra, timeout=240):
    import json
    import os
    env = dict(os.environ, **env_extra)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(HERE.parent / "bench.py"), *args], env=env, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_bench_gpus_flag_starts_the_ranks_itself():
    """``bench.py --gpus 2`` without a launcher starts two fresh rank processes (here both on
    device 0 over gloo, a labelled rehearsal) and reports a 2-GPU line whose frames equal the 1-rank line's
    (reference loop being sharded: cli.py:553-622)."""
    common = ["--config", "c3", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-e2e", "--no-pmc", "--no-trace"]
    one = _bench_line(["--gpus", "1", *common], {})
    two = _bench_line(["--gpus", "2", *common], {"FRA_DIST_BACKEND": "gloo"})
    assert one["n_gpus"] == 1 and "rehearsal" not in one
    assert two["n_gpus"] == 2 and two["rehearsal"].startswith("2 ranks on")
    assert len(two["per_rank"]) == 2 and all(r["frame_bytes"] > 0 for r in two["per_rank"])
    assert two["config"]["compressed_bytes"] == one["config"]["compressed_bytes"]
    assert sum(r["frame_bytes"] for r in two["per_rank"]) == one["config"]["compressed_bytes"]
    assert two["config"]["split"] == "frames" and "frame range" in two["config"]["parallelism"]
    assert one["analysis_instance"]["first_execute"] == 17


def test_bench_gpus_flag_refuses_more_ranks_than_gpus():
    import os
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "FRA_DIST_BACKEND"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(HERE.parent / "bench.py"), "--gpus", "64", "--config", "c3"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "GPU(s) visible" in r.stderr
