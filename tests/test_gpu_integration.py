"""INTEGRATION.md's ctypes binding, run exactly as written, against the CPU oracle.

The `encode_tiles` snippet of INTEGRATION.md §3 (the reference-side binding a maintainer would add in
place of the pyflac call, `/root/reference/docs/sonos-pyflac.txt:3205-3262`) is extracted from the
document and executed with only the library path pointed at the in-tree build; its streams must equal
the oracle's (86-byte header + frames, FRA-1) byte for byte.  This is the one-shot `fra_encode` entry
(SURVEY.md §8(b) item 1).
"""
import re
from pathlib import Path

import numpy as np
import pytest

import oracle as O
from flac_raster import _native as N

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _snippet():
    text = (ROOT / "INTEGRATION.md").read_text()
    blocks = re.findall(r"```python\n(.*?)```", text, flags=re.S)
    code = next(b for b in blocks if "def encode_tiles" in b)
    lib = str(N._LIB_PATH)
    code = re.sub(r'C\.CDLL\("[^"]*"\)', f"C.CDLL({lib!r})", code)
    ns = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    return ns


@pytest.mark.parametrize("dtype", ["uint16", "int16"])
def test_integration_snippet_fra_encode_matches_oracle(dtype):
    N.load()  # fails loudly when the HIP library or the device is missing
    ns = _snippet()
    rng = np.random.default_rng(7)
    B, H, W = 3, 300, 520
    base = np.cumsum(rng.integers(-40, 41, size=(B, H, W)), axis=2)
    raster = (base - base.min() + (0 if dtype == "uint16" else -20000)).astype(dtype)
    # full frames, a ragged last frame, and a tile on the raster edge
    tiles = [(0, 0, 128, 256), (128, 0, 100, 333), (200, 256, 100, 264)]
    streams, params = ns["encode_tiles"](raster, tiles, level=5)
    assert len(streams) == len(tiles)
    for (r, c, h, w), got, (mn, mx) in zip(tiles, streams, params):
        inter = raster[:, r:r + h, c:c + w].transpose(1, 2, 0).reshape(-1, B)
        audio, omn, omx = O.normalize(inter, 16)
        exp = O.encode(audio, O.sample_rate_for_pixels(h * w), level=5)
        assert (mn, mx) == (float(omn), float(omx))
        assert got == exp, f"tile {(r, c, h, w)}: {len(got)} vs {len(exp)} bytes"
        dec, sr, bps, _ = O.decode(got)
        assert (sr, bps) == (O.sample_rate_for_pixels(h * w), 16)
        assert np.array_equal(dec, audio.astype(np.int32))
