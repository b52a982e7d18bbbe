"""Test configuration.

* ``-m gpu`` tests run the HIP encoder on an MI355X and compare with the CPU oracle
  (``oracle/``, test infrastructure only).  They FAIL (never skip) when the extension or the
  device is missing, so a silent fallback cannot pass.
* everything else runs on the CPU (oracle vs committed golden fixtures, host logic, ABI exports).
"""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "flac-raster_amd", ROOT / "oracle", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
