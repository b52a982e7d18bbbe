"""FLAC decoding for the read side, on the native decoder ``fra_decode``.

``FileDecoder(path).process()`` reproduces what the reference gets from
``pyflac.FileDecoder(path).process()`` (``converter.py:179-183``, ``cli.py:477-483``): pyflac hands
each decoded block (int16 for 16-bps streams, int32 for 32-bps) to a ``soundfile.SoundFile`` opened
with the WAV default subtype PCM_16, then returns ``sf.read(always_2d=True)`` = float64 samples / 32768
(``docs/sonos-pyflac.txt:1571-1640, 1809-1854``).  libsndfile's int -> short conversion keeps the
upper 16 bits (``x >> 16``), so 32-bps streams come back truncated (F8) -- reproduced here, since
``flac_to_tiff`` denormalises those floats.  ``decode_flac`` returns the exact integers.
"""

from __future__ import annotations

from pathlib import Path
from typing import Tuple, Union

import numpy as np

from . import _native


def decode_flac(data: bytes, concat: bool = False) -> Tuple[np.ndarray, int, int]:
    """Exact decode -> ((N, C) int16 for 16-bps / int32 otherwise, sample_rate, bps)."""
    samples, info = _native.decode(bytes(data), concat=concat)
    if info.bps <= 16:
        samples = samples.astype(np.int16)
    return samples, info.sample_rate, info.bps


def pcm16_float(samples: np.ndarray) -> np.ndarray:
    """The SoundFile PCM_16 write + float64 read round trip of pyflac's FileDecoder."""
    s = np.asarray(samples)
    if s.dtype == np.int16:
        return s.astype(np.float64) / 32768.0
    return (s.astype(np.int32) >> 16).astype(np.float64) / 32768.0


class FileDecoder:
    """``pyflac.FileDecoder`` stand-in: ``process()`` -> (float64 (N, C), sample_rate)."""

    def __init__(self, input_file: Union[str, Path], output_file: Union[str, Path] = None):
        self.input_file = Path(input_file)
        self.output_file = output_file

    def process(self) -> Tuple[np.ndarray, int]:
        samples, sr, _ = decode_flac(self.input_file.read_bytes())
        return pcm16_float(samples), sr
