"""pyflac-compatible ``StreamEncoder`` backed by the MI355X encoder.

Drop-in for the two reference call sites::

    encoder = pyflac.StreamEncoder(write_callback=cb, sample_rate=sr,
                                   compression_level=level, blocksize=4096)
    encoder._channels = channels; encoder._bits_per_sample = bps   # overridden, see F3
    encoder.process(audio)
    encoder.finish()

(``converter.py:139-154``, ``spatial_encoder.py:291-304``; pyflac 3.0.0 semantics from
``docs/sonos-pyflac.txt:1968-2014, 2175-2212, 2311-2332``):

* the first ``process()`` fixes ``channels = samples.shape[1]`` and
  ``bits_per_sample = samples.dtype.itemsize * 8`` (int16 -> 16-bps, int32 -> 32-bps FLAC);
* ``blocksize=0`` takes the level's default (1152 for levels 0-2, 4096 for 3-8);
* the write callback receives, in order, ``fLaC`` (4 B), the STREAMINFO block (38 B) and the
  VORBIS_COMMENT block (44 B) with ``num_samples = 0``, then one call per frame with
  ``num_samples = blocksize of that frame`` and ``current_frame = frame number``
  (libFLAC 1.4.3 stream encoder, ``:6601-6637``);
* encoding happens on the GPU at ``finish()`` (libFLAC emits full blocks during ``process``; the
  bytes and the callback sequence are the same, only the timing of the calls differs).
"""

from __future__ import annotations

import enum
import logging
from typing import Callable, List, Optional

import numpy as np

from . import _native


class EncoderState(enum.Enum):
    OK = 0
    UNINITIALIZED = 1
    OGG_ERROR = 2
    VERIFY_DECODER_ERROR = 3
    VERIFY_MISMATCH_IN_AUDIO_DATA = 4
    CLIENT_ERROR = 5
    IO_ERROR = 6
    FRAMING_ERROR = 7
    MEMORY_ALLOCATION_ERROR = 8

    def __str__(self):
        return "FLAC__STREAM_ENCODER_" + self.name


class EncoderInitException(Exception):
    """Invalid encoder configuration (pyflac raises this from ``init_stream``)."""

    def __init__(self, code, msg: str = ""):
        super().__init__(msg or str(code))
        self.code = code


class EncoderProcessException(Exception):
    """Encoding failed (pyflac raises this when ``process_interleaved`` returns false)."""


def default_blocksize(level: int) -> int:
    """libFLAC's per-level block size (``sonos-pyflac.txt:6926-6934``)."""
    return 1152 if level <= 2 else 4096


class StreamEncoder:
    """GPU FLAC stream encoder with pyflac's constructor, ``process``/``finish`` and callbacks."""

    def __init__(self, sample_rate: int, write_callback: Callable[[bytes, int, int, int], None],
                 seek_callback: Callable = None, tell_callback: Callable = None, metadata_callback: Callable = None,
                 compression_level: int = 5, blocksize: int = 0, streamable_subset: bool = True,
                 verify: bool = False, limit_min_bitrate: bool = False, device: int = 0):
        self.write_callback = write_callback
        self.seek_callback = seek_callback
        self.tell_callback = tell_callback
        self.metadata_callback = metadata_callback
        self._sample_rate = sample_rate
        self._blocksize = blocksize
        self._compression_level = compression_level
        self._streamable_subset = streamable_subset
        self._verify = verify
        self._limit_min_bitrate = limit_min_bitrate
        self._device = device
        self._channels = None
        self._bits_per_sample = None
        self._initialised = False
        self._chunks: List[np.ndarray] = []
        self._state = EncoderState.UNINITIALIZED
        self.logger = logging.getLogger("flac_raster.encoder")

    @property
    def state(self) -> EncoderState:
        return self._state

    def _init(self):
        if not 0 <= int(self._compression_level) <= 8:
            raise EncoderInitException("INVALID_COMPRESSION_LEVEL", "compression level must be 0..8")
        if self._bits_per_sample not in (16, 32):
            raise EncoderInitException(
                "INVALID_BITS_PER_SAMPLE",
                f"{self._bits_per_sample}-bit samples: the GPU encoder takes int16 or int32 arrays")
        if not 1 <= self._channels <= 8:
            raise EncoderInitException("INVALID_NUMBER_OF_CHANNELS", f"{self._channels} channels (1..8)")
        bs = self._blocksize or default_blocksize(self._compression_level)
        if not 16 <= bs <= 4096:
            raise EncoderInitException("INVALID_BLOCK_SIZE", f"blocksize {bs} (16..4096 on this encoder)")
        if not 0 < self._sample_rate < (1 << 20):
            raise EncoderInitException("INVALID_SAMPLE_RATE", f"sample rate {self._sample_rate}")
        self._bs = bs
        self._initialised = True
        self._state = EncoderState.OK

    def process(self, samples: np.ndarray):
        if not isinstance(samples, np.ndarray):
            raise TypeError("Processing only supports numpy arrays")
        if not self._initialised:
            self._channels = samples.shape[1] if samples.ndim > 1 else 1
            self._bits_per_sample = samples.dtype.itemsize * 8
            self._init()
        s = samples.reshape(len(samples), -1) if samples.ndim != 2 else samples
        if s.shape[1] != self._channels:
            self._state = EncoderState.CLIENT_ERROR
            raise EncoderProcessException(str(self._state))
        dt = np.int16 if self._bits_per_sample == 16 else np.int32
        self._chunks.append(np.ascontiguousarray(s).astype(dt, copy=True))

    def finish(self) -> bool:
        if not self._initialised:
            return True
        samples = (np.concatenate(self._chunks) if len(self._chunks) != 1 else self._chunks[0])
        self._chunks = []
        try:
            info, frames, offsets = _native.encode_interleaved(samples, self._sample_rate, self._compression_level,
                                                               self._bs, self._device, return_offsets=True)
        except _native.NativeError as e:
            self._state = EncoderState.MEMORY_ALLOCATION_ERROR
            raise EncoderProcessException(str(e)) from e
        header = _native.stream_header(self._channels, self._bits_per_sample, self._sample_rate, self._bs)
        self._emit(header[:4], 0, 0)
        self._emit(header[4:42], 0, 0)
        self._emit(header[42:86], 0, 0)
        n = len(samples)
        mv = memoryview(frames)
        for i in range(len(offsets) - 1):
            a, b = int(offsets[i]), int(offsets[i + 1])
            self._emit(bytes(mv[a:b]), min(self._bs, n - i * self._bs), i)
        self._initialised = False
        self._state = EncoderState.UNINITIALIZED
        return True

    def _emit(self, buf: bytes, num_samples: int, current_frame: int):
        try:
            self.write_callback(buf, len(buf), num_samples, current_frame)
        except Exception as e:  # pyflac maps callback exceptions to FATAL_ERROR
            self._state = EncoderState.CLIENT_ERROR
            raise EncoderProcessException(str(e)) from e


def encode_array(samples: np.ndarray, sample_rate: int, compression_level: int = 5, blocksize: int = 4096,
                 device: int = 0) -> bytes:
    """Whole-stream convenience: ``bytes`` of header + frames for (N, C) int16/int32 samples."""
    out = bytearray()
    enc = StreamEncoder(sample_rate, lambda b, n, s, f: out.extend(b), compression_level=compression_level,
                        blocksize=blocksize, device=device)
    enc.process(np.asarray(samples))
    enc.finish()
    return bytes(out)
