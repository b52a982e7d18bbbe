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
  ``bits_per_sample = samples.dtype.itemsize * 8`` (int16 -> 16-bps, int32 -> 32-bps FLAC) and
  initialises the stream: the write callback receives ``fLaC`` (4 B), the STREAMINFO block (38 B) and
  the VORBIS_COMMENT block (44 B) with ``num_samples = 0`` right there, as libFLAC's ``init_stream``
  does under pyflac's ``_init`` (``:1986-1991``, ``:2200-2212``);
* ``blocksize=0`` takes the level's default (1152 for levels 0-2, 4096 for 3-8);
* every ``process()`` encodes, on the GPU, the complete blocks it can and calls back once per frame
  (``num_samples`` = the frame's block size, ``current_frame`` = its number).  Like libFLAC 1.4.3's
  ``process_interleaved`` (stream_encoder.c keeps one sample of look-ahead, ``OVERREAD_``: a block is
  encoded once blocksize + 1 samples are buffered, the final block only by ``finish()``), the samples
  of the last block stay buffered until more arrive or ``finish()`` flushes them.  libFLAC's source is
  not in this container; that timing rule is restated from the public libFLAC sources and is not
  pinned by a fixture here.  Bytes are independent of how the samples are split across calls.
* GPU plans are cached per block count, so repeated calls of one size reuse their device workspace.
"""

from __future__ import annotations

import enum
import logging
from collections import OrderedDict
from typing import Callable, Optional

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

    _PLAN_CACHE = 4

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
        self._pending: Optional[np.ndarray] = None
        self._next_frame = 0
        self._plans: "OrderedDict" = OrderedDict()  # block count -> (plan, page-locked output buffer)
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
        self._dtype = np.int16 if self._bits_per_sample == 16 else np.int32
        self._pending = np.empty((0, self._channels), self._dtype)
        self._next_frame = 0
        self._initialised = True
        self._state = EncoderState.OK
        # libFLAC init_stream: the stream header reaches the write callback during initialisation
        header = _native.stream_header(self._channels, self._bits_per_sample, self._sample_rate, self._bs)
        self._emit(header[:4], 0, 0)
        self._emit(header[4:42], 0, 0)
        self._emit(header[42:86], 0, 0)

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
        s = np.ascontiguousarray(s).astype(self._dtype, copy=False)
        pend = np.concatenate([self._pending, s]) if len(self._pending) else np.ascontiguousarray(s)
        nblk = (len(pend) - 1) // self._bs if len(pend) > self._bs else 0  # one sample of look-ahead
        if nblk:
            self._encode_emit(pend[: nblk * self._bs])
            pend = pend[nblk * self._bs:]
        # always an own copy (<= blocksize rows): the caller may refill its buffer before the next call
        self._pending = pend.copy()

    def finish(self) -> bool:
        if not self._initialised:
            return True
        if len(self._pending):
            self._encode_emit(self._pending)
        self._pending = None
        self.close()
        self._initialised = False
        self._state = EncoderState.UNINITIALIZED
        return True

    def _plan_key(self, n: int):
        return ("shim", self._device, np.dtype(self._dtype).str, self._channels, n, self._compression_level,
                self._bs, self._sample_rate)

    def _plan_for(self, n: int):
        if n in self._plans:
            self._plans.move_to_end(n)
            return self._plans[n]

        def make():
            ctx = _native.default_context(self._device)
            C = self._channels
            plan = _native.Plan(ctx, None, False, self._dtype, C, (1, n * C, C), [(0, 0, 1, n)],
                                self._compression_level, self._bs, 0, self._sample_rate)
            cap, _ = plan.capacity()
            return (plan, _native.pinned_empty(cap, np.uint8))

        ent = _native.acquire_plan(self._plan_key(n), make)
        self._plans[n] = ent
        while len(self._plans) > self._PLAN_CACHE:
            k, old = self._plans.popitem(last=False)
            _native.release_plan(self._plan_key(k), old)
        return ent

    def _encode_emit(self, block: np.ndarray):
        n = len(block)
        try:
            plan, out = self._plan_for(n)
            plan.set_first_frame(self._next_frame)
            plan.encode_host(block, out)
            nfr = (n + self._bs - 1) // self._bs
            offsets = plan.frame_offsets(nfr)
        except _native.NativeError as e:
            self._state = EncoderState.MEMORY_ALLOCATION_ERROR
            raise EncoderProcessException(str(e)) from e
        mv = memoryview(out)
        for i in range(nfr):
            a, b = int(offsets[i]), int(offsets[i + 1])
            self._emit(bytes(mv[a:b]), min(self._bs, n - i * self._bs), self._next_frame + i)
        self._next_frame += nfr

    def close(self):
        """Hand this encoder's GPU plans back to the process-wide pool (the next encoder of the same
        shape reuses them).  Also done by ``finish()`` and on garbage collection."""
        for k, ent in self._plans.items():
            _native.release_plan(self._plan_key(k), ent)
        self._plans.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

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
