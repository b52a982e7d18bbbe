"""ctypes binding of ``libflac_raster_amd.so`` (C ABI: ``include/flac_raster_amd.h``).

This is the only compute path of the package: there is no CPU fallback.  If the library is
missing, or no GPU is visible, every encode call raises :class:`NativeUnavailable` loudly.
The library is built in-tree by ``flac-raster_amd/csrc/Makefile`` (``__graft_entry__.build()``).
"""

from __future__ import annotations

import ctypes as C
import os
import threading
import time
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

import numpy as np

# FRA_LIB_PATH: load another build of the library (same-box A/B experiments, tools/gpu_ab.sh)
_LIB_PATH = Path(os.environ.get("FRA_LIB_PATH") or Path(__file__).resolve().parent / "_lib" / "libflac_raster_amd.so")
_lib = None
_lock = threading.RLock()  # re-entrant: __del__ (cyclic GC) may run while this thread holds it

DTYPE_CODES = {
    np.dtype(np.uint8): 0, np.dtype(np.int8): 1, np.dtype(np.uint16): 2, np.dtype(np.int16): 3,
    np.dtype(np.uint32): 4, np.dtype(np.int32): 5, np.dtype(np.float32): 6, np.dtype(np.float64): 7,
}


class NativeUnavailable(RuntimeError):
    """The HIP extension is not built or no MI355X (gfx950) device is visible."""


class NativeError(RuntimeError):
    pass


class OutputTooSmall(NativeError):
    def __init__(self, needed: int):
        super().__init__(f"output buffer too small: {needed} bytes needed")
        self.needed = needed


class Window(C.Structure):
    _fields_ = [("row_off", C.c_int32), ("col_off", C.c_int32), ("height", C.c_int32), ("width", C.c_int32)]


class Job(C.Structure):
    _fields_ = [
        ("raster", C.c_void_p), ("raster_on_device", C.c_int32), ("dtype", C.c_int32), ("channels", C.c_int32),
        ("band_stride", C.c_int64), ("row_stride", C.c_int64), ("col_stride", C.c_int64),
        ("windows", C.POINTER(Window)), ("nwindows", C.c_int32), ("level", C.c_int32), ("blocksize", C.c_int32),
        ("norm", C.c_int32), ("sample_rate", C.c_int32), ("first_frame", C.c_int32),
    ]


class StreamInfo(C.Structure):
    _fields_ = [
        ("offset", C.c_uint64), ("frame_bytes", C.c_uint64), ("data_min", C.c_double), ("data_max", C.c_double),
        ("sample_rate", C.c_int32), ("bps", C.c_int32), ("channels", C.c_int32), ("nframes", C.c_int32),
    ]


class Decoded(C.Structure):
    _fields_ = [
        ("sample_rate", C.c_int32), ("channels", C.c_int32), ("bps", C.c_int32), ("blocksize", C.c_int32),
        ("nframes", C.c_int64), ("nsamples", C.c_uint64), ("nstreams", C.c_int32), ("audio_offset", C.c_uint64),
    ]


DECODE_CONCAT = 1
E_SPACE = -6


class TiffChunk(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("bytes", C.c_uint64), ("row0", C.c_int32), ("col0", C.c_int32),
                ("rows", C.c_int32), ("cols", C.c_int32), ("plane", C.c_int32), ("pad", C.c_int32)]


class TiffLayout(C.Structure):
    _fields_ = [("compression", C.c_int32), ("predictor", C.c_int32), ("bytes_per_sample", C.c_int32),
                ("samples_per_pixel", C.c_int32), ("is_float", C.c_int32), ("big_endian", C.c_int32),
                ("bands", C.c_int32), ("win_row", C.c_int32), ("win_col", C.c_int32), ("win_h", C.c_int32),
                ("win_w", C.c_int32), ("pad", C.c_int32), ("dst_band_stride", C.c_int64),
                ("dst_row_stride", C.c_int64)]

EXPORTS = [
    "fra_last_error", "fra_abi_version", "fra_device_count", "fra_free", "fra_ctx_create", "fra_ctx_destroy",
    "fra_plan_create", "fra_plan_set_raster", "fra_plan_execute", "fra_plan_sync", "fra_plan_result",
    "fra_plan_download", "fra_plan_device_output", "fra_plan_enable_timing", "fra_plan_timing",
    "fra_plan_destroy", "fra_encode", "fra_stream_header", "fra_synth_raster", "fra_device_alloc",
    "fra_device_free", "fra_memcpy_d2h", "fra_memcpy_h2d", "fra_plan_frame_offsets", "fra_normalize",
    "fra_decode", "fra_plan_encode_host", "fra_plan_capacity", "fra_host_alloc", "fra_host_free",
    "fra_host_register", "fra_host_unregister", "fra_tiff_decode", "fra_plan_set_first_frame",
    "fra_plan_flags", "fra_plan_encode_host_progress", "fra_tiff_compress_bound", "fra_tiff_compress",
    "fra_plan_encode_ring", "fra_plan_host_band_rows", "fra_plan_create_ranged",
]


def library_path() -> Path:
    return _LIB_PATH


def load():
    """Load the shared library (no GPU needed just to load it)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not _LIB_PATH.exists():
            raise NativeUnavailable(
                f"{_LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
                "(make -C flac-raster_amd/csrc)")
        L = C.CDLL(str(_LIB_PATH))
        vp, i32, u64 = C.c_void_p, C.c_int32, C.c_uint64
        L.fra_last_error.restype = C.c_char_p
        L.fra_abi_version.restype = C.c_int
        L.fra_device_count.argtypes = [C.POINTER(C.c_int)]
        L.fra_free.argtypes = [vp]
        L.fra_ctx_create.argtypes = [C.c_int, C.POINTER(vp)]
        L.fra_ctx_destroy.argtypes = [vp]
        L.fra_plan_create.argtypes = [vp, C.POINTER(Job), C.POINTER(vp)]
        L.fra_plan_set_raster.argtypes = [vp, vp, i32]
        L.fra_plan_execute.argtypes = [vp]
        L.fra_plan_sync.argtypes = [vp]
        L.fra_plan_result.argtypes = [vp, C.POINTER(StreamInfo), C.POINTER(u64)]
        L.fra_plan_download.argtypes = [vp, vp, u64]
        L.fra_plan_device_output.argtypes = [vp, C.POINTER(vp), C.POINTER(u64)]
        L.fra_plan_enable_timing.argtypes = [vp, i32]
        L.fra_plan_timing.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(i32)]
        L.fra_plan_destroy.argtypes = [vp]
        L.fra_encode.argtypes = [C.c_int, C.POINTER(Job), C.POINTER(vp), C.POINTER(u64), C.POINTER(StreamInfo)]
        L.fra_stream_header.argtypes = [vp, i32, i32, i32, i32]
        L.fra_synth_raster.argtypes = [vp, i32, u64, i32, i32, i32, vp]
        L.fra_device_alloc.argtypes = [vp, u64, C.POINTER(vp)]
        L.fra_device_free.argtypes = [vp, vp]
        L.fra_memcpy_d2h.argtypes = [vp, vp, vp, u64]
        L.fra_memcpy_h2d.argtypes = [vp, vp, vp, u64]
        L.fra_plan_frame_offsets.argtypes = [vp, C.POINTER(u64), u64]
        pd = C.POINTER(C.c_double)
        L.fra_normalize.argtypes = [vp, vp, i32, i32, u64, i32, pd, pd, vp, pd, pd]
        L.fra_decode.argtypes = [vp, u64, i32, C.POINTER(Decoded), C.POINTER(C.POINTER(C.c_int32))]
        L.fra_plan_encode_host.argtypes = [vp, vp, vp, u64, C.POINTER(u64)]
        L.fra_plan_capacity.argtypes = [vp, C.POINTER(u64), C.POINTER(i32)]
        L.fra_plan_set_first_frame.argtypes = [vp, i32]
        L.fra_plan_flags.argtypes = [vp, C.POINTER(i32)]
        L.fra_host_alloc.argtypes = [u64, C.POINTER(vp)]
        L.fra_host_free.argtypes = [vp]
        L.fra_host_register.argtypes = [vp, u64]
        L.fra_host_unregister.argtypes = [vp]
        L.fra_tiff_decode.argtypes = [vp, u64, C.POINTER(TiffLayout), C.POINTER(TiffChunk), i32, vp, i32]
        L.fra_plan_encode_host_progress.argtypes = [vp, vp, vp, u64, C.POINTER(u64), vp]
        if hasattr(L, "fra_plan_create_ranged"):  # (r05; older builds load for same-box A/Bs)
            L.fra_plan_create_ranged.argtypes = [vp, C.POINTER(Job), C.POINTER(C.c_int32), C.POINTER(vp)]
        if hasattr(L, "fra_plan_encode_ring"):
            L.fra_plan_encode_ring.argtypes = [vp, vp, C.c_int64, vp, u64, C.POINTER(u64), vp, vp]
            L.fra_plan_host_band_rows.argtypes = [vp, C.POINTER(C.c_int64)]
        L.fra_tiff_compress_bound.argtypes = [i32, u64]
        L.fra_tiff_compress_bound.restype = u64
        L.fra_tiff_compress.argtypes = [i32, i32, vp, u64, i32, vp, u64, C.POINTER(u64), i32]
        _lib = L
        return L


def _check(rc: int):
    if rc != 0:
        msg = load().fra_last_error()
        raise NativeError(f"flac_raster_amd error {rc}: {msg.decode() if msg else ''}")


def device_count() -> int:
    n = C.c_int(0)
    load().fra_device_count(C.byref(n))
    return n.value


def stream_header(channels: int, bps: int, sample_rate: int, blocksize: int = 4096) -> bytes:
    buf = (C.c_uint8 * 86)()
    _check(load().fra_stream_header(buf, channels, bps, sample_rate, blocksize))
    return bytes(buf)


_PIN_POOL_BYTES = int(os.environ.get("FRA_PINNED_POOL_MB", "8192")) << 20
_pin_pool: List[Tuple[int, int]] = []  # (capacity, ptr) of released page-locked blocks kept for reuse
_pin_lock = threading.RLock()  # re-entrant, as _lock


class _PinnedBlock:
    """Owner of one page-locked host allocation (``fra_host_alloc``), exposed to numpy.  Released blocks
    go to a small pool (``FRA_PINNED_POOL_MB``, default 8 GiB) because pinning pages costs far more than
    copying through them; the pool reuses a block of at most twice the requested size."""

    def __init__(self, nbytes: int):
        nbytes = max(1, int(nbytes))
        ptr, cap = None, 0
        with _pin_lock:
            best = None
            for k, (c, p) in enumerate(_pin_pool):
                if nbytes <= c <= 2 * nbytes and (best is None or c < _pin_pool[best][0]):
                    best = k
            if best is not None:
                cap, ptr = _pin_pool.pop(best)
        if ptr is None:
            p = C.c_void_p()
            _check(load().fra_host_alloc(nbytes, C.byref(p)))
            ptr, cap = p.value, nbytes
        self.ptr = ptr
        self.capacity = cap
        self.nbytes = nbytes
        self.__array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (self.ptr, False), "version": 3}

    def __del__(self):
        try:
            if not self.ptr:
                return
            ptr, self.ptr = self.ptr, None
            with _pin_lock:
                pooled = sum(c for c, _ in _pin_pool)
                if pooled + self.capacity <= _PIN_POOL_BYTES:
                    _pin_pool.append((self.capacity, ptr))
                    return
            load().fra_host_free(C.c_void_p(ptr))
        except Exception:
            pass


def release_pinned_pool():
    """Free every pooled page-locked block."""
    with _pin_lock:
        blocks = list(_pin_pool)
        _pin_pool.clear()
    for _, p in blocks:
        load().fra_host_free(C.c_void_p(p))


def pinned_empty(shape, dtype) -> np.ndarray:
    """``np.empty`` in page-locked host memory (full-rate PCIe DMA; freed with the array).  Needs the
    HIP runtime (a GPU box); raises :class:`NativeError` without one."""
    dt = np.dtype(dtype)
    shape = (shape,) if isinstance(shape, int) else tuple(shape)
    n = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
    return np.asarray(_PinnedBlock(n)).view(dt)[: n // dt.itemsize].reshape(shape)


def is_pinned(a: np.ndarray) -> bool:
    base = a
    while base is not None and not isinstance(base, _PinnedBlock):
        base = getattr(base, "base", None)
    return base is not None


class HostRegistration:
    """``hipHostRegister`` of an existing host array for the lifetime of a ``with`` block."""

    def __init__(self, a: np.ndarray):
        self.a = a
        self.ok = False

    def __enter__(self):
        if self.a.nbytes and not is_pinned(self.a):
            _check(load().fra_host_register(C.c_void_p(self.a.ctypes.data), self.a.nbytes))
            self.ok = True
        return self.a

    def __exit__(self, *exc):
        if self.ok:
            load().fra_host_unregister(C.c_void_p(self.a.ctypes.data))
            self.ok = False


class Context:
    """One HIP device + stream (``fra_ctx``)."""

    def __init__(self, device: int = 0):
        L = load()
        if device_count() == 0:
            raise NativeUnavailable("no HIP device visible: the flac_raster encoder requires an MI355X (gfx950)")
        h = C.c_void_p()
        _check(L.fra_ctx_create(device, C.byref(h)))
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            load().fra_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def alloc(self, nbytes: int) -> int:
        p = C.c_void_p()
        _check(load().fra_device_alloc(self.h, nbytes, C.byref(p)))
        return p.value

    def free(self, ptr: int):
        _check(load().fra_device_free(self.h, C.c_void_p(ptr)))

    def h2d(self, dev: int, arr: np.ndarray):
        a = np.ascontiguousarray(arr)
        _check(load().fra_memcpy_h2d(self.h, C.c_void_p(dev), a.ctypes.data_as(C.c_void_p), a.nbytes))

    def d2h(self, arr: np.ndarray, dev: int):
        _check(load().fra_memcpy_d2h(self.h, arr.ctypes.data_as(C.c_void_p), C.c_void_p(dev), arr.nbytes))

    def normalize(self, data: np.ndarray, bps: int, data_min=None, data_max=None):
        """normalize_to_audio on this context's GPU (fra_normalize).  Returns (audio, mn, mx)."""
        a = np.ascontiguousarray(data)
        if a.dtype not in DTYPE_CODES:
            raise TypeError(f"unsupported dtype {a.dtype}")
        out = np.empty(a.shape, dtype=np.int16 if bps == 16 else np.int32)
        mn, mx = C.c_double(), C.c_double()
        omin = C.byref(C.c_double(float(data_min))) if data_min is not None else None
        omax = C.byref(C.c_double(float(data_max))) if data_max is not None else None
        _check(load().fra_normalize(self.h, a.ctypes.data_as(C.c_void_p), 0, DTYPE_CODES[a.dtype], a.size, bps, omin,
                                    omax, out.ctypes.data_as(C.c_void_p), C.byref(mn), C.byref(mx)))
        return out, mn.value, mx.value

    def synth(self, kind: int, seed: int, bands: int, height: int, width: int, dev_out: int):
        _check(load().fra_synth_raster(self.h, kind, seed, bands, height, width, C.c_void_p(dev_out)))


class Plan:
    """Device workspace for one job (``fra_plan``): windows of one raster -> FLAC frame streams."""

    def __init__(self, ctx: Context, raster_ptr: Optional[int], on_device: bool, dtype: np.dtype, channels: int,
                 strides: Tuple[int, int, int], windows: Sequence[Tuple[int, int, int, int]], level: int = 5,
                 blocksize: int = 4096, norm: int = 16, sample_rate: int = 0, keepalive=None,
                 frame_ranges: Optional[Sequence[Tuple[int, int]]] = None):
        """``frame_ranges``: per window (first frame, count; count -1 = to the end) -- the plan encodes only
        those frames of each window's stream (``fra_plan_create_ranged``; normalisation over the whole
        window, frame numbers of the whole stream)."""
        L = load()
        self.ctx = ctx
        self.nwin = len(windows)
        self._wins = (Window * max(1, self.nwin))(*[Window(*w) for w in windows])
        self._keep = keepalive
        job = Job()
        job.raster = C.c_void_p(raster_ptr) if raster_ptr else None
        job.raster_on_device = 1 if on_device else 0
        job.dtype = DTYPE_CODES[np.dtype(dtype)]
        job.channels = channels
        job.band_stride, job.row_stride, job.col_stride = strides
        job.windows = self._wins
        job.nwindows = self.nwin
        job.level = level
        job.blocksize = blocksize
        job.norm = norm
        job.sample_rate = sample_rate
        h = C.c_void_p()
        if frame_ranges is None:
            _check(L.fra_plan_create(ctx.h, C.byref(job), C.byref(h)))
        else:
            if len(frame_ranges) != self.nwin:
                raise ValueError("one (first, count) frame range per window")
            self._ranges = (C.c_int32 * max(2, 2 * self.nwin))(*[int(v) for fr in frame_ranges for v in fr])
            _check(L.fra_plan_create_ranged(ctx.h, C.byref(job), self._ranges, C.byref(h)))
        self.h = h

    def set_raster(self, ptr: int, on_device: bool, keepalive=None):
        self._keep = keepalive
        _check(load().fra_plan_set_raster(self.h, C.c_void_p(ptr), 1 if on_device else 0))

    def execute(self):
        _check(load().fra_plan_execute(self.h))

    def sync(self):
        _check(load().fra_plan_sync(self.h))

    def result(self) -> Tuple[List[StreamInfo], int]:
        infos = (StreamInfo * max(1, self.nwin))()
        total = C.c_uint64()
        _check(load().fra_plan_result(self.h, infos, C.byref(total)))
        return list(infos)[: self.nwin], total.value

    def download(self) -> Tuple[List[StreamInfo], bytes]:
        infos, total = self.result()
        buf = np.empty(max(1, total), dtype=np.uint8)
        _check(load().fra_plan_download(self.h, buf.ctypes.data_as(C.c_void_p), total))
        return infos, buf[:total].tobytes()

    def set_first_frame(self, n: int):
        """FLAC frame number of every stream's first frame for the next execute (pyflac shim)."""
        _check(load().fra_plan_set_first_frame(self.h, int(n)))

    def flags(self) -> int:
        """``FRA_PLAN_*`` bits: 2 cross-execute pipelined, 4 full frames on the per-wave analysis kernel, 8 (with 4)
        its next execute keeps residuals up to 17 bits (else 16; picked per execute from an earlier one's count of
        waves that needed bit 16); 1, direct write, is never set since r03."""
        f = C.c_int32()
        _check(load().fra_plan_flags(self.h, C.byref(f)))
        return f.value

    def capacity(self) -> Tuple[int, int]:
        """(upper bound of the output bytes, number of host-pipeline row bands)."""
        cap, nb = C.c_uint64(), C.c_int32()
        _check(load().fra_plan_capacity(self.h, C.byref(cap), C.byref(nb)))
        return cap.value, nb.value

    def encode_host(self, raster: np.ndarray, out: np.ndarray) -> int:
        """Pipelined host raster -> host frames (``fra_plan_encode_host``): row bands of the raster go
        H2D while earlier bands are analysed, and each band's frames come back D2H as soon as they are
        assembled.  ``raster`` must have the plan's dtype/strides; ``out`` is a uint8 buffer (page-locked
        for full rate).  Returns the total frame bytes; raises :class:`OutputTooSmall` (with ``.needed``)
        if ``out`` is too small -- the frames then stay on the device (``download``)."""
        total = C.c_uint64()
        self._keep = raster
        rc = load().fra_plan_encode_host(self.h, C.c_void_p(raster.ctypes.data), C.c_void_p(out.ctypes.data),
                                         out.nbytes, C.byref(total))
        if rc == E_SPACE:
            raise OutputTooSmall(total.value)
        _check(rc)
        return total.value

    def encode_host_progress(self, raster: np.ndarray, out: np.ndarray, rows_ready: np.ndarray) -> int:
        """:meth:`encode_host` over a raster still being produced (``fra_plan_encode_host_progress``): a
        producer thread fills ``raster`` top to bottom and publishes the rows done in ``rows_ready[0]``
        (int64; -1 = failed); each row band's H2D copy waits for its rows."""
        if rows_ready.dtype != np.int64 or rows_ready.size < 1:
            raise ValueError("rows_ready must be an int64 array of >= 1 element")
        total = C.c_uint64()
        self._keep = raster
        rc = load().fra_plan_encode_host_progress(self.h, C.c_void_p(raster.ctypes.data),
                                                  C.c_void_p(out.ctypes.data), out.nbytes, C.byref(total),
                                                  C.c_void_p(rows_ready.ctypes.data))
        if rc == E_SPACE:
            raise OutputTooSmall(total.value)
        _check(rc)
        return total.value

    def host_band_rows(self) -> int:
        """Rows of the tallest host row band (``fra_plan_host_band_rows``)."""
        m = C.c_int64()
        _check(load().fra_plan_host_band_rows(self.h, C.byref(m)))
        return m.value

    def encode_ring(self, ring: np.ndarray, out: np.ndarray, rows_ready: np.ndarray, rows_done: np.ndarray) -> int:
        """:meth:`encode_host_progress` with bounded host memory (``fra_plan_encode_ring``): ``ring`` is
        ``(B, ring_rows, W)`` and holds image row r at ring row ``r % ring_rows``; the call publishes in
        ``rows_done[0]`` the rows whose H2D copy completed (the producer may then reuse their ring rows)."""
        for a in (rows_ready, rows_done):
            if a.dtype != np.int64 or a.size < 1:
                raise ValueError("rows_ready / rows_done must be int64 arrays of >= 1 element")
        total = C.c_uint64()
        self._keep = ring
        rc = load().fra_plan_encode_ring(self.h, C.c_void_p(ring.ctypes.data), ring.shape[1],
                                         C.c_void_p(out.ctypes.data), out.nbytes, C.byref(total),
                                         C.c_void_p(rows_ready.ctypes.data), C.c_void_p(rows_done.ctypes.data))
        if rc == E_SPACE:
            raise OutputTooSmall(total.value)
        _check(rc)
        return total.value

    def frame_offsets(self, nframes: int) -> np.ndarray:
        """Byte offset of every frame in the concatenated output (+ total at the end)."""
        off = np.empty(nframes + 1, dtype=np.uint64)
        _check(load().fra_plan_frame_offsets(self.h, off.ctypes.data_as(C.POINTER(C.c_uint64)), nframes + 1))
        return off

    def device_output(self) -> Tuple[int, int]:
        p, cap = C.c_void_p(), C.c_uint64()
        _check(load().fra_plan_device_output(self.h, C.byref(p), C.byref(cap)))
        return p.value, cap.value

    def enable_timing(self, on: bool = True):
        _check(load().fra_plan_enable_timing(self.h, 1 if on else 0))

    def timing(self) -> Tuple[List[float], int]:
        ms = (C.c_float * 4)()
        n = C.c_int32()
        _check(load().fra_plan_timing(self.h, ms, C.byref(n)))
        return list(ms), n.value

    def close(self):
        if getattr(self, "h", None):
            load().fra_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = {}

# Process-wide pool of idle plans keyed by job shape: the reference creates one encoder per tile
# (spatial_encoder.py:291-304), and tiles of one raster share a few shapes, so a released plan (with its
# page-locked output buffer) is handed to the next encoder of the same shape instead of rebuilding the
# device workspace (~20 ms of allocations and table uploads).  Plans are used by one owner at a time.
_PLAN_POOL_MAX = int(os.environ.get("FRA_PLAN_POOL", "16"))
_plan_pool: "dict" = {}
_plan_pool_n = 0


def acquire_plan(key, factory):
    """An idle pooled plan entry for ``key`` or a new one from ``factory()``; the caller owns it until
    :func:`release_plan`."""
    global _plan_pool_n
    with _lock:
        lst = _plan_pool.get(key)
        if lst:
            _plan_pool_n -= 1
            return lst.pop()
    return factory()


def release_plan(key, entry):
    """Return a plan entry ``(plan, ...)`` to the pool (closed instead when the pool is full)."""
    global _plan_pool_n
    with _lock:
        if _plan_pool_n < _PLAN_POOL_MAX:
            _plan_pool.setdefault(key, []).append(entry)
            _plan_pool_n += 1
            return
    entry[0].close()


def default_context(device: int = 0) -> Context:
    with _lock:
        ctx = _default_ctx.get(device)
    if ctx is None:
        ctx = Context(device)
        with _lock:
            _default_ctx[device] = ctx
    return ctx


def _element_strides(a: np.ndarray) -> Tuple[int, int, int]:
    es = a.dtype.itemsize
    if any(st < 0 or st % es for st in a.strides):
        raise ValueError("raster strides must be non-negative multiples of the item size")
    return tuple(st // es for st in a.strides)


def encode_windows_buffer(raster: np.ndarray, windows, level: int = 5, blocksize: int = 4096, norm: int = 16,
                          sample_rate: int = 0, device: int = 0, pinned: bool = True,
                          rows_ready: Optional[np.ndarray] = None, frame_ranges=None):
    """Encode windows of a band-planar host raster ``(B, H, W)`` (any non-negative strides, e.g. a row
    band view of a larger raster) through the pipelined host path (``fra_plan_encode_host``).

    Returns ``(infos, frames)``: ``frames`` is a uint8 array (page-locked unless ``pinned=False``) with
    every window's FLAC frames concatenated in window order; ``infos[i].offset/.frame_bytes`` slice it.
    ``rows_ready``: the raster is still being filled by a producer thread that publishes the rows done
    in ``rows_ready[0]`` (``fra_plan_encode_host_progress``).  ``frame_ranges``: (first frame, count) per
    window (``fra_plan_create_ranged``).
    """
    a = np.asarray(raster)
    if a.ndim == 2:
        a = a[None]
    if a.dtype not in DTYPE_CODES:
        raise TypeError(f"unsupported dtype {a.dtype}")
    if not a.dtype.isnative:
        a = a.astype(a.dtype.newbyteorder("="))
    B = a.shape[0]
    ctx = default_context(device)
    plan = Plan(ctx, None, False, a.dtype, B, _element_strides(a), windows, level, blocksize, norm, sample_rate,
                frame_ranges=frame_ranges)
    try:
        cap, _ = plan.capacity()
        out = pinned_empty(cap, np.uint8) if pinned else np.empty(cap, np.uint8)
        total = plan.encode_host(a, out) if rows_ready is None else plan.encode_host_progress(a, out, rows_ready)
        infos, _ = plan.result()
        return infos, out[:total]
    finally:
        plan.close()


def ring_rows_for(band_rows: int, step: int, height: int) -> int:
    """Ring height for :func:`encode_windows_ring`: two host bands + one producer step (so the producer
    decodes band b+1 while band b is copied; band + step is the minimum that cannot deadlock), in whole
    producer steps, capped at the raster height."""
    step = max(1, step)
    rows = -(-(2 * band_rows + step) // step) * step
    return int(min(height, rows))


def encode_windows_ring(shape, dtype, windows, fill, level: int = 5, blocksize: int = 4096, norm: int = 16,
                        sample_rate: int = 0, device: int = 0, step: int = 0, ring_rows: int = 0):
    """Encode windows of a band-planar raster of ``shape`` ``(B, H, W)`` that never exists whole in host
    memory (``fra_plan_encode_ring``): a producer thread calls ``fill(dst, r0, r1)`` to write image rows
    ``[r0, r1)`` of every band into ``dst`` (a ``(B, r1 - r0, W)`` view of a page-locked ring), in steps of
    ``step`` rows (default: the tallest host band), top to bottom; each step waits until the encoder's H2D
    copies have released its ring rows.  Host memory: the ring (``ring_rows`` rows, default
    :func:`ring_rows_for`) + the frames (a lazily committed buffer: only the written bytes are resident).

    Returns ``(infos, frames, ring_rows)`` as :func:`encode_windows_buffer` (``frames`` not page-locked)."""
    B, H, W = shape
    dt = np.dtype(dtype)
    if dt not in DTYPE_CODES:
        raise TypeError(f"unsupported dtype {dt}")
    ctx = default_context(device)
    plan = Plan(ctx, None, False, dt, B, (H * W, W, 1), windows, level, blocksize, norm, sample_rate)
    th = None
    rows_ready = np.zeros(1, np.int64)
    rows_done = np.zeros(1, np.int64)
    stop = []
    try:
        band = max(1, plan.host_band_rows())
        step = int(step) if step and step > 0 else band
        R = int(ring_rows) if ring_rows else ring_rows_for(band, step, H)
        if R < min(H, band + step):
            raise ValueError(f"ring of {R} rows < band {band} + step {step}")
        ring = pinned_empty((B, R, W), dt)
        cap, _ = plan.capacity()
        out = np.empty(cap, np.uint8)  # pages are committed as the frames land
        errors: list = []

        def produce():
            try:
                r0 = 0
                while r0 < H:
                    r1 = min(H, r0 + step)
                    while rows_done[0] < r1 - R:  # the encoder still copies these ring rows
                        if stop:
                            return
                        time.sleep(0.0002)
                    r = r0
                    while r < r1:  # split where the ring wraps
                        rr = r % R
                        n = min(r1 - r, R - rr)
                        fill(ring[:, rr:rr + n, :], r, r + n)
                        r += n
                    rows_ready[0] = r1
                    r0 = r1
            except BaseException as e:  # reported to the encoder (rows_ready = -1), re-raised below
                errors.append(e)
                rows_ready[0] = -1

        th = threading.Thread(target=produce, name="ring-producer", daemon=True)
        th.start()
        try:
            total = plan.encode_ring(ring, out, rows_ready, rows_done)
        except BaseException:
            stop.append(1)
            th.join()
            if errors:
                raise errors[0]
            raise
        th.join()
        if errors:
            raise errors[0]
        infos, _ = plan.result()
        return infos, out[:total], R
    finally:
        plan.close()


def encode_windows(raster: np.ndarray, windows, level: int = 5, blocksize: int = 4096, norm: int = 16,
                   sample_rate: int = 0, device: int = 0, path: str = "host"):
    """Encode windows of a band-planar host raster ``(B, H, W)`` (or ``(H, W)``).

    Returns ``(infos, frames_bytes)``: ``frames_bytes`` holds every window's FLAC frames
    concatenated in window order; ``infos[i].offset/.frame_bytes`` slice it.  ``path="host"`` is the
    pipelined host path (``fra_plan_encode_host``); ``path="device"`` copies the whole raster first and
    runs ``fra_plan_execute`` (frame groups per ``FRA_GROUPS``) then ``fra_plan_download``.
    """
    if path == "host":
        infos, buf = encode_windows_buffer(raster, windows, level, blocksize, norm, sample_rate, device)
        return infos, buf.tobytes()
    a = np.ascontiguousarray(raster)
    if a.ndim == 2:
        a = a[None]
    B, H, W = a.shape
    ctx = default_context(device)
    plan = Plan(ctx, a.ctypes.data, False, a.dtype, B, (H * W, W, 1), windows, level, blocksize, norm,
                sample_rate, keepalive=a)
    try:
        plan.execute()
        plan.sync()
        return plan.download()
    finally:
        plan.close()


def encode_interleaved(samples: np.ndarray, sample_rate: int, level: int = 5, blocksize: int = 4096,
                       device: int = 0, return_offsets: bool = False):
    """pyflac ``StreamEncoder.process(samples); finish()`` semantics: samples (N, C) int16/int32
    already in the audio domain; bps = itemsize*8.  Returns (info, frames) or, with
    ``return_offsets``, (info, frames, per-frame byte offsets + total)."""
    s = np.asarray(samples)
    if s.ndim == 1:
        s = s.reshape(-1, 1)
    if s.dtype not in (np.int16, np.int32):
        s = s.astype(np.int32)
    s = np.ascontiguousarray(s)
    N, Ch = s.shape
    ctx = default_context(device)
    # treat the (N, C) array as one raster row of N pixels with C interleaved bands
    plan = Plan(ctx, s.ctypes.data, False, s.dtype, Ch, (1, N * Ch, Ch), [(0, 0, 1, N)] if N else [(0, 0, 0, 0)],
                level, blocksize, 0, sample_rate, keepalive=s)
    try:
        plan.execute()
        plan.sync()
        infos, data = plan.download()
        if return_offsets:
            return infos[0], data, plan.frame_offsets(infos[0].nframes)
        return infos[0], data
    finally:
        plan.close()

def decode(data: bytes, concat: bool = False) -> Tuple[np.ndarray, Decoded]:
    """Native FLAC decode (fra_decode; host code, no GPU needed).  Returns ((N, C) int32, info)."""
    L = load()
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    info = Decoded()
    ptr = C.POINTER(C.c_int32)()
    _check(L.fra_decode(buf.ctypes.data_as(C.c_void_p), len(data), DECODE_CONCAT if concat else 0, C.byref(info),
                        C.byref(ptr)))
    try:
        n = info.nsamples * info.channels
        out = np.ctypeslib.as_array(ptr, shape=(max(1, n),))[:n].copy() if n else np.zeros(0, np.int32)
    finally:
        L.fra_free(ptr)
    return out.reshape(-1, info.channels), info


def tiff_compress(compression: int, chunks: np.ndarray, level: int = 6, threads: int = 0):
    """Compress equal-size raw TIFF chunks (``chunks``: uint8 array (nchunks, chunk_bytes), file layout,
    predictor already applied) with LZW (5) or deflate (8) on the native thread pool
    (``fra_tiff_compress``).  Returns a list of ``bytes``, one per chunk."""
    chunks = np.ascontiguousarray(chunks, dtype=np.uint8)
    n, cb = chunks.shape
    L = load()
    stride = int(L.fra_tiff_compress_bound(int(compression), int(cb)))
    dst = np.empty(max(1, n) * stride, np.uint8)
    sizes = np.zeros(max(1, n), np.uint64)
    _check(L.fra_tiff_compress(int(compression), int(level), C.c_void_p(chunks.ctypes.data), int(cb), int(n),
                               C.c_void_p(dst.ctypes.data), stride, sizes.ctypes.data_as(C.POINTER(C.c_uint64)),
                               int(threads)))
    return [dst[i * stride:i * stride + int(sizes[i])].tobytes() for i in range(n)]
