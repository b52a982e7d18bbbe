"""ctypes wrapper around oracle/libfr_oracle.so -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / CPU baseline.  The product package
(``flac-raster_amd/flac_raster``) never imports it and has no CPU fallback.

See ``oracle/fr_oracle.c`` for what is restated from the reference and where parity is
pinned (decode of the libFLAC golden ``sample_rgb.flac``; normalisation fixtures generated
from the reference's ``normalization.py`` by ``tests/golden/make_golden.py``).
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB = None

DTYPE_CODES = {
    np.dtype(np.uint8): 0,
    np.dtype(np.int8): 1,
    np.dtype(np.uint16): 2,
    np.dtype(np.int16): 3,
    np.dtype(np.uint32): 4,
    np.dtype(np.int32): 5,
    np.dtype(np.float32): 6,
    np.dtype(np.float64): 7,
}


def build() -> Path:
    """Compile the oracle with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _HERE / "libfr_oracle.so"


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    so = _HERE / "libfr_oracle.so"
    src = _HERE / "fr_oracle.c"
    if not so.exists() or (src.exists() and src.stat().st_mtime > so.stat().st_mtime):
        build()
    L = C.CDLL(str(so))
    p = C.c_void_p
    L.ora_minmax.argtypes = [p, C.c_int, C.c_size_t, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.ora_minmax.restype = C.c_int64
    L.ora_normalize.argtypes = [p, C.c_int, C.c_size_t, C.c_int, C.c_double, C.c_double, p]
    L.ora_crc8.argtypes = [p, C.c_size_t]
    L.ora_crc8.restype = C.c_uint
    L.ora_crc16.argtypes = [p, C.c_size_t]
    L.ora_crc16.restype = C.c_uint
    L.ora_encode.argtypes = [p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                             C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_size_t), p, p]
    L.ora_decode.argtypes = [p, C.c_size_t, C.POINTER(C.POINTER(C.c_int32)), C.POINTER(C.c_int64),
                             C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int64)]
    L.ora_free.argtypes = [p]
    L.ora_stream_header.argtypes = [p, C.c_int, C.c_int, C.c_int, C.c_int]
    L.ora_stream_header.restype = C.c_size_t
    L.ora_window_tukey.argtypes = [p, C.c_int, C.c_double]
    L.ora_window_set.argtypes = [p, C.c_int, C.c_int]
    L.ora_num_windows.argtypes = [C.c_int]
    L.ora_autocorr.argtypes = [p, C.c_int, C.c_int, p]
    L.ora_autocorr_int.argtypes = [p, C.c_int, C.c_int, p]
    L.ora_levinson.argtypes = [p, C.c_int, p, p]
    L.ora_quantize.argtypes = [p, C.c_int, C.c_int, p, C.POINTER(C.c_int)]
    L.ora_det_log2.argtypes = [C.c_double]
    L.ora_det_log2.restype = C.c_double
    L.ora_sample_rate_for_pixels.argtypes = [C.c_int64]
    L.ora_set_stereo.argtypes = [C.c_int]
    L.ora_set_lpc_keep.argtypes = [C.c_int]
    _LIB = L
    return L


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def minmax(data: np.ndarray):
    a = np.ascontiguousarray(data)
    mn, mx = C.c_double(), C.c_double()
    lib().ora_minmax(_ptr(a), DTYPE_CODES[a.dtype], a.size, C.byref(mn), C.byref(mx))
    return mn.value, mx.value


def normalize(data: np.ndarray, bps: int, mn=None, mx=None):
    """normalize_to_audio restated (normalization.py:126-202); returns (audio, mn, mx)."""
    a = np.ascontiguousarray(data)
    if mn is None or mx is None:
        m0, m1 = minmax(a)
        mn = m0 if mn is None else mn
        mx = m1 if mx is None else mx
    out = np.empty(a.shape, dtype=np.int16 if bps == 16 else np.int32)
    lib().ora_normalize(_ptr(a), DTYPE_CODES[a.dtype], a.size, bps, float(mn), float(mx), _ptr(out))
    return out, mn, mx


def sample_rate_for_pixels(px: int) -> int:
    return lib().ora_sample_rate_for_pixels(int(px))


def crc8(b: bytes) -> int:
    a = np.frombuffer(b, dtype=np.uint8)
    return lib().ora_crc8(_ptr(a), a.size)


def crc16(b: bytes) -> int:
    a = np.frombuffer(b, dtype=np.uint8)
    return lib().ora_crc16(_ptr(a), a.size)


def set_stereo(enable: bool):
    """FRA-1 3.1b mid-side stereo on/off (test hook: report the size gain over independent channels)."""
    lib().ora_set_stereo(1 if enable else 0)


def set_lpc_keep(k: int):
    """FRA-1 3.7b override (test hook): -1 = the level table's rule, 0 = evaluate every LPC window, k = k."""
    lib().ora_set_lpc_keep(int(k))


def encode(samples: np.ndarray, sample_rate: int, level: int = 5, blocksize: int = 4096,
           with_header: bool = True, bps: int | None = None, return_info: bool = False):
    """Encode interleaved samples (N, C) int16/int32 -> FLAC bytes (pyflac semantics, F3:
    bps = itemsize*8 unless given)."""
    s = np.asarray(samples)
    if s.ndim == 1:
        s = s.reshape(-1, 1)
    if bps is None:
        bps = s.dtype.itemsize * 8
    x = np.ascontiguousarray(s.astype(np.int32))
    N, Ch = x.shape
    out = C.POINTER(C.c_uint8)()
    n = C.c_size_t()
    nfr = (N + blocksize - 1) // blocksize
    fb = np.zeros(max(nfr, 1), dtype=np.int64)
    info = np.zeros((max(nfr, 1), Ch, 4), dtype=np.int32)
    rc = lib().ora_encode(_ptr(x), N, Ch, bps, sample_rate, blocksize, level, int(with_header),
                          C.byref(out), C.byref(n), _ptr(fb), _ptr(info))
    if rc != 0:
        raise ValueError(f"ora_encode failed rc={rc}")
    data = C.string_at(out, n.value)
    lib().ora_free(out)
    if return_info:
        return data, fb[:nfr], info[:nfr]
    return data


def decode(flac: bytes):
    """Decode -> (samples (N,C) int32, sample_rate, bps, nframes).  Raises on CRC/format error."""
    a = np.frombuffer(flac, dtype=np.uint8)
    out = C.POINTER(C.c_int32)()
    N = C.c_int64()
    ch, bps, sr, nf = C.c_int(), C.c_int(), C.c_int(), C.c_int64()
    rc = lib().ora_decode(_ptr(a), a.size, C.byref(out), C.byref(N), C.byref(ch), C.byref(bps),
                          C.byref(sr), C.byref(nf))
    if rc != 0:
        raise ValueError(f"ora_decode failed rc={rc}")
    arr = np.ctypeslib.as_array(out, shape=(N.value * ch.value,)).copy() if N.value else np.zeros(0, np.int32)
    lib().ora_free(out)
    return arr.reshape(-1, ch.value), sr.value, bps.value, nf.value


def stream_header(channels: int, bps: int, sample_rate: int, blocksize: int = 4096) -> bytes:
    buf = np.zeros(128, dtype=np.uint8)
    n = lib().ora_stream_header(_ptr(buf), channels, bps, sample_rate, blocksize)
    return buf[:n].tobytes()


def window_set(n: int, nsub: int) -> np.ndarray:
    nw = lib().ora_num_windows(nsub)
    w = np.zeros((max(nw, 1), n), dtype=np.float32)
    lib().ora_window_set(_ptr(w), n, nsub)
    return w[:nw]


def autocorr(wf: np.ndarray, maxlag: int) -> np.ndarray:
    a = np.ascontiguousarray(wf, dtype=np.float32)
    out = np.zeros(maxlag + 1, dtype=np.float64)
    lib().ora_autocorr(_ptr(a), a.size, maxlag, _ptr(out))
    return out


def autocorr_int(v: np.ndarray, maxlag: int) -> np.ndarray:
    """FRA-1 3.5b: exact autocorrelation of integer windowed samples (streams of <= 16 bps)."""
    a = np.ascontiguousarray(v, dtype=np.int32)
    out = np.zeros(maxlag + 1, dtype=np.float64)
    lib().ora_autocorr_int(_ptr(a), a.size, maxlag, _ptr(out))
    return out


def levinson(autoc: np.ndarray, max_order: int):
    a = np.ascontiguousarray(autoc, dtype=np.float64)
    lp = np.zeros((max_order, 32), dtype=np.float64)
    err = np.zeros(max_order, dtype=np.float64)
    n = lib().ora_levinson(_ptr(a), max_order, _ptr(lp), _ptr(err))
    return lp, err, n


def quantize(lp: np.ndarray, order: int, precision: int):
    a = np.ascontiguousarray(lp, dtype=np.float64)
    q = np.zeros(32, dtype=np.int32)
    sh = C.c_int()
    rc = lib().ora_quantize(_ptr(a), order, precision, _ptr(q), C.byref(sh))
    return (q[:order], sh.value) if rc == 0 else None


def frame_bytes_total(flac: bytes, header_len: int = 86) -> int:
    return len(flac) - header_len
