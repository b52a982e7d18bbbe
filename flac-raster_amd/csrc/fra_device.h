// fra_device.h -- device helpers shared by the encode kernels (fra_analyze.hip, fra_kernels.hip).
//
// Every floating-point helper on the decision path evaluates exactly the op sequence of its
// oracle counterpart in oracle/fr_oracle.c (compile with -ffp-contract=off; IEEE add/mul/div/fma
// are correctly rounded on gfx950 and x86-64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "fra_internal.h"

#pragma clang fp contract(off)

namespace fra {

#ifndef FRA_LOAD_STAMP
#define FRA_LOAD_STAMP(k, dep)  // diagnostic hook (fra_analyze.hip, FRA_STAMPS_FINE builds only)
#endif

// ---------------------------------------------------------------- ordered keys for nanmin/nanmax
__device__ __forceinline__ unsigned long long okey(double v) {
  unsigned long long b = (unsigned long long)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double unkey(unsigned long long k) {
  unsigned long long b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double((long long)b);
}

// ---------------------------------------------------------------- typed loads
template <int SRC>
__device__ __forceinline__ double load_f64(const void* base, int64_t e) {
  if constexpr (SRC == ST_U8) return (double)((const uint8_t*)base)[e];
  else if constexpr (SRC == ST_I8) return (double)((const int8_t*)base)[e];
  else if constexpr (SRC == ST_U16) return (double)((const uint16_t*)base)[e];
  else if constexpr (SRC == ST_I16) return (double)((const int16_t*)base)[e];
  else if constexpr (SRC == ST_U32) return (double)((const uint32_t*)base)[e];
  else if constexpr (SRC == ST_I32) return (double)((const int32_t*)base)[e];
  else if constexpr (SRC == ST_F32) return (double)((const float*)base)[e];
  else return ((const double*)base)[e];
}
template <int SRC>
__device__ __forceinline__ int32_t load_raw_int(const void* base, int64_t e) {
  if constexpr (SRC == ST_I16) return (int32_t)((const int16_t*)base)[e];
  else if constexpr (SRC == ST_I32) return ((const int32_t*)base)[e];
  else return 0;  // norm == 0 is only accepted for int16/int32 samples (fra_plan_create)
}

// ---------------------------------------------------------------- normalize_to_audio
struct NormParams {
  double mn, range, rcp, scale;
  bool to16;
  int mode;  // 0 raw ints, else normalise
};
__device__ __forceinline__ NormParams norm_params(int norm, const NormDev& nd) {
  NormParams p;
  p.mode = norm;
  p.to16 = norm == 16;
  p.scale = norm == 16 ? 32767.0 : 8388607.0;
  double mn, mx;
  if (nd.mnkey == ~0ull) {  // no non-NaN value: nanmin/nanmax -> NaN
    mn = __longlong_as_double(0x7FF8000000000000ll);
    mx = mn;
  } else {
    mn = unkey(nd.mnkey);
    mx = unkey(nd.mxkey);
  }
  p.mn = mn;
  p.range = (mx <= mn) ? 1.0 : (mx - mn);  // normalization.py:154-159
  p.rcp = 1.0 / p.range;
  return p;
}
__device__ __forceinline__ NormParams norm_params(const StreamDev& st, const NormDev& nd) { return norm_params(st.norm, nd); }
// t/range for the integer dtypes by Markstein's reciprocal refinement: bit-identical to the IEEE
// quotient for every t = 2*(x-mn) in [0, 2R], R integer (exhaustively verified for R < 2^16 by
// tools/verify_markstein.c; theorem-backed for 32-bit integers: no under/overflow is possible).
__device__ __forceinline__ double div_markstein(double t, double b, double y) {
  const double q0 = t * y;
  const double r = fma(-q0, b, t);
  return fma(r, y, q0);
}
// normalization.py:162-187, op order as numpy evaluates ((2.0*(x-mn))/R)-1.0, clip, NaN->0, *scale, trunc
template <int SRC>
__device__ __forceinline__ int32_t norm_sample(double x, const NormParams& p) {
  double t = x - p.mn;
  t = 2.0 * t;
  if constexpr (SRC == ST_F32 || SRC == ST_F64) t = t / p.range;
  else t = div_markstein(t, p.range, p.rcp);
  t = t - 1.0;
  if (t < -1.0) t = -1.0;
  else if (t > 1.0) t = 1.0;
  if (t != t) t = 0.0;
  t = t * p.scale;
  return p.to16 ? (int32_t)(int16_t)(int32_t)t : (int32_t)t;
}
template <int SRC>
__device__ __forceinline__ int32_t fetch_sample(const void* base, int64_t e, const NormParams& np) {
  if (np.mode == 0) return load_raw_int<SRC>(base, e);
  return norm_sample<SRC>(load_f64<SRC>(base, e), np);
}

template <int SRC> struct RawType { using T = double; };
template <> struct RawType<ST_U8> { using T = uint8_t; };
template <> struct RawType<ST_I8> { using T = int8_t; };
template <> struct RawType<ST_U16> { using T = uint16_t; };
template <> struct RawType<ST_I16> { using T = int16_t; };
template <> struct RawType<ST_U32> { using T = uint32_t; };
template <> struct RawType<ST_I32> { using T = int32_t; };
template <> struct RawType<ST_F32> { using T = float; };

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));  // a 16x16 int32 MFMA tile / 16 int8 MFMA operands

// normalisation-table index of a <= 16-bit integer raster value: its bit pattern as an unsigned integer
// (k_norm_lut fills the entries of the tile's values mn..mx)
template <int SRC, typename T>
__device__ __forceinline__ uint32_t lut_index(T v) {
  if constexpr (SRC == ST_U8 || SRC == ST_I8) return (uint32_t)(uint8_t)v;
  else return (uint32_t)(uint16_t)v;
}

template <typename T, int V>
struct alignas(sizeof(T) * V) VecT {
  T v[V];
};

// Load channel c of frame fr into smp[0..n): lane-contiguous (coalesced) reads; all of a thread's
// loads are issued before any is consumed (latency overlap), addresses advance incrementally (no
// per-sample division or 64-bit multiply).  VEC: 8-byte vectors of V = 8/itemsize samples (the
// host checked that no vector straddles a row and all are aligned: JobArgs::vec8), thread t owns
// vectors t + 256k; otherwise one element per lane, samples t + 256k.  Returns per-thread OR/min/max.
template <int SRC, bool VEC, typename SmpT>
__device__ __forceinline__ void load_raw_t(const void* base, const WaveDev& wd, const StreamDev* stp, const FrameDev* frp,
                                           int c, typename RawType<SRC>::T (&raw)[kMaxBlock / kThreads]) {
  using T = typename RawType<SRC>::T;
  constexpr int K = kMaxBlock / kThreads;
  constexpr int V = VEC ? 8 / (int)sizeof(T) : 1;
  const T* src = (const T*)base;
  const int n = wd.n, w = (int)wd.width, t = threadIdx.x;
  if constexpr (VEC) {  // (addresses from the frame's WaveDev only: no StreamDev round trip before the loads)
    using VT = VecT<T, V>;
    int col = (int)wd.col0 + t * V, row = 0;
    if (col >= w) {
      const int q = (int)((unsigned)col / (unsigned)w);
      row += q;
      col -= q * w;
    }
    const int64_t rs = (int64_t)wd.row_stride;
    int64_t e = wd.off0 + (int64_t)c * wd.band_stride + (int64_t)row * rs + col;
    const int step = kThreads * V;
    const int64_t wrap = rs - (int64_t)w;
    const int64_t e_first = wd.off0 + (int64_t)c * wd.band_stride + (int64_t)wd.col0;
#pragma unroll
    for (int kv = 0; kv < K / V; kv++) {
      const VT x = *(const VT*)(src + (((t + kv * kThreads) * V < n) ? e : e_first));
#pragma unroll
      for (int ee = 0; ee < V; ee++) raw[kv * V + ee] = x.v[ee];
      col += step;
      e += step;
      if (col >= w) {
        if (w >= step) { col -= w; e += wrap; }
        else {
          const int q = (int)((unsigned)col / (unsigned)w);
          col -= q * w;
          e += (int64_t)q * wrap;
        }
      }
    }
  } else {  // (element strides: StreamDev / FrameDev read here only, not kept live through the kernel)
  const StreamDev& st = *stp;
  const FrameDev& fr = *frp;
  int col = fr.col0 + t, row = fr.row0;
  if (col >= w) {
    const int q = (int)((unsigned)col / (unsigned)w);
    row += q;
    col -= q * w;
  }
  int64_t e = st.base_off + (int64_t)c * st.band_stride + (int64_t)row * st.row_stride + (int64_t)col * st.col_stride;
  const int64_t step = (int64_t)kThreads * st.col_stride;
  const int64_t wrap = st.row_stride - (int64_t)w * st.col_stride;
  // address of sample 0 (valid whenever n >= 1): out-of-range lanes re-read it, so the loads are
  // unconditional and the compiler can keep all K in flight
  const int64_t e_first = st.base_off + (int64_t)c * st.band_stride + (int64_t)fr.row0 * st.row_stride +
                          (int64_t)fr.col0 * st.col_stride;
#pragma unroll
  for (int k = 0; k < K; k++) {
    raw[k] = src[(t + k * kThreads < n) ? e : e_first];
    col += kThreads;
    e += step;
    if (col >= w) {
      if (w >= kThreads) { col -= w; e += wrap; }
      else {
        const int q = (int)((unsigned)col / (unsigned)w);
        col -= q * w;
        e += (int64_t)q * wrap;
      }
    }
  }
  }
}
// FRA-1 3.1b: the mid (L + R) >> 1 (msmode 1) or side L - R (msmode 2) of channels 0 and 1 into smp
// (32-bit instance only; |l|, |r| < 2^15 since mid-side streams are 16-bps).  Channel 0 is parked in this
// thread's own smp slots, then combined with channel 1.
template <int SRC, bool VEC>
__device__ __forceinline__ void load_mid_side_t(const void* base, const WaveDev& wd, const StreamDev* st, const FrameDev* fr,
                                             const NormParams& np, const int32_t* lut, int32_t* smp, uint32_t& orv,
                                             int32_t& vmin, int32_t& vmax, int msmode) {
  using T = typename RawType<SRC>::T;
  constexpr int K = kMaxBlock / kThreads;
  constexpr int V = VEC ? 8 / (int)sizeof(T) : 1;
  constexpr bool kLutType = SRC == ST_U8 || SRC == ST_I8 || SRC == ST_U16 || SRC == ST_I16;
  const int n = wd.n, t = threadIdx.x;
  auto sidx_of = [&](int k) { return VEC ? (t + (k / V) * kThreads) * V + (k % V) : t + k * kThreads; };
  auto audio = [&](T r) -> int32_t {
    if (kLutType && lut) return lut[lut_index<SRC>(r)];
    return np.mode == 0 ? (int32_t)r : norm_sample<SRC>((double)r, np);
  };
  T raw[K];
  load_raw_t<SRC, VEC, int32_t>(base, wd, st, fr, 0, raw);
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int i = sidx_of(k);
    if (i < n) smp[sidx(smp, i)] = audio(raw[k]);
  }
  load_raw_t<SRC, VEC, int32_t>(base, wd, st, fr, 1, raw);
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int i = sidx_of(k);
    if (i < n) {
      const int32_t l = smp[sidx(smp, i)], r = audio(raw[k]);
      const int32_t v = msmode == 1 ? ((l + r) >> 1) : l - r;
      smp[sidx(smp, i)] = v;
      orv |= (uint32_t)v;
      vmin = min(vmin, v);
      vmax = max(vmax, v);
    }
  }
}
// Load channel c of frame fr into smp[0..n) as audio integers (LUT / float64 normalisation, or raw
// ints when norm == 0): all of a thread's loads are issued before any is consumed.  Returns
// per-thread OR/min/max.  msmode != 0: the mid-side virtual channels (32-bit instance).
template <int SRC, bool VEC, typename SmpT>
__device__ __forceinline__ void load_channel_t(const void* base, const WaveDev& wd, const StreamDev* st, const FrameDev* fr, int c,
                                               const NormParams& np, const int32_t* lut, SmpT* smp, uint32_t& orv,
                                               int32_t& vmin, int32_t& vmax, int msmode) {
  if constexpr (std::is_same<SmpT, int32_t>::value) {
    if (msmode) {
      load_mid_side_t<SRC, VEC>(base, wd, st, fr, np, lut, smp, orv, vmin, vmax, msmode);
      return;
    }
  }
  using T = typename RawType<SRC>::T;
  constexpr int K = kMaxBlock / kThreads;
  constexpr int V = VEC ? 8 / (int)sizeof(T) : 1;
  const int n = wd.n, t = threadIdx.x;
  auto sidx_of = [&](int k) { return VEC ? (t + (k / V) * kThreads) * V + (k % V) : t + k * kThreads; };
  T raw[K];
  load_raw_t<SRC, VEC, SmpT>(base, wd, st, fr, c, raw);
  FRA_LOAD_STAMP(12, (int)raw[0] + (int)raw[K - 1])
  if constexpr (SRC == ST_U8 || SRC == ST_I8 || SRC == ST_U16 || SRC == ST_I16) {
    if (lut) {  // <= 16-bit integers: the normalised sample of value v is lut[lut_index(v)] (k_norm_lut)
      int32_t v[K];
#pragma unroll
      for (int k = 0; k < K; k++) v[k] = lut[lut_index<SRC>(raw[k])];
      FRA_LOAD_STAMP(13, v[0] + v[K - 1])
#pragma unroll
      for (int k = 0; k < K; k++) {
        const int i = sidx_of(k);
        if (i < n) {
          smp[sidx(smp, i)] = (SmpT)v[k];
          orv |= (uint32_t)v[k];
          vmin = min(vmin, v[k]);
          vmax = max(vmax, v[k]);
        }
      }
      return;
    }
  }
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int i = sidx_of(k);
    if (i < n) {
      int32_t v;
      if (np.mode == 0) v = (int32_t)raw[k];
      else v = norm_sample<SRC>((double)raw[k], np);
      smp[sidx(smp, i)] = (SmpT)v;
      orv |= (uint32_t)v;
      vmin = min(vmin, v);
      vmax = max(vmax, v);
    }
  }
  FRA_LOAD_STAMP(13, (int)orv)  // (diagnostic build only: normalised values stored)
}
// Fast path of the 16-bit instance (full 4096-sample frames of a <= 16-bit integer raster, 8-byte vectors,
// host-checked 32-bit byte offsets JobArgs::off32): per lane 32-bit offsets from a uniform frame-row base
// (saddr loads), LUT gathers by the raw value from a uniform table base, the samples packed as int16 pairs
// and stored 4 at a time (ds_write_b64: a thread's 4 or 8 consecutive samples lie in one 16-sample chunk),
// OR / min / max on the packed pairs (v_pk_min_i16 / v_pk_max_i16).  No per-sample bounds (n == 4096).
template <int SRC>
__device__ __forceinline__ void load_lut_full_t(const void* base, const WaveDev& wd, int c,
                                                const int32_t* lut, int16_t* smp, uint32_t& orv, int32_t& vmin,
                                                int32_t& vmax) {
  using T = typename RawType<SRC>::T;
  constexpr int V = 8 / (int)sizeof(T);                 // samples per 8-byte vector
  constexpr int NV = kMaxBlock / kThreads / V;          // vectors per thread
  constexpr int step = kThreads * V;
  using VT = VecT<T, V>;
  const int w = (int)wd.width, t = threadIdx.x;
  const char* b0 = (const char*)((const T*)base + wd.off0 + (int64_t)c * wd.band_stride);
  const uint32_t rsb = wd.row_stride * (uint32_t)sizeof(T);
  int col = (int)wd.col0 + t * V;
  uint32_t roff = 0;
  if (col >= w) {
    const int q = (int)((unsigned)col / (unsigned)w);
    col -= q * w;
    roff = (uint32_t)q * rsb;
  }
  VT x[NV];
#pragma unroll
  for (int kv = 0; kv < NV; kv++) {
    x[kv] = *(const VT*)(b0 + (roff + (uint32_t)col * (uint32_t)sizeof(T)));
    col += step;
    if (col >= w) {
      if (w >= step) { col -= w; roff += rsb; }
      else {
        const int q = (int)((unsigned)col / (unsigned)w);
        col -= q * w;
        roff += (uint32_t)q * rsb;
      }
    }
  }
  FRA_LOAD_STAMP(12, (int)x[0].v[0] + (int)x[NV - 1].v[V - 1])
  int32_t g[NV * V];
#pragma unroll
  for (int kv = 0; kv < NV; kv++)
#pragma unroll
    for (int e = 0; e < V; e++) g[kv * V + e] = lut[lut_index<SRC>(x[kv].v[e])];
  FRA_LOAD_STAMP(13, g[0] + g[NV * V - 1])
  uint32_t orp = 0;
  i16x2 pmin = {32767, 32767}, pmax = {-32768, -32768};
#pragma unroll
  for (int kv = 0; kv < NV; kv++) {
    const int i = (t + kv * kThreads) * V;
#pragma unroll
    for (int h = 0; h < V / 4; h++) {
      const uint32_t p0 = __builtin_amdgcn_perm((uint32_t)g[kv * V + 4 * h + 1], (uint32_t)g[kv * V + 4 * h], 0x05040100u);
      const uint32_t p1 = __builtin_amdgcn_perm((uint32_t)g[kv * V + 4 * h + 3], (uint32_t)g[kv * V + 4 * h + 2], 0x05040100u);
      *reinterpret_cast<uint2*>(smp + sidx(smp, i + 4 * h)) = make_uint2(p0, p1);
      orp |= p0 | p1;
      const i16x2 a0 = __builtin_bit_cast(i16x2, p0), a1 = __builtin_bit_cast(i16x2, p1);
      pmin = __builtin_elementwise_min(pmin, __builtin_elementwise_min(a0, a1));
      pmax = __builtin_elementwise_max(pmax, __builtin_elementwise_max(a0, a1));
    }
  }
  // OR of the int16 patterns: same trailing zeros as the OR of the sign-extended samples
  orv |= (orp | (orp >> 16)) & 0xFFFFu;
  vmin = min(vmin, min((int32_t)pmin.x, (int32_t)pmin.y));
  vmax = max(vmax, max((int32_t)pmax.x, (int32_t)pmax.y));
}
__device__ __forceinline__ bool load_lut_full(int src, const void* base, const WaveDev& wd, int c,
                                              const int32_t* lut, int16_t* smp, uint32_t& orv, int32_t& vmin,
                                              int32_t& vmax) {
  switch (src) {  // wave-uniform dispatch
    case ST_U8: load_lut_full_t<ST_U8>(base, wd, c, lut, smp, orv, vmin, vmax); return true;
    case ST_I8: load_lut_full_t<ST_I8>(base, wd, c, lut, smp, orv, vmin, vmax); return true;
    case ST_U16: load_lut_full_t<ST_U16>(base, wd, c, lut, smp, orv, vmin, vmax); return true;
    case ST_I16: load_lut_full_t<ST_I16>(base, wd, c, lut, smp, orv, vmin, vmax); return true;
    default: return false;
  }
}

template <typename SmpT>
__device__ __forceinline__ void load_channel(int src, bool vec8, const void* base, const WaveDev& wd, const StreamDev* st, const FrameDev* fr,
                                             int c, const NormParams& np, const int32_t* lut, SmpT* smp,
                                             uint32_t& orv, int32_t& vmin, int32_t& vmax, int msmode) {
  if (vec8) {
    switch (src) {  // wave-uniform dispatch; f64 never takes the vector path
      case ST_U8: load_channel_t<ST_U8, true, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); return;
      case ST_I8: load_channel_t<ST_I8, true, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); return;
      case ST_U16: load_channel_t<ST_U16, true, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); return;
      case ST_I16: load_channel_t<ST_I16, true, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); return;
      case ST_U32: load_channel_t<ST_U32, true, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); return;
      case ST_I32: load_channel_t<ST_I32, true, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); return;
      case ST_F32: load_channel_t<ST_F32, true, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); return;
      default: break;
    }
  }
  switch (src) {  // wave-uniform dispatch
    case ST_U8: load_channel_t<ST_U8, false, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); break;
    case ST_I8: load_channel_t<ST_I8, false, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); break;
    case ST_U16: load_channel_t<ST_U16, false, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); break;
    case ST_I16: load_channel_t<ST_I16, false, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); break;
    case ST_U32: load_channel_t<ST_U32, false, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); break;
    case ST_I32: load_channel_t<ST_I32, false, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); break;
    case ST_F32: load_channel_t<ST_F32, false, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); break;
    default: load_channel_t<ST_F64, false, SmpT>(base, wd, st, fr, c, np, lut, smp, orv, vmin, vmax, msmode); break;
  }
}

// ---------------------------------------------------------------- DPP helpers (gfx9 encodings)
enum : int { DPP_SHR1 = 0x111, DPP_SHR2 = 0x112, DPP_SHR4 = 0x114, DPP_SHR8 = 0x118, DPP_BC15 = 0x142, DPP_BC31 = 0x143 };
template <int CTRL, int RM>
__device__ __forceinline__ uint32_t dpp32(uint32_t v, uint32_t old = 0) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, RM, 0xF, false);
}
template <int CTRL, int RM>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  const uint32_t lo = dpp32<CTRL, RM>((uint32_t)v), hi = dpp32<CTRL, RM>((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
template <int CTRL, int RM>
__device__ __forceinline__ double dppf64(double v) {
  return __longlong_as_double((long long)dpp64<CTRL, RM>((uint64_t)__double_as_longlong(v)));
}
// step s of the upper-lane tree: lane j adds lane j - 2^s (the lower half of its 2^(s+1) group)
template <int S>
__device__ __forceinline__ uint64_t up_add64(uint64_t v) {
  if constexpr (S == 0) return v + dpp64<DPP_SHR1, 0xF>(v);
  else if constexpr (S == 1) return v + dpp64<DPP_SHR2, 0xF>(v);
  else if constexpr (S == 2) return v + dpp64<DPP_SHR4, 0xF>(v);
  else if constexpr (S == 3) return v + dpp64<DPP_SHR8, 0xF>(v);
  else if constexpr (S == 4) return v + dpp64<DPP_BC15, 0xA>(v);
  else return v + dpp64<DPP_BC31, 0xC>(v);
}
template <int S>
__device__ __forceinline__ uint32_t up_add32(uint32_t v) {
  if constexpr (S == 0) return v + dpp32<DPP_SHR1, 0xF>(v);
  else if constexpr (S == 1) return v + dpp32<DPP_SHR2, 0xF>(v);
  else if constexpr (S == 2) return v + dpp32<DPP_SHR4, 0xF>(v);
  else if constexpr (S == 3) return v + dpp32<DPP_SHR8, 0xF>(v);
  else if constexpr (S == 4) return v + dpp32<DPP_BC15, 0xA>(v);
  else return v + dpp32<DPP_BC31, 0xC>(v);
}
// FRA-1 autocorrelation tree over one wave's 64 chunk partials; result at lane 63
__device__ __forceinline__ double tree64(double v) {
  v = v + dppf64<DPP_SHR1, 0xF>(v);
  v = v + dppf64<DPP_SHR2, 0xF>(v);
  v = v + dppf64<DPP_SHR4, 0xF>(v);
  v = v + dppf64<DPP_SHR8, 0xF>(v);
  v = v + dppf64<DPP_BC15, 0xA>(v);
  v = v + dppf64<DPP_BC31, 0xC>(v);
  return v;
}
// FRA-1 autocorrelation: the wave's 64 chunk partials of every lag reduced by the descending-stride
// tree (32, 16, 8, 4, 2, 1; oracle ora_autocorr), as a reduce-scatter: strides 32 and 16 pair TWO
// lags per v_permlane32/16_swap + add (each lane keeps one of the two node sums), the in-row strides
// run the remaining values through DPP row_shr (upper lane keeps the node).  Every node is the sum
// of the same two child nodes as in the oracle (IEEE addition is commutative), so the result is
// bit-identical.  Lag sums are stored to red[lag] by lanes 15/31/47/63.
__device__ __forceinline__ void swap32_f64(double& x, double& y) {
  const uint64_t a = (uint64_t)__double_as_longlong(x), b = (uint64_t)__double_as_longlong(y);
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)a, (uint32_t)b, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(a >> 32), (uint32_t)(b >> 32), false, false);
  x = __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0]));
  y = __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
}
__device__ __forceinline__ void swap16_f64(double& x, double& y) {
  const uint64_t a = (uint64_t)__double_as_longlong(x), b = (uint64_t)__double_as_longlong(y);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)a, (uint32_t)b, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(a >> 32), (uint32_t)(b >> 32), false, false);
  x = __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0]));
  y = __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
}
template <int NL>
__device__ __forceinline__ void autocorr_reduce_wave(const double (&acc)[NL], double* red, int lane) {
  constexpr int N32 = (NL + 1) / 2, N16 = (N32 + 1) / 2;
  double w[N32];
#pragma unroll
  for (int k = 0; k < N32; k++) {  // stride 32: lanes < 32 keep lag 2k, lanes >= 32 lag 2k+1
    double x = acc[2 * k], y = (2 * k + 1 < NL) ? acc[2 * k + 1] : acc[2 * k];
    swap32_f64(x, y);
    w[k] = x + y;
  }
  double z[N16];
#pragma unroll
  for (int k = 0; k < N16; k++) {  // stride 16: row r keeps w[2k + (r & 1)] of half r >> 1
    double x = w[2 * k], y = (2 * k + 1 < N32) ? w[2 * k + 1] : w[2 * k];
    swap16_f64(x, y);
    z[k] = x + y;
  }
#pragma unroll
  for (int k = 0; k < N16; k++) {  // strides 8, 4, 2, 1 inside the row: node at lane 15 of the row
    double v = z[k];
    v = v + dppf64<DPP_SHR8, 0xF>(v);
    v = v + dppf64<DPP_SHR4, 0xF>(v);
    v = v + dppf64<DPP_SHR2, 0xF>(v);
    v = v + dppf64<DPP_SHR1, 0xF>(v);
    if ((lane & 15) == 15) {
      const int r = lane >> 4;
      const int wi = (2 * k + 1 < N32) ? 2 * k + (r & 1) : 2 * k;
      const int lag = (2 * wi + 1 < NL) ? 2 * wi + (r >> 1) : 2 * wi;
      red[lag] = v;
    }
  }
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {  // wave-uniform result
  v += dpp32<DPP_SHR1, 0xF>(v);
  v += dpp32<DPP_SHR2, 0xF>(v);
  v += dpp32<DPP_SHR4, 0xF>(v);
  v += dpp32<DPP_SHR8, 0xF>(v);
  v += dpp32<DPP_BC15, 0xA>(v);
  v += dpp32<DPP_BC31, 0xC>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint32_t wave_min32(uint32_t v) {  // wave-uniform result
  v = min(v, dpp32<DPP_SHR1, 0xF>(v, ~0u));
  v = min(v, dpp32<DPP_SHR2, 0xF>(v, ~0u));
  v = min(v, dpp32<DPP_SHR4, 0xF>(v, ~0u));
  v = min(v, dpp32<DPP_SHR8, 0xF>(v, ~0u));
  v = min(v, dpp32<DPP_BC15, 0xA>(v, ~0u));
  v = min(v, dpp32<DPP_BC31, 0xC>(v, ~0u));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
template <int CTRL, int RM>
__device__ __forceinline__ uint64_t dpp64_old(uint64_t v, uint64_t old) {
  const uint32_t lo = dpp32<CTRL, RM>((uint32_t)v, (uint32_t)old), hi = dpp32<CTRL, RM>((uint32_t)(v >> 32), (uint32_t)(old >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {  // wave-uniform result
  v = min(v, dpp64_old<DPP_SHR1, 0xF>(v, ~0ull));
  v = min(v, dpp64_old<DPP_SHR2, 0xF>(v, ~0ull));
  v = min(v, dpp64_old<DPP_SHR4, 0xF>(v, ~0ull));
  v = min(v, dpp64_old<DPP_SHR8, 0xF>(v, ~0ull));
  v = min(v, dpp64_old<DPP_BC15, 0xA>(v, ~0ull));
  v = min(v, dpp64_old<DPP_BC31, 0xC>(v, ~0ull));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t wave_or32(uint32_t v) {
  v |= dpp32<DPP_SHR1, 0xF>(v);
  v |= dpp32<DPP_SHR2, 0xF>(v);
  v |= dpp32<DPP_SHR4, 0xF>(v);
  v |= dpp32<DPP_SHR8, 0xF>(v);
  v |= dpp32<DPP_BC15, 0xA>(v);
  v |= dpp32<DPP_BC31, 0xC>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// inclusive prefix sum over the wave (Hillis-Steele inside rows, then row broadcasts)
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t v) {
  v += dpp32<DPP_SHR1, 0xF>(v);
  v += dpp32<DPP_SHR2, 0xF>(v);
  v += dpp32<DPP_SHR4, 0xF>(v);
  v += dpp32<DPP_SHR8, 0xF>(v);
  v += dpp32<DPP_BC15, 0xA>(v);
  v += dpp32<DPP_BC31, 0xC>(v);
  return v;
}

// ---------------------------------------------------------------- integer helpers
__device__ __forceinline__ uint64_t zz64(int64_t r) {
  return r >= 0 ? ((uint64_t)r << 1) : ((((uint64_t)(-(r + 1))) << 1) | 1u);
}
__device__ __forceinline__ uint32_t zz32(int32_t r) { return ((uint32_t)r << 1) ^ (uint32_t)(r >> 31); }
// |a - b| + acc for int32 a, b given as a ^ 2^31, b ^ 2^31 (unsigned order == signed order): one
// v_sad_u32.  The estimate sums are 2 * sum |r|.
constexpr uint32_t kBias = 0x80000000u;
__device__ __forceinline__ uint32_t sad_acc(uint32_t ab, uint32_t bb, uint32_t acc) {
  // forced: from the select form the compiler emitted v_sub_co + v_cndmask + v_add3 (and an s_nop for the
  // vcc hazard) wherever one operand was the constant bias -- three VALU instructions instead of one
  uint32_t d;
  asm("v_sad_u32 %0, %1, %2, %3" : "=v"(d) : "v"(ab), "v"(bb), "v"(acc));
  return d;
}
// b - a + 2^31 - 1 (mod 2^32) in one v_xad_u32: the biased difference of two values of the same bias
__device__ __forceinline__ uint32_t xad_bias(uint32_t a, uint32_t b) {
  uint32_t d;
  asm("v_xad_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(0x7FFFFFFFu), "v"(b));
  return d;
}
__device__ __forceinline__ uint64_t abs2_64(int64_t r) { return 2 * (uint64_t)(r < 0 ? -r : r); }
__device__ __forceinline__ int bitlen64(uint64_t v) { return v ? 64 - __clzll((long long)v) : 0; }

// Rice parameter estimate == oracle rice_pick: kc = bitlen(S / n) computed without
// a division: kc = smallest k >= 0 with S < n*2^k, which is max(0, bitlen(S)-bitlen(n)) or one more.
__device__ __forceinline__ uint64_t rice_est2(uint64_t n, uint64_t S, int k) {
  const uint64_t lo = n * (uint64_t)((1u << k) - 1u);
  const uint64_t tail = (2 * S > lo) ? ((2 * S - lo) >> (k + 1)) : 0;
  return n * (uint64_t)(k + 1) + tail;
}
__device__ __forceinline__ void rice_pick(uint64_t n, uint64_t S, int& k_out, uint64_t& bits_out) {
  const int a = bitlen64(S), b = bitlen64(n);
  int kc = a > b ? a - b : 0;
  if (S >= (n << kc)) kc++;
  const int lo = kc - 2 < 0 ? 0 : kc - 2, hi = kc + 1 > 30 ? 30 : kc + 1;
  uint64_t best = rice_est2(n, S, lo);
  int bk = lo;
  for (int k = lo + 1; k <= hi; k++) {
    const uint64_t e = rice_est2(n, S, k);
    if (e < best) { best = e; bk = k; }
  }
  k_out = bk;
  bits_out = best;
}

// the same pick in 32-bit arithmetic, valid (bit-identical) whenever S < 2^29 and n < 2^13: then
// kc <= bitlen(S) - bitlen(n) + 1, so n * 2^k < 2^31 for every candidate k <= kc + 1, 2S < 2^30, and no
// intermediate wraps; n * (2^k - 1) as (n << k) - n, n * (k + 1) on the 24-bit multiplier
// Branch-free (r05): the <= 4 candidates lo .. lo + 3 (hi - lo <= 3) are all evaluated and the ones past hi
// masked, so lanes with different ranges run one straight instruction stream (the loop with a per-lane trip
// count ran under exec masking: ~3 SALU per trip plus the loop's own branches); same first-minimum rule.
__device__ __forceinline__ void rice_pick32(uint32_t n, uint32_t S, int& k_out, uint32_t& bits_out) {
  const int a = S ? 32 - __clz((int)S) : 0, b = n ? 32 - __clz((int)n) : 0;
  int kc = a > b ? a - b : 0;
  kc += S >= (n << kc) ? 1 : 0;
  const int lo = kc - 2 < 0 ? 0 : kc - 2, hi = kc + 1 > 30 ? 30 : kc + 1;
  auto est = [&](int k) -> uint32_t {
    const uint32_t l = (n << k) - n;
    const uint32_t tail = (2 * S > l) ? ((2 * S - l) >> (k + 1)) : 0u;
    return __umul24(n, (uint32_t)(k + 1)) + tail;
  };
  uint32_t best = est(lo);
  int bk = lo;
#pragma unroll
  for (int dk = 1; dk <= 3; dk++) {
    const int k = lo + dk;
    const uint32_t e = est(k <= 30 ? k : 30);
    const bool take = k <= hi && e < best;
    best = take ? e : best;
    bk = take ? k : bk;
  }
  k_out = bk;
  bits_out = best;
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)v, m, 64);
  const uint32_t hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  for (int off = 32; off >= 1; off >>= 1) v += shfl_xor_u64(v, off);
  return v;
}

// ---------------------------------------------------------------- LPC analysis helpers
// deterministic log2 -- same op sequence as oracle ora_det_log2 (series terms
// multiplied by the correctly rounded constants 1/(2k+1); the only division is t)
__device__ inline double det_log2(double x) {
  constexpr double kInvOdd[12] = {1.0,      1.0 / 3,  1.0 / 5,  1.0 / 7,  1.0 / 9,  1.0 / 11,
                                  1.0 / 13, 1.0 / 15, 1.0 / 17, 1.0 / 19, 1.0 / 21, 1.0 / 23};
  int e;
  double m = frexp(x, &e);
  m = m * 2.0;
  e = e - 1;
  const double t = (m - 1.0) / (m + 1.0);
  const double t2 = t * t;
  double sum = 0.0, p = t;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    sum = sum + p * kInvOdd[k];
    p = p * t2;
  }
  return (double)e + 2.0 * sum * 1.4426950408889634;
}
// expected bits of LPC order o from its LD error (== oracle best_order_by_error's per-order term)
__device__ inline double order_bits(double e, int n, int o, int overhead) {
  double bps;
  if (e > 0.0) {
    bps = 0.5 * det_log2(0.5 * e / (double)n);
    if (bps < 0.0) bps = 0.0;
  } else if (e < 0.0) bps = 1e32;
  else bps = 0.0;
  return bps * (double)(n - o) + (double)(o * overhead);
}
// FRA-1 3.7b window score (== oracle window_score): the expected bits of a window's chosen order o with its LD
// error taken relative to the window's own energy ac0, so a partial window ranks against the full one
__device__ inline double window_score(double e, double ac0, int n, int o, int overhead) {
  const double rel = e / ac0;
  double bps;
  if (rel > 0.0) bps = 0.5 * det_log2(0.5 * rel);
  else if (rel < 0.0) bps = 1e32;
  else bps = -1e32;
  return bps * (double)(n - o) + (double)(o * overhead);
}
__device__ inline int best_order_by_error(const double* err, int norders, int n, int overhead) {
  double best = 0.0;
  int bo = 1;
  for (int o = 1; o <= norders; o++) {
    const double bits = order_bits(err[o - 1], n, o, overhead);
    if (o == 1 || bits < best) { best = bits; bo = o; }
  }
  return bo;
}

// Levinson-Durbin run uniformly by a whole wave from register-resident autocorrelation: errors
// stay in registers (errv), coefficient rows go to LDS from lane 0 only.  Same op sequence as
// oracle ora_levinson.
// LD coefficient rows, row i (order i + 1, i + 1 entries) at lp[i (i + 1) / 2 ...] (triangular)
__host__ __device__ constexpr int lp_row(int i) { return i * (i + 1) / 2; }
template <int MAXLAG>
__device__ inline int levinson_wave(const double (&ac)[MAXLAG + 1], int max_order, double* lp,
                                    double (&errv)[MAXLAG], bool writer) {
  double lpc[MAXLAG];
#pragma unroll
  for (int j = 0; j < MAXLAG; j++) { lpc[j] = 0.0; errv[j] = 0.0; }
  double err = ac[0];
  int result = max_order;
  bool done = false;
#pragma unroll
  for (int i = 0; i < MAXLAG; i++) {
    if (!done && i < max_order) {
      double r = -ac[i + 1];
#pragma unroll
      for (int j = 0; j < i; j++) r = r - lpc[j] * ac[i - j];
      r = r / err;
      lpc[i] = r;
#pragma unroll
      for (int j = 0; j < (i >> 1); j++) {
        const double tmp = lpc[j];
        lpc[j] = lpc[j] + r * lpc[i - 1 - j];
        lpc[i - 1 - j] = lpc[i - 1 - j] + r * tmp;
      }
      if (i & 1) lpc[i >> 1] = lpc[i >> 1] + lpc[i >> 1] * r;
      err = err * (1.0 - r * r);
      if (writer) {  // rows stored as lpc (the reader negates the one row it quantises)
#pragma unroll
        for (int j = 0; j <= i; j++) lp[lp_row(i) + j] = lpc[j];
      }
      errv[i] = err;
      if (!(err > 0.0)) {
        result = (err == 0.0) ? i + 1 : i;
        done = true;
      }
    }
  }
  return result;
}
// Levinson-Durbin, same op sequence as oracle ora_levinson; loops unrolled to the
// compile-time bound so the recursion state stays in registers.
template <int MAXLAG>
__device__ inline int levinson(const double* autoc, int max_order, double (*lp)[kMaxLpc], double* err_out) {
  double lpc[MAXLAG];
#pragma unroll
  for (int j = 0; j < MAXLAG; j++) lpc[j] = 0.0;
  double err = autoc[0];
  int result = max_order;
  bool done = false;
#pragma unroll
  for (int i = 0; i < MAXLAG; i++) {
    if (!done && i < max_order) {
      double r = -autoc[i + 1];
#pragma unroll
      for (int j = 0; j < i; j++) r = r - lpc[j] * autoc[i - j];
      r = r / err;
      lpc[i] = r;
#pragma unroll
      for (int j = 0; j < (i >> 1); j++) {
        const double tmp = lpc[j];
        lpc[j] = lpc[j] + r * lpc[i - 1 - j];
        lpc[i - 1 - j] = lpc[i - 1 - j] + r * tmp;
      }
      if (i & 1) lpc[i >> 1] = lpc[i >> 1] + lpc[i >> 1] * r;
      err = err * (1.0 - r * r);
#pragma unroll
      for (int j = 0; j <= i; j++) lp[i][j] = -lpc[j];
      err_out[i] = err;
      if (!(err > 0.0)) {
        result = (err == 0.0) ? i + 1 : i;
        done = true;
      }
    }
  }
  return result;
}

__device__ __forceinline__ double rnd_half_away(double x) {
  double t = trunc(x);
  const double d = x - t;
  if (d >= 0.5) t = t + 1.0;
  else if (d <= -0.5) t = t - 1.0;
  return t;
}
// qlp quantisation with error feedback; false if not representable
template <int MAXLAG>
__device__ inline bool quantize(const double* lp, int order, int precision, int32_t* q, int& shift_out) {
  double cmax = 0.0;
#pragma unroll
  for (int j = 0; j < MAXLAG; j++) {
    if (j < order) {
      const double a = fabs(lp[j]);
      if (a > cmax) cmax = a;
    }
  }
  if (!(cmax > 0.0)) return false;
  int e;
  (void)frexp(cmax, &e);
  int shift = precision - 1 - e;
  if (shift > 15) shift = 15;
  if (shift < 0) return false;
  const int32_t qmax = (1 << (precision - 1)) - 1, qmin = -(1 << (precision - 1));
  double errf = 0.0;
#pragma unroll
  for (int j = 0; j < MAXLAG; j++) {
    if (j < order) {
      errf = errf + ldexp(lp[j], shift);
      const double qd = rnd_half_away(errf);
      int32_t qi = (int32_t)qd;
      if (qi > qmax) qi = qmax;
      if (qi < qmin) qi = qmin;
      errf = errf - (double)qi;
      q[j] = qi;
    } else {
      q[j] = 0;
    }
  }
  shift_out = shift;
  return true;
}

// ---------------------------------------------------------------- residual evaluators
// x[12 + jj] = sample i0 + jj; x[0..11] = the 12 preceding samples (0 before the block start).
template <bool B32, int O>
__device__ __forceinline__ int64_t fixed_res(const int32_t* x, int jj) {
  const int b = 12 + jj;
  if constexpr (B32) {
    const int64_t s0 = x[b];
    if constexpr (O == 0) return s0;
    else if constexpr (O == 1) return s0 - (int64_t)x[b - 1];
    else if constexpr (O == 2) return s0 - 2 * (int64_t)x[b - 1] + (int64_t)x[b - 2];
    else if constexpr (O == 3) return s0 - 3 * (int64_t)x[b - 1] + 3 * (int64_t)x[b - 2] - (int64_t)x[b - 3];
    else return s0 - 4 * (int64_t)x[b - 1] + 6 * (int64_t)x[b - 2] - 4 * (int64_t)x[b - 3] + (int64_t)x[b - 4];
  } else {
    const int32_t s0 = x[b];
    if constexpr (O == 0) return s0;
    else if constexpr (O == 1) return s0 - x[b - 1];
    else if constexpr (O == 2) return s0 - 2 * x[b - 1] + x[b - 2];
    else if constexpr (O == 3) return s0 - 3 * x[b - 1] + 3 * x[b - 2] - x[b - 3];
    else return s0 - 4 * x[b - 1] + 6 * x[b - 2] - 4 * x[b - 3] + x[b - 4];
  }
}
template <bool B32, int O>
__device__ __forceinline__ int64_t lpc_res(const int32_t* x, int jj, const int32_t* q, int sh) {
  const int b = 12 + jj;
  if constexpr (B32) {
    int64_t sum = 0;
#pragma unroll
    for (int j = 0; j < O; j++) sum += (int64_t)q[j] * (int64_t)x[b - 1 - j];
    return (int64_t)x[b] - (sum >> sh);
  } else {
    int32_t sum = 0;
#pragma unroll
    for (int j = 0; j < O; j++) sum += q[j] * x[b - 1 - j];
    return (int64_t)(x[b] - (sum >> sh));
  }
}
// residual of sample jj for a runtime model (slow paths only)
template <bool B32>
__device__ __forceinline__ int64_t model_res(const int32_t* x, int jj, int type, int o, const int32_t* q, int sh) {
  if (type == 2) {
    switch (o) {
      case 0: return fixed_res<B32, 0>(x, jj);
      case 1: return fixed_res<B32, 1>(x, jj);
      case 2: return fixed_res<B32, 2>(x, jj);
      case 3: return fixed_res<B32, 3>(x, jj);
      default: return fixed_res<B32, 4>(x, jj);
    }
  }
  const int b = 12 + jj;
  if constexpr (B32) {
    int64_t sum = 0;
#pragma unroll
    for (int j = 0; j < kMaxLpc; j++)
      if (j < o) sum += (int64_t)q[j] * (int64_t)x[b - 1 - j];
    return (int64_t)x[b] - (sum >> sh);
  } else {
    int32_t sum = 0;
#pragma unroll
    for (int j = 0; j < kMaxLpc; j++)
      if (j < o) sum += q[j] * x[b - 1 - j];
    return (int64_t)(x[b] - (sum >> sh));
  }
}

// ---------------------------------------------------------------- generic residual body
// r = x[i] - ((sum_j q[j] * x[i-1-j]) >> sh), q[j] = 0 for j >= order; x[12 + jj] = sample i0 + jj
template <bool B32, int MAXO>
__device__ __forceinline__ int64_t gres(const int32_t* x, int jj, const int32_t* q, int sh) {
  const int b = 12 + jj;
  if constexpr (B32) {
    int64_t sum = 0;
#pragma unroll
    for (int j = 0; j < MAXO; j++) sum += (int64_t)q[j] * (int64_t)x[b - 1 - j];
    return (int64_t)x[b] - (sum >> sh);
  } else {
    int32_t sum = 0;
#pragma unroll
    for (int j = 0; j < MAXO; j++) sum += __mul24(q[j], x[b - 1 - j]);
    return (int64_t)(x[b] - (sum >> sh));
  }
}
// the same predictor read from the LDS sample array (slow path: irregular frames only)
template <bool B32, int MAXO, typename SmpT>
__device__ __forceinline__ int64_t gres_lds(const SmpT* smp, int i, const int32_t* q, int sh) {
  if constexpr (B32) {
    int64_t sum = 0;
    for (int j = 0; j < MAXO; j++) sum += (int64_t)q[j] * (int64_t)smp[sidx(smp, max(0, i - 1 - j))];
    return (int64_t)smp[sidx(smp, i)] - (sum >> sh);
  } else {
    int32_t sum = 0;
    for (int j = 0; j < MAXO; j++) sum += __mul24(q[j], (int32_t)smp[sidx(smp, max(0, i - 1 - j))]);
    return (int64_t)((int32_t)smp[sidx(smp, i)] - (sum >> sh));
  }
}

// OR a value of `width` bits (1..32, already masked) at bit position pos of a big-endian word buffer
__device__ __forceinline__ void lds_put(uint32_t* buf, uint32_t pos, uint32_t v, int width) {
  // v already masked to width (1..32); MSB-first bit order within big-endian words
  const uint32_t w0 = pos >> 5, off = pos & 31;
  const int end = (int)off + width;
  if (end <= 32) {
    atomicOr(&buf[w0], v << (32 - end));
  } else {
    atomicOr(&buf[w0], v >> (end - 32));
    atomicOr(&buf[w0 + 1], v << (64 - end));
  }
}

// Branch-free variant for the residual loops: always ORs into words w0 and w0 + 1 (the second OR may
// be of zero bits), so a wave issues two LDS ops per code instead of three when its lanes split
// over the two cases.  Needs one spare zeroed word after the last one written.
__device__ __forceinline__ void lds_put2(uint32_t* buf, uint32_t pos, uint32_t v, int width) {
  const uint32_t w0 = pos >> 5;
  const uint64_t x = ((uint64_t)v << (64 - width)) >> (pos & 31);
  atomicOr(&buf[w0], (uint32_t)(x >> 32));
  atomicOr(&buf[w0 + 1], (uint32_t)x);
}

// A code left-aligned in 32 bits (its first bit at bit 31, zeros below its last bit) written at bit
// position P: both words it can touch are ORed unconditionally (shift counts use P mod 32 in hardware).
__device__ __forceinline__ void lds_put_al(uint32_t* buf, uint32_t P, uint32_t cal) {
  const uint32_t w0 = P >> 5;
  atomicOr(&buf[w0], cal >> (P & 31u));
  atomicOr(&buf[w0 + 1], __builtin_amdgcn_alignbit(cal, 0u, P & 31u));
}

// ---------------------------------------------------------------- 16-bit sample pairs (k_analyze, k_analyze_w)
// int16 storage is read as aligned dword pairs and sign-extended (2 samples per dword, even sample low)
__device__ __forceinline__ int32_t lo16(uint32_t v) { return (int32_t)(int16_t)(v & 0xFFFFu); }
__device__ __forceinline__ int32_t hi16(uint32_t v) { return (int32_t)v >> 16; }
typedef short fra_short2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fra_short2 pack_pair(int32_t lo, int32_t hi) {
  return __builtin_bit_cast(fra_short2, __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u));
}
// D[j] = samples (x[2j], x[2j+1]); the dot2 operand pair (x[k], x[k+1]) is a word itself for even k,
// one v_alignbit for odd k
__device__ __forceinline__ uint32_t pair_at(const uint32_t (&D)[14], int k) {
  return (k & 1) ? __builtin_amdgcn_alignbit(D[(k + 1) >> 1], D[(k - 1) >> 1], 16) : D[k >> 1];
}
__device__ __forceinline__ int32_t sample_at(const uint32_t (&D)[14], int k) {
  return (k & 1) ? hi16(D[k >> 1]) : lo16(D[k >> 1]);
}
template <int NP>
__device__ __forceinline__ void q_pairs_rev(const int32_t* q, fra_short2 (&Q)[NP]) {
#pragma unroll
  for (int p = 0; p < NP; p++) Q[p] = pack_pair(q[2 * p + 1], q[2 * p]);
}
// prediction of x[b]: sum_p dot2((x[b-2-2p], x[b-1-2p]), (q[2p+1], q[2p]))
template <int NP>
__device__ __forceinline__ int32_t pred_raw(const uint32_t (&D)[14], int b, const fra_short2 (&Q)[NP]) {
  int32_t acc = 0;
#pragma unroll
  for (int p = 0; p < NP; p++)
    acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(fra_short2, pair_at(D, b - 2 - 2 * p)), Q[p], acc, false);
  return acc;
}

// apodization coefficients of samples i0 .. i0 + 16 + MAXLAG - 1 of one window (row of the plan's window
// table, exactly n entries used): unconditional vector loads when the whole span lies inside the block,
// else only the entries below n (the others are never multiplied: wf = 0 past n) -- no read past the
// window the frame owns (the table is allocated at its exact size)
template <int MAXLAG>
__device__ __forceinline__ void load_window(const float* win, int i0, int n, float (&w)[kChunk + MAXLAG]) {
  if (i0 + kChunk + MAXLAG <= n) {
#pragma unroll
    for (int j = 0; j < kChunk + MAXLAG; j++) w[j] = win[i0 + j];
  } else {
#pragma unroll
    for (int j = 0; j < kChunk + MAXLAG; j++) w[j] = i0 + j < n ? win[i0 + j] : 0.0f;
  }
}

// L2 prefetch hint (k_analyze, k_analyze_w): one dword per 128-byte line of the raw rows of the subframe DIST
// blocks ahead in dispatch order (linear block id over the (frames, channels) grid; a multiple of 8 keeps
// the same XCD, blocks being dealt round-robin over the XCDs).  Nothing depends on the words but the speed.
template <typename T, int DIST>
__device__ __forceinline__ uint32_t prefetch_rows(const JobArgs& a, int lane) {
  const uint32_t nx = gridDim.x;
  const uint64_t L = (uint64_t)blockIdx.x + (uint64_t)blockIdx.y * nx + DIST;
  if (L >= (uint64_t)nx * gridDim.y) return 0u;
  const int xp = (int)(L % nx), yp = (int)(L / nx);  // uniform
  const FrameDev f2 = a.frames[a.frame_base + xp];
  const StreamDev s2 = a.streams[f2.stream];
  if (yp >= s2.channels || s2.ms || f2.n != kMaxBlock || s2.col_stride != 1) return 0u;
  const char* b0 = (const char*)((const T*)a.raster + s2.base_off + (int64_t)yp * s2.band_stride +
                                 (int64_t)f2.row0 * s2.row_stride);
  const uint32_t w = (uint32_t)s2.width, rsb = (uint32_t)s2.row_stride * (uint32_t)sizeof(T);
  // the 64-sample run of this lane (inside the subframe: n == 4096) spans <= 128 bytes: its first and
  // last samples cover every line it touches (dword-aligned down)
  auto word = [&](uint32_t c) -> uint32_t {
    const uint32_t q = c / w;
    return *(const uint32_t*)(b0 + ((q * rsb + (c - q * w) * (uint32_t)sizeof(T)) & ~3u));
  };
  const uint32_t c0 = (uint32_t)f2.col0 + 64u * (uint32_t)lane;
  return word(c0) ^ word(c0 + 63u);
}

// ---------------------------------------------------------------- cross-lane gathers and the partition search
__device__ __forceinline__ uint32_t bperm32(uint32_t v, int src) {  // lane src's v (ds_bpermute)
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
__device__ __forceinline__ uint64_t bperm64(uint64_t v, int src) {
  return ((uint64_t)bperm32((uint32_t)(v >> 32), src) << 32) | bperm32((uint32_t)v, src);
}

// Partition-order search (FRA-1 3.8) on a register of finest partition sums (lane p < 2^P), without LDS: node
// (level q, index j) -- the sum of finest partitions [j 2^(P-q), (j+1) 2^(P-q)) -- is needed at lane 2^q + j;
// the upper-lane tree leaves it after step P - q - 1 at lane (j+1) 2^(P-q) - 1, one ds_bpermute per step.
// Same nodes, tree, tie rule and outputs as the oracle's per-level loop (p = pm..0, keep '<='); every node sum
// < 2^29 runs in 32-bit arithmetic (rice_pick32, bit-identical); kreg lane j < 2^bp = partition j's Rice parameter
__device__ __forceinline__ void porder_search_reg(uint64_t Sv, int P, int pm, int n, int o, int lane, uint64_t& best_out,
                                                int& bp_out, uint32_t& kreg, uint64_t* total_out = nullptr) {
  const int p = lane ? 31 - __clz(lane) : 0;  // this lane's level; j = lane - 2^p
  const int jn = lane - (1 << p);
  uint32_t bits32 = 0;
  bool big = false;
  int kn = 0;
  uint32_t tot6 = 0;
  bool big6 = false;
  int k6 = 0;
  if (__all(Sv < (1ull << 23))) {  // every node sum < 2^29: 32-bit arithmetic (rice_pick32), bit-identical
    uint32_t S = (uint32_t)Sv;
    // level P <= 5: the finest sums themselves (every ds_bpermute runs on all 64 lanes: a source lane outside
    // EXEC would read as 0, so none may sit under a lane-dependent condition)
    const uint32_t fin = bperm32(S, jn & 63);
    uint32_t nv = p == P ? fin : 0u;
#define FRA_NODE_STEP32(S_)                                                        \
  if (P > S_) {                                                                    \
    S = up_add32<S_>(S);                                                           \
    const uint32_t tv = bperm32(S, (((jn + 1) << (S_ + 1)) - 1) & 63);             \
    nv = p == P - S_ - 1 ? tv : nv;                                                \
  }
    FRA_NODE_STEP32(0) FRA_NODE_STEP32(1) FRA_NODE_STEP32(2)
    FRA_NODE_STEP32(3) FRA_NODE_STEP32(4) FRA_NODE_STEP32(5)
#undef FRA_NODE_STEP32
    if (total_out) *total_out = (uint32_t)__builtin_amdgcn_readlane((int)nv, 1);  // node (0, 0): the block total
    {  // every lane (no exec masking), the result kept where the lane holds a node of a searched level
      int kq;
      uint32_t bq;
      rice_pick32((uint32_t)((n >> p) - (jn == 0 ? o : 0)), nv, kq, bq);
      const bool act = lane >= 1 && p <= P && p <= pm;
      kn = act ? kq : 0;
      bits32 = act ? bq : 0u;
      big = act && kq > 14;
    }
    if (P == 6 && pm == 6) {  // level 6: the finest sums at lane j
      uint32_t b6;
      rice_pick32((uint32_t)((n >> 6) - (lane == 0 ? o : 0)), (uint32_t)Sv, k6, b6);
      tot6 = wave_sum32(b6);
      big6 = __any(k6 > 14);
    }
  } else {
    uint64_t S = Sv;
    const uint64_t fin = bperm64(S, jn & 63);
    uint64_t nv = p == P ? fin : 0ull;
#define FRA_NODE_STEP(S_)                                                          \
  if (P > S_) {                                                                    \
    S = up_add64<S_>(S);                                                           \
    const uint64_t tv = bperm64(S, (((jn + 1) << (S_ + 1)) - 1) & 63);             \
    nv = p == P - S_ - 1 ? tv : nv;                                                \
  }
    FRA_NODE_STEP(0) FRA_NODE_STEP(1) FRA_NODE_STEP(2)
    FRA_NODE_STEP(3) FRA_NODE_STEP(4) FRA_NODE_STEP(5)
#undef FRA_NODE_STEP
    if (total_out)
      *total_out = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(nv >> 32), 1) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)nv, 1);
    if (lane >= 1 && p <= P && p <= pm) {
      uint64_t bits;
      rice_pick((uint64_t)((n >> p) - (jn == 0 ? o : 0)), nv, kn, bits);
      bits32 = (uint32_t)bits;
      big = kn > 14;
    }
    if (P == 6 && pm == 6) {
      uint64_t b6;
      rice_pick((uint64_t)((n >> 6) - (lane == 0 ? o : 0)), Sv, k6, b6);
      tot6 = wave_sum32((uint32_t)b6);
      big6 = __any(k6 > 14);
    }
  }
  const uint64_t bigm = __ballot(big);
  uint32_t tot[7];
  uint32_t v = bits32;
  tot[0] = (uint32_t)__builtin_amdgcn_readlane((int)v, 1);
  v += dpp32<DPP_SHR1, 0xF>(v);
  tot[1] = (uint32_t)__builtin_amdgcn_readlane((int)v, 3);
  v += dpp32<DPP_SHR2, 0xF>(v);
  tot[2] = (uint32_t)__builtin_amdgcn_readlane((int)v, 7);
  v += dpp32<DPP_SHR4, 0xF>(v);
  tot[3] = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
  v += dpp32<DPP_SHR8, 0xF>(v);
  tot[4] = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
  v += dpp32<DPP_BC15, 0xA>(v);
  tot[5] = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
  tot[6] = tot6;
  // orders pm .. 0, '<=' keeps the smaller order: unrolled over the compile-time order so tot[q] and the
  // masks are plain registers (a runtime q compiled to a select chain over tot[] per step, ~40 SALU each)
  uint64_t best = 0;
  int bp = pm;
  bool first = true;
#pragma unroll
  for (int q = 6; q >= 0; q--) {
    if (q <= pm) {
      const bool bq = q == 6 ? big6 : ((bigm >> (1u << (q % 6))) & ((1ull << (1u << (q % 6))) - 1)) != 0;
      const uint64_t t = (uint64_t)tot[q] + (uint64_t)(1u << q) * (bq ? 5 : 4) + 6;
      if (first || t <= best) { best = t; bp = q; }
      first = false;
    }
  }
  best_out = best;
  bp_out = bp;
  // partition j's parameter at order bp: node (bp, j) sits at lane 2^bp + j (level 6: k6 at lane j)
  const int kl = __shfl(kn, ((1 << (bp < 6 ? bp : 0)) + lane) & 63, 64);
  kreg = (uint32_t)(bp == 6 ? k6 : kl);
}

#ifdef FRA_STAMPS
// diagnostic build only (csrc/Makefile `wstamps`, tools/wstamp_phases.py): lane 0 of the first kWStampW waves
// stores s_memtime after each phase, inside the real steady state
constexpr unsigned kWStampW = 1u << 18, kWStampN = 16;
__device__ unsigned long long g_fra_wstamps[kWStampW * kWStampN];
#define FRA_WSTAMP(k)                                                                            \
  if (lane == 0) {                                                                               \
    const unsigned wi_ = blockIdx.x * gridDim.y + blockIdx.y;                                    \
    if (wi_ < kWStampW) g_fra_wstamps[wi_ * kWStampN + (k)] = __builtin_amdgcn_s_memtime();      \
  }
#define FRA_WSTAMP_VAL(k, v)                                                                     \
  if (lane == 0) {                                                                               \
    const unsigned wi_ = blockIdx.x * gridDim.y + blockIdx.y;                                    \
    if (wi_ < kWStampW) g_fra_wstamps[wi_ * kWStampN + (k)] = (unsigned long long)(v);            \
  }
// FRA_WSTAMP_FINE: the load phase split at forced waits (metadata, raw rows, LUT gathers + LDS stores)
#ifdef FRA_WSTAMP_FINE
#define FRA_WSTAMP_WAIT(k)                                      \
  {                                                             \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
    FRA_WSTAMP(k)                                               \
  }
#endif
#endif
#ifndef FRA_WSTAMP
#define FRA_WSTAMP(k)
#define FRA_WSTAMP_VAL(k, v)
#endif
#ifndef FRA_WSTAMP_WAIT
#define FRA_WSTAMP_WAIT(k) {}
#endif
// phase-stop diagnostic builds (csrc/Makefile `wstops`, tools/pmc_stall_phases.sh): every subframe is first
// described as VERBATIM (valid sizes: the frame scan and the assembly stay inside their buffers; the bytes
// are meaningless), then the wave returns after phase k, keeping that phase's results alive through the
// descriptor's unused cval
#ifdef FRA_WSTOP
#define FRA_WSTOP_AT(k, keep)                      \
  if (FRA_WSTOP == (k)) {                          \
    if (lane == 0) d->cval = (int32_t)(keep);      \
    return;                                        \
  }
#define FRA_WSTOP_AT_T(k, keep)                    \
  if (FRA_WSTOP == (k)) {                          \
    if (lane == 0) d->cval = (int32_t)(keep);      \
    return true;                                   \
  }
#else
#define FRA_WSTOP_AT(k, keep)
#define FRA_WSTOP_AT_T(k, keep)
#endif

// ---------------------------------------------------------------- frame header (RFC 9639 9.1)
__host__ __device__ inline int utf8_len(uint32_t v) {
  if (v < 0x80) return 1;
  if (v < 0x800) return 2;
  if (v < 0x10000) return 3;
  if (v < 0x200000) return 4;
  if (v < 0x4000000) return 5;
  return 6;
}
__device__ inline int frame_header(uint8_t* h, const StreamDev& st, const FrameDev& fr, int chan_code) {
  int bsx, srx, srv;
  const int bc = bs_code(fr.n, &bsx);
  const int sc = sr_code(st.sample_rate, &srx, &srv);
  int p = 0;
  h[p++] = 0xFF;
  h[p++] = 0xF8;
  h[p++] = (uint8_t)((bc << 4) | sc);
  h[p++] = (uint8_t)((chan_code << 4) | (bps_code(st.bps) << 1));
  const uint32_t v = (uint32_t)fr.index + st.frame_number0;
  const int nb = utf8_len(v);
  if (nb == 1) h[p++] = (uint8_t)v;
  else {
    h[p++] = (uint8_t)(((0xFF00u >> nb) & 0xFF) | (v >> (6 * (nb - 1))));
    for (int i = nb - 2; i >= 0; i--) h[p++] = (uint8_t)(0x80 | ((v >> (6 * i)) & 0x3F));
  }
  if (bsx == 8) h[p++] = (uint8_t)(fr.n - 1);
  else if (bsx == 16) { h[p++] = (uint8_t)((fr.n - 1) >> 8); h[p++] = (uint8_t)(fr.n - 1); }
  if (srx == 8) h[p++] = (uint8_t)srv;
  else if (srx == 16) { h[p++] = (uint8_t)(srv >> 8); h[p++] = (uint8_t)srv; }
  return p;
}
__device__ inline int frame_header_len(const StreamDev& st, const FrameDev& fr) {
  int bsx, srx, srv;
  bs_code(fr.n, &bsx);
  sr_code(st.sample_rate, &srx, &srv);
  return 4 + utf8_len((uint32_t)fr.index + st.frame_number0) + bsx / 8 + srx / 8 + 1;  // + CRC-8
}

}  // namespace fra
