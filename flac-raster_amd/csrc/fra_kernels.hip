// fra_kernels.hip -- CDNA4 (gfx950) kernels of the FLAC raster encode path.
//
// Replaces the libFLAC 1.4.3 encoder that pyflac.StreamEncoder.process()/finish() drives at
// src/flac_raster/converter.py:139-154 and src/flac_raster/spatial_encoder.py:291-304, fused with
// normalize_to_audio (src/flac_raster/normalization.py:126-202) and the band interleave
// (converter.py:99-110 / spatial_encoder.py:209-213).  The decisions follow the FRA-1 rule of
// DESIGN.md section 3, restated independently on the CPU in oracle/fr_oracle.c; every kernel
// here must produce byte-identical streams to that oracle.
//
// Kernels (launch order per job):
//   k_norm_init   per stream: reset min/max keys
//   k_minmax      per (row segment, stream): nanmin/nanmax over all bands of the window (a3)
//   k_analyze     per (frame, channel) = subframe: normalise, wasted bits, windows,
//                 autocorrelation, Levinson-Durbin, qlp, model search, exact Rice bits -> SfDesc
//   k_frame_bytes per frame: header + subframe bits + pad + CRC-16 -> bytes
//   (hipcub exclusive scan of frame bytes -> frame byte offsets)
//   k_pack        per frame: re-read + re-normalise, residual of the chosen model, bit-pack into
//                 an LDS bit buffer, flush to HBM at the frame's byte offset, CRC-8/CRC-16
//
// Numerics: compiled with -ffp-contract=off; every float/double expression on the decision path
// is evaluated in exactly the order the oracle uses (IEEE add/mul/div are correctly rounded on
// gfx950 and on x86-64, so identical op sequences give identical bits).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fra_internal.h"

#pragma clang fp contract(off)

namespace fra {

// ============================================================================ helpers
__device__ __forceinline__ unsigned long long okey(double v) {
  unsigned long long b = (unsigned long long)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double unkey(unsigned long long k) {
  unsigned long long b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double((long long)b);
}

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
  else if constexpr (SRC == ST_U8) return (int32_t)((const uint8_t*)base)[e];
  else if constexpr (SRC == ST_I8) return (int32_t)((const int8_t*)base)[e];
  else if constexpr (SRC == ST_U16) return (int32_t)((const uint16_t*)base)[e];
  else if constexpr (SRC == ST_U32) return (int32_t)((const uint32_t*)base)[e];
  else return 0;
}

// normalize_to_audio for one value (normalization.py:162-187), op order as numpy evaluates it
__device__ __forceinline__ int32_t norm_sample(double x, double mn, double range, double scale, bool to16) {
  double t = x - mn;
  t = 2.0 * t;
  t = t / range;
  t = t - 1.0;
  if (t < -1.0) t = -1.0;
  else if (t > 1.0) t = 1.0;
  if (t != t) t = 0.0;
  t = t * scale;
  return to16 ? (int32_t)(int16_t)(int32_t)t : (int32_t)t;
}

struct NormParams {
  double mn, range, scale;
  bool to16;
  int mode;  // 0 raw ints, else normalise
};
__device__ __forceinline__ NormParams norm_params(const StreamDev& st, const NormDev& nd) {
  NormParams p;
  p.mode = st.norm;
  p.to16 = st.norm == 16;
  p.scale = st.norm == 16 ? 32767.0 : 8388607.0;
  double mn, mx;
  if (nd.mnkey == ~0ull) {  // no non-NaN value: nanmin/nanmax -> NaN
    mn = __longlong_as_double(0x7FF8000000000000ll);
    mx = mn;
  } else {
    mn = unkey(nd.mnkey);
    mx = unkey(nd.mxkey);
  }
  p.mn = mn;
  p.range = (mx <= mn) ? 1.0 : (mx - mn);
  return p;
}

template <int SRC>
__device__ __forceinline__ int32_t fetch_sample(const void* base, int64_t e, const NormParams& np) {
  if (np.mode == 0) return load_raw_int<SRC>(base, e);
  return norm_sample(load_f64<SRC>(base, e), np.mn, np.range, np.scale, np.to16);
}

// element offset of sample i of channel c of frame fr
__device__ __forceinline__ int64_t sample_elem(const StreamDev& st, const FrameDev& fr, int c, int i) {
  int col = fr.col0 + i;
  int row = fr.row0;
  if (col >= st.width) {
    int q = (unsigned)col / (unsigned)st.width;
    row += q;
    col -= q * st.width;
  }
  return st.base_off + (int64_t)c * st.band_stride + (int64_t)row * st.row_stride + (int64_t)col * st.col_stride;
}

__device__ __forceinline__ uint64_t zz64(int64_t r) {
  return r >= 0 ? ((uint64_t)r << 1) : ((((uint64_t)(-(r + 1))) << 1) | 1u);
}
__device__ __forceinline__ int bitlen64(uint64_t v) { return v ? 64 - __clzll((long long)v) : 0; }

// Rice parameter estimate, identical to oracle rice_pick/rice_est2
__device__ __forceinline__ uint64_t rice_est2(uint64_t n, uint64_t S, int k) {
  uint64_t lo = n * (uint64_t)((1u << k) - 1u);
  uint64_t tail = (2 * S > lo) ? ((2 * S - lo) >> (k + 1)) : 0;
  return n * (uint64_t)(k + 1) + tail;
}
__device__ __forceinline__ void rice_pick(uint64_t n, uint64_t S, int& k_out, uint64_t& bits_out) {
  uint64_t mean = n ? S / n : 0;
  int kc = bitlen64(mean);
  int lo = kc - 2 < 0 ? 0 : kc - 2, hi = kc + 1 > 30 ? 30 : kc + 1;
  uint64_t best = rice_est2(n, S, lo);
  int bk = lo;
  for (int k = lo + 1; k <= hi; k++) {
    uint64_t e = rice_est2(n, S, k);
    if (e < best) { best = e; bk = k; }
  }
  k_out = bk;
  bits_out = best;
}

// 64-bit wave reductions via 32-bit halves
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  for (int off = 32; off >= 1; off >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, off, 64);
    uint32_t hi = __shfl_xor((uint32_t)(v >> 32), off, 64);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
  uint32_t lo = __shfl((uint32_t)v, src, 64);
  uint32_t hi = __shfl((uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}

// deterministic log2 -- same op sequence as oracle ora_det_log2
__device__ double det_log2(double x) {
  int e;
  double m = frexp(x, &e);
  m = m * 2.0;
  e = e - 1;
  double t = (m - 1.0) / (m + 1.0);
  double t2 = t * t;
  double sum = 0.0, p = t;
  for (int k = 0; k < 12; k++) {
    sum = sum + p / (double)(2 * k + 1);
    p = p * t2;
  }
  return (double)e + 2.0 * sum * 1.4426950408889634;
}

__device__ int best_order_by_error(const double* err, int norders, int n, int overhead) {
  double best = 0.0;
  int bo = 1;
  for (int o = 1; o <= norders; o++) {
    double e = err[o - 1], bps;
    if (e > 0.0) {
      bps = 0.5 * det_log2(0.5 * e / (double)n);
      if (bps < 0.0) bps = 0.0;
    } else if (e < 0.0) bps = 1e32;
    else bps = 0.0;
    double bits = bps * (double)(n - o) + (double)(o * overhead);
    if (o == 1 || bits < best) { best = bits; bo = o; }
  }
  return bo;
}

// Levinson-Durbin -- same op sequence as oracle ora_levinson
__device__ int levinson(const double* autoc, int max_order, double (*lp)[kMaxLpc], double* err_out) {
  double lpc[kMaxLpc];
  double err = autoc[0];
  for (int i = 0; i < max_order; i++) {
    double r = -autoc[i + 1];
    for (int j = 0; j < i; j++) r = r - lpc[j] * autoc[i - j];
    r = r / err;
    lpc[i] = r;
    int j;
    for (j = 0; j < (i >> 1); j++) {
      double tmp = lpc[j];
      lpc[j] = lpc[j] + r * lpc[i - 1 - j];
      lpc[i - 1 - j] = lpc[i - 1 - j] + r * tmp;
    }
    if (i & 1) lpc[j] = lpc[j] + lpc[j] * r;
    err = err * (1.0 - r * r);
    for (j = 0; j <= i; j++) lp[i][j] = -lpc[j];
    err_out[i] = err;
    if (err > 0.0) continue;
    return err == 0.0 ? i + 1 : i;
  }
  return max_order;
}

__device__ __forceinline__ double rnd_half_away(double x) {
  double t = trunc(x);
  double d = x - t;
  if (d >= 0.5) t = t + 1.0;
  else if (d <= -0.5) t = t - 1.0;
  return t;
}

// qlp quantisation with error feedback; returns false if not representable
__device__ bool quantize(const double* lp, int order, int precision, int32_t* q, int& shift_out) {
  double cmax = 0.0;
  for (int j = 0; j < order; j++) {
    double a = fabs(lp[j]);
    if (a > cmax) cmax = a;
  }
  if (!(cmax > 0.0)) return false;
  int e;
  (void)frexp(cmax, &e);
  int shift = precision - 1 - e;
  if (shift > 15) shift = 15;
  if (shift < 0) return false;
  int32_t qmax = (1 << (precision - 1)) - 1, qmin = -(1 << (precision - 1));
  double errf = 0.0;
  for (int j = 0; j < order; j++) {
    errf = errf + ldexp(lp[j], shift);
    double qd = rnd_half_away(errf);
    int32_t qi = (int32_t)qd;
    if (qi > qmax) qi = qmax;
    if (qi < qmin) qi = qmin;
    errf = errf - (double)qi;
    q[j] = qi;
  }
  shift_out = shift;
  return true;
}

// ============================================================================ k_norm_init / k_minmax
__global__ void k_norm_init(NormDev* nd, int nstreams) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nstreams) {
    nd[i].mnkey = ~0ull;
    nd[i].mxkey = 0ull;
  }
}

// grid: x = row segment (row * segs_per_row + seg), y = stream.  nanmin/nanmax over all bands.
template <int SRC>
__global__ void __launch_bounds__(256) k_minmax(const void* raster, const StreamDev* streams, NormDev* nd) {
  const StreamDev st = streams[blockIdx.y];
  if (st.norm == 0) return;
  const int segs = (st.width + 4095) >> 12;
  const int seg = blockIdx.x;
  if (seg >= segs * st.height) return;
  const int row = seg / segs, c0 = (seg - row * segs) << 12;
  const int c1 = min(st.width, c0 + 4096);
  unsigned long long kmin = ~0ull, kmax = 0ull;
  for (int b = 0; b < st.channels; b++) {
    const int64_t rb = st.base_off + (int64_t)b * st.band_stride + (int64_t)row * st.row_stride;
    for (int col = c0 + threadIdx.x; col < c1; col += 256) {
      double v = load_f64<SRC>(raster, rb + (int64_t)col * st.col_stride);
      if (v == v) {
        unsigned long long k = okey(v);
        kmin = k < kmin ? k : kmin;
        kmax = k > kmax ? k : kmax;
      }
    }
  }
  for (int off = 32; off >= 1; off >>= 1) {
    unsigned long long a = ((unsigned long long)__shfl_xor((uint32_t)(kmin >> 32), off, 64) << 32) |
                           __shfl_xor((uint32_t)kmin, off, 64);
    unsigned long long b = ((unsigned long long)__shfl_xor((uint32_t)(kmax >> 32), off, 64) << 32) |
                           __shfl_xor((uint32_t)kmax, off, 64);
    kmin = a < kmin ? a : kmin;
    kmax = b > kmax ? b : kmax;
  }
  __shared__ unsigned long long smn[4], smx[4];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { smn[wv] = kmin; smx[wv] = kmax; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; w++) {
      kmin = smn[w] < kmin ? smn[w] : kmin;
      kmax = smx[w] > kmax ? smx[w] : kmax;
    }
    if (kmin != ~0ull) {
      atomicMin(&nd[blockIdx.y].mnkey, kmin);
      atomicMax(&nd[blockIdx.y].mxkey, kmax);
    }
  }
}

// ============================================================================ k_analyze
// LDS layout (bytes): samples 16 KiB | windowed floats / partition sums 16.5 KiB | small tables
struct AnalyzeSmem {
  int32_t smp[kMaxBlock];
  union {
    float wf[kMaxBlock + 32];
    unsigned long long psum[kMaxModels][kMaxPart];
    unsigned long long esum[kMaxPart][3];
  } u;
  double red[4][kMaxLpc + 1];
  double autoc[kMaxLpc + 1];
  double lp[kMaxLpc][kMaxLpc];
  double err[kMaxLpc];
  int32_t mcoef[kMaxModels][kMaxLpc];
  int32_t mtype[kMaxModels], morder[kMaxModels], mshift[kMaxModels], mvalid[kMaxModels], mporder[kMaxModels];
  unsigned long long mest[kMaxModels];
  uint32_t ired[4][3];
  int32_t kpart[kMaxPart];
  int32_t nord, olo, ohi, winner;
};

// residual for sample at register position jj (x[12 + jj] is the sample), model m
template <bool B32>
__device__ __forceinline__ int64_t model_residual(const int32_t* x, int jj, int type, int o, const int32_t* q, int shift) {
  const int b = 12 + jj;
  if (type == 2) {
    if constexpr (B32) {
      int64_t s0 = x[b], s1 = x[b - 1], s2 = x[b - 2], s3 = x[b - 3], s4 = x[b - 4];
      switch (o) {
        case 0: return s0;
        case 1: return s0 - s1;
        case 2: return s0 - 2 * s1 + s2;
        case 3: return s0 - 3 * s1 + 3 * s2 - s3;
        default: return s0 - 4 * s1 + 6 * s2 - 4 * s3 + s4;
      }
    } else {
      int32_t s0 = x[b], s1 = x[b - 1], s2 = x[b - 2], s3 = x[b - 3], s4 = x[b - 4];
      switch (o) {
        case 0: return s0;
        case 1: return s0 - s1;
        case 2: return s0 - 2 * s1 + s2;
        case 3: return s0 - 3 * s1 + 3 * s2 - s3;
        default: return s0 - 4 * s1 + 6 * s2 - 4 * s3 + s4;
      }
    }
  } else {
    if constexpr (B32) {
      int64_t sum = 0;
#pragma unroll
      for (int j = 0; j < kMaxLpc; j++)
        if (j < o) sum += (int64_t)q[j] * (int64_t)x[b - 1 - j];
      return (int64_t)x[b] - (sum >> shift);
    } else {
      int32_t sum = 0;
#pragma unroll
      for (int j = 0; j < kMaxLpc; j++)
        if (j < o) sum += q[j] * x[b - 1 - j];
      return (int64_t)(x[b] - (sum >> shift));
    }
  }
}

template <int SRC, bool B32>
__global__ void __launch_bounds__(kThreads) k_analyze(JobArgs a) {
  __shared__ AnalyzeSmem S;
  const int g = blockIdx.x, c = blockIdx.y, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const FrameDev fr = a.frames[g];
  const StreamDev st = a.streams[fr.stream];
  if (c >= st.channels) return;
  const int n = fr.n;
  const int bps = st.bps;
  const LevelCfg cfg = level_cfg(a.level);
  const NormParams np = norm_params(st, a.norm[fr.stream]);
  SfDesc* d = &a.sf[(size_t)g * a.cmax + c];

  // ---- 1. load + normalise (coalesced: lane-contiguous samples)
  uint32_t orv = 0;
  int32_t vmin = INT32_MAX, vmax = INT32_MIN;
  for (int i = t; i < n; i += kThreads) {
    int32_t v = fetch_sample<SRC>(a.raster, sample_elem(st, fr, c, i), np);
    S.smp[i] = v;
    orv |= (uint32_t)v;
    vmin = min(vmin, v);
    vmax = max(vmax, v);
  }
  for (int off = 32; off >= 1; off >>= 1) {
    orv |= __shfl_xor(orv, off, 64);
    vmin = min(vmin, __shfl_xor(vmin, off, 64));
    vmax = max(vmax, __shfl_xor(vmax, off, 64));
  }
  if (lane == 0) { S.ired[wv][0] = orv; S.ired[wv][1] = (uint32_t)vmin; S.ired[wv][2] = (uint32_t)vmax; }
  __syncthreads();
  orv = S.ired[0][0] | S.ired[1][0] | S.ired[2][0] | S.ired[3][0];
  vmin = min(min((int32_t)S.ired[0][1], (int32_t)S.ired[1][1]), min((int32_t)S.ired[2][1], (int32_t)S.ired[3][1]));
  vmax = max(max((int32_t)S.ired[0][2], (int32_t)S.ired[1][2]), max((int32_t)S.ired[2][2], (int32_t)S.ired[3][2]));

  // ---- 2. CONSTANT (3.2)
  if (vmin == vmax) {
    if (t == 0) {
      d->type = 0; d->order = 0; d->wasted = 0; d->sbps = (uint8_t)bps; d->cval = vmin;
      d->bits = 8u + (uint32_t)bps; d->porder = 0; d->method = 0; d->precision = 0; d->shift = 0;
    }
    return;
  }
  // ---- 3. wasted bits (3.3)
  const int w = __builtin_ctz(orv);
  const int sbps = bps - w;
  if (w) {
    __syncthreads();
    for (int i = t; i < n; i += kThreads) S.smp[i] = S.smp[i] >> w;
  }
  const uint64_t hdr = 8u + (uint64_t)(w ? w : 0);
  const uint64_t verb = hdr + (uint64_t)n * (uint64_t)sbps;
  __syncthreads();

  // register window: x[12 + jj] = sample 16t + jj, x[0..11] = the 12 preceding samples
  int32_t x[12 + kChunk];
  const int i0 = t * kChunk;
#pragma unroll
  for (int j = 0; j < 12 + kChunk; j++) {
    int i = i0 - 12 + j;
    x[j] = (i >= 0 && i < n) ? S.smp[i] : 0;
  }

  // ---- 4. model table: fixed orders
  const int fmax = n - 1 < 4 ? n - 1 : 4;
  if (t < kMaxModels) {
    S.mvalid[t] = 0;
    S.mtype[t] = t < 5 ? 2 : 3;
    S.morder[t] = t < 5 ? t : 0;
    S.mshift[t] = 0;
    if (t < 5 && t <= fmax) S.mvalid[t] = 1;
  }
  // ---- 5. LPC analysis per window (3.4-3.7)
  const int lmax = cfg.max_lpc < n - 1 ? cfg.max_lpc : n - 1;
  const int prec = qlp_precision(bps, n);
  if (cfg.nsub > 0 && lmax > 0) {
    for (int wi = 0; wi < a.nwin; wi++) {
      const float* win = a.win + ((size_t)fr.win * a.nwin + wi) * a.blocksize;
      __syncthreads();
      for (int i = t; i < n + 32; i += kThreads) S.u.wf[i] = (i < n) ? (float)S.smp[i] * win[i] : 0.0f;
      __syncthreads();
      float wl[kChunk + kMaxLpc];
#pragma unroll
      for (int j = 0; j < kChunk + kMaxLpc; j++) wl[j] = S.u.wf[i0 + j];
      // FRA-1 chunk partials: per lag, sequential over the thread's 16 samples.  The product of two
      // floats is exact in double, so fma(a, b, acc) == acc + a*b bit for bit (oracle op order).
      double acc[kMaxLpc + 1];
#pragma unroll
      for (int l = 0; l <= kMaxLpc; l++) acc[l] = 0.0;
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) {
        const double a0 = (double)wl[jj];
#pragma unroll
        for (int l = 0; l <= kMaxLpc; l++)
          if (l <= lmax && i0 + jj + l < n) acc[l] = fma(a0, (double)wl[jj + l], acc[l]);
      }
      // pairwise tree over the 256 chunk partials: strides 1..32 in-wave, 64/128 across waves
#pragma unroll
      for (int l = 0; l <= kMaxLpc; l++) {
        if (l > lmax) continue;
        double v = acc[l];
        for (int off = 1; off < 64; off <<= 1) {
          double o = __shfl_down(v, off, 64);
          v = v + o;
        }
        if (lane == 0) S.red[wv][l] = v;
      }
      __syncthreads();
      if (t == 0) {
        for (int l = 0; l <= lmax; l++) S.autoc[l] = (S.red[0][l] + S.red[1][l]) + (S.red[2][l] + S.red[3][l]);
        int nord = 0;
        if (S.autoc[0] != 0.0) nord = levinson(S.autoc, lmax, S.lp, S.err);
        int olo = 1, ohi = nord;
        if (wi > 0 && nord > 0) { olo = ohi = best_order_by_error(S.err, nord, n, prec + sbps); }
        S.nord = nord; S.olo = olo; S.ohi = ohi;
      }
      __syncthreads();
      const int nord = S.nord, olo = S.olo, ohi = S.ohi;
      if (nord > 0) {
        const int o = olo + t;
        if (t < kMaxLpc && o <= ohi) {
          const int m = wi == 0 ? 5 + o - 1 : 5 + kMaxLpc + wi - 1;
          int32_t q[kMaxLpc];
          int sh = 0;
          bool ok = quantize(S.lp[o - 1], o, prec, q, sh);
          S.mtype[m] = 3; S.morder[m] = o; S.mshift[m] = sh; S.mvalid[m] = ok ? 1 : 0;
          for (int j = 0; j < kMaxLpc; j++) S.mcoef[m][j] = (ok && j < o) ? q[j] : 0;
        }
      }
    }
  }
  __syncthreads();

  // ---- 6. residual partition sums at the finest level P for every valid model (3.8)
  const int P = max_porder(n, 0, cfg.max_porder);
  const int psz = n >> P;
  for (int i = t; i < kMaxModels * kMaxPart; i += kThreads) (&S.u.psum[0][0])[i] = 0ull;
  __syncthreads();
  for (int m = 0; m < kMaxModels; m++) {
    if (!S.mvalid[m]) continue;  // uniform (LDS)
    const int type = S.mtype[m], o = S.morder[m], sh = S.mshift[m];
    int32_t q[kMaxLpc];
#pragma unroll
    for (int j = 0; j < kMaxLpc; j++) q[j] = S.mcoef[m][j];
    int pidx = i0 < n ? i0 / psz : 0;
    int pend = (pidx + 1) * psz;
    uint64_t acc = 0;
    bool ovf = false;
#pragma unroll
    for (int jj = 0; jj < kChunk; jj++) {
      const int i = i0 + jj;
      if (i < n && i >= o) {
        if (i >= pend) {
          if (acc) atomicAdd(&S.u.psum[m][pidx], (unsigned long long)acc);
          acc = 0;
          pidx = i / psz;
          pend = (pidx + 1) * psz;
        }
        int64_t r = model_residual<B32>(x, jj, type, o, q, sh);
        if constexpr (B32) ovf |= (r > INT32_MAX || r < INT32_MIN);
        acc += zz64(r);
      }
    }
    if (acc) atomicAdd(&S.u.psum[m][pidx], (unsigned long long)acc);
    if constexpr (B32) {
      if (__any(ovf) && lane == 0) S.mvalid[m] = 0;  // benign race: every writer stores 0
    }
  }
  __syncthreads();

  // ---- 7. best partition order per model (one wave per model)
  for (int m = wv; m < kMaxModels; m += 4) {
    if (!S.mvalid[m]) continue;
    const int o = S.morder[m];
    const int pm = max_porder(n, o, cfg.max_porder);
    uint64_t Sj = lane < (1 << P) ? S.u.psum[m][lane] : 0ull;
    for (int p = P - 1; p >= pm; p--) {
      uint64_t a0 = shfl_u64(Sj, (2 * lane) & 63), a1 = shfl_u64(Sj, (2 * lane + 1) & 63);
      Sj = lane < (1 << p) ? a0 + a1 : 0ull;
    }
    uint64_t best = 0;
    int bp = pm;
    for (int p = pm; p >= 0; p--) {
      const int npp = 1 << p;
      uint64_t bits = 0;
      int k = 0;
      if (lane < npp) {
        uint64_t cnt = (uint64_t)((n >> p) - (lane == 0 ? o : 0));
        rice_pick(cnt, Sj, k, bits);
      }
      const bool big = __any(lane < npp && k > 14);
      uint64_t tot = wave_sum_u64(bits) + (uint64_t)npp * (big ? 5 : 4) + 6;
      if (p == pm || tot <= best) { best = tot; bp = p; }
      uint64_t a0 = shfl_u64(Sj, (2 * lane) & 63), a1 = shfl_u64(Sj, (2 * lane + 1) & 63);
      Sj = lane < (npp >> 1) ? a0 + a1 : 0ull;
    }
    if (lane == 0) {
      const bool lpc = S.mtype[m] == 3;
      S.mest[m] = hdr + (uint64_t)o * sbps + (lpc ? 9 + (uint64_t)o * prec : 0) + best;
      S.mporder[m] = bp;
    }
  }
  __syncthreads();
  if (t == 0) {
    int win = -1;
    uint64_t be = 0;
    for (int m = 0; m < kMaxModels; m++) {
      if (!S.mvalid[m]) continue;
      if (win < 0 || S.mest[m] < be) { be = S.mest[m]; win = m; }
    }
    S.winner = win;
  }
  __syncthreads();

  // ---- 8. exact Rice bits for the winner (3.9): k per partition refined over k-1..k+1
  const int m = S.winner;
  const int type = S.mtype[m], o = S.morder[m], sh = S.mshift[m], ps = S.mporder[m];
  if (wv == 0) {
    uint64_t Sj = lane < (1 << P) ? S.u.psum[m][lane] : 0ull;
    for (int p = P - 1; p >= ps; p--) {
      uint64_t a0 = shfl_u64(Sj, (2 * lane) & 63), a1 = shfl_u64(Sj, (2 * lane + 1) & 63);
      Sj = lane < (1 << p) ? a0 + a1 : 0ull;
    }
    if (lane < (1 << ps)) {
      uint64_t cnt = (uint64_t)((n >> ps) - (lane == 0 ? o : 0));
      int k;
      uint64_t bits;
      rice_pick(cnt, Sj, k, bits);
      S.kpart[lane] = k;
    }
  }
  __syncthreads();
  for (int i = t; i < kMaxPart * 3; i += kThreads) (&S.u.esum[0][0])[i] = 0ull;
  __syncthreads();
  {
    int32_t q[kMaxLpc];
#pragma unroll
    for (int j = 0; j < kMaxLpc; j++) q[j] = S.mcoef[m][j];
    const int pz = n >> ps;
    int pidx = i0 < n ? i0 / pz : 0, pend = (pidx + 1) * pz;
    int k = S.kpart[pidx];
    uint64_t e0 = 0, e1 = 0, e2 = 0;
#pragma unroll
    for (int jj = 0; jj < kChunk; jj++) {
      const int i = i0 + jj;
      if (i < n && i >= o) {
        if (i >= pend) {
          atomicAdd(&S.u.esum[pidx][0], (unsigned long long)e0);
          atomicAdd(&S.u.esum[pidx][1], (unsigned long long)e1);
          atomicAdd(&S.u.esum[pidx][2], (unsigned long long)e2);
          e0 = e1 = e2 = 0;
          pidx = i / pz;
          pend = (pidx + 1) * pz;
          k = S.kpart[pidx];
        }
        uint64_t u = zz64(model_residual<B32>(x, jj, type, o, q, sh));
        e0 += k > 0 ? (u >> (k - 1)) : 0;
        e1 += u >> k;
        e2 += u >> (k + 1);
      }
    }
    if (i0 < n) {
      atomicAdd(&S.u.esum[pidx][0], (unsigned long long)e0);
      atomicAdd(&S.u.esum[pidx][1], (unsigned long long)e1);
      atomicAdd(&S.u.esum[pidx][2], (unsigned long long)e2);
    }
  }
  __syncthreads();
  if (wv == 0) {
    const int npp = 1 << ps;
    uint64_t best = 0;
    int bk = 0;
    if (lane < npp) {
      const uint64_t cnt = (uint64_t)((n >> ps) - (lane == 0 ? o : 0));
      const int k0 = S.kpart[lane];
      bool first = true;
      for (int kk = k0 - 1; kk <= k0 + 1; kk++) {
        if (kk < 0 || kk > 30) continue;
        uint64_t e = cnt * (uint64_t)(kk + 1) + S.u.esum[lane][kk - k0 + 1];
        if (first || e < best) { best = e; bk = kk; first = false; }
      }
    }
    const bool big = __any(lane < npp && bk > 14);
    const uint64_t tot = wave_sum_u64(lane < npp ? best : 0ull) + (uint64_t)npp * (big ? 5 : 4) + 6;
    const uint64_t exact = hdr + (uint64_t)o * sbps + (type == 3 ? 9 + (uint64_t)o * prec : 0) + tot;
    const bool verbatim = exact >= verb;
    if (lane < npp) d->k[lane] = (uint8_t)bk;
    if (lane < kMaxLpc) d->coef[lane] = S.mcoef[m][lane];
    if (lane == 0) {
      d->wasted = (uint8_t)w;
      d->sbps = (uint8_t)sbps;
      d->cval = 0;
      if (verbatim) {
        d->type = 1; d->order = 0; d->porder = 0; d->method = 0; d->precision = 0; d->shift = 0;
        d->bits = (uint32_t)verb;
      } else {
        d->type = (uint8_t)type; d->order = (uint8_t)o; d->porder = (uint8_t)ps; d->method = big ? 1 : 0;
        d->precision = (uint8_t)(type == 3 ? prec : 0); d->shift = (int8_t)sh;
        d->bits = (uint32_t)exact;
      }
    }
  }
}

// ============================================================================ frame header
__device__ __host__ inline int utf8_len(uint32_t v) {
  if (v < 0x80) return 1;
  if (v < 0x800) return 2;
  if (v < 0x10000) return 3;
  if (v < 0x200000) return 4;
  if (v < 0x4000000) return 5;
  return 6;
}
// writes header bytes (without CRC-8) into h, returns length
__device__ inline int frame_header(uint8_t* h, const StreamDev& st, const FrameDev& fr) {
  int bsx, srx, srv;
  const int bc = bs_code(fr.n, &bsx);
  const int sc = sr_code(st.sample_rate, &srx, &srv);
  int p = 0;
  h[p++] = 0xFF;
  h[p++] = 0xF8;
  h[p++] = (uint8_t)((bc << 4) | sc);
  h[p++] = (uint8_t)(((st.channels - 1) << 4) | (bps_code(st.bps) << 1));
  const uint32_t v = (uint32_t)fr.index;
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
  return 4 + utf8_len((uint32_t)fr.index) + bsx / 8 + srx / 8 + 1;  // + CRC-8
}

__global__ void k_frame_bytes(JobArgs a) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g > a.nframes_total) return;
  if (g == a.nframes_total) { a.frame_bytes[g] = 0; return; }  // scan input tail
  const FrameDev fr = a.frames[g];
  const StreamDev st = a.streams[fr.stream];
  uint64_t bits = (uint64_t)frame_header_len(st, fr) * 8;
  for (int c = 0; c < st.channels; c++) bits += a.sf[(size_t)g * a.cmax + c].bits;
  a.frame_bytes[g] = ((bits + 7) >> 3) + 2;
}

// ============================================================================ k_pack
__device__ __forceinline__ uint32_t gf_mul16(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int i = 15; i >= 0; i--) {
    r <<= 1;
    if (r & 0x10000u) r ^= 0x18005u;
    if ((b >> i) & 1u) r ^= a;
  }
  return r & 0xFFFFu;
}

constexpr int kBufWords = kMaxBlock + 16;  // >= max subframe bits (< 4096*32 + 64) / 32 + carry

struct PackSmem {
  int32_t smp[kMaxBlock];
  uint32_t buf[kBufWords];
  uint16_t crctab[256];
  uint32_t xpow[40];      // x^(2^i) mod P
  uint32_t scan[4];
  uint32_t crcred[4];
  uint32_t crc;           // running CRC-16 of flushed bytes
  uint32_t carry;
  SfDesc desc;
  uint8_t hdr[24];
};

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

// Flush buf[0..nfull) = frame-local words [wbase, wbase+nfull) to HBM at byte F + 4*wbase and fold
// their bytes into the running CRC-16.  Whole block participates.
__device__ void flush_words(PackSmem& S, int nfull, uint8_t* out, uint64_t F, int wbase) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  for (int j = t; j < nfull; j += kThreads) {
    const uint32_t v = S.buf[j];
    uint8_t* p = out + F + 4ull * (uint64_t)(wbase + j);
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
  }
  if (nfull == 0) return;
  // parallel CRC: virtual sequence = (pad zero words) ++ buf[0..nfull), split into 256 groups of G words
  int lg = 0;
  while ((kThreads << lg) < nfull) lg++;
  const int G = 1 << lg;
  const int pad = kThreads * G - nfull;
  uint32_t c = 0;
  for (int v = t * G; v < (t + 1) * G; v++) {
    const int j = v - pad;
    if (j < 0) continue;
    const uint32_t wd = S.buf[j];
#pragma unroll
    for (int b = 3; b >= 0; b--) c = ((c << 8) ^ S.crctab[((c >> 8) ^ (wd >> (8 * b))) & 0xFF]) & 0xFFFF;
  }
  // tree: level l combines (left, right) with right length G*2^l words = 32*G*2^l bits -> x^(2^(5+lg+l))
  for (int l = 0; l < 6; l++) {
    const uint32_t r = __shfl_down(c, 1 << l, 64);
    if ((lane & ((2 << l) - 1)) == 0) c = gf_mul16(c, S.xpow[5 + lg + l]) ^ r;
  }
  if (lane == 0) S.crcred[wv] = c;
  __syncthreads();
  if (t == 0) {
    uint32_t c01 = gf_mul16(S.crcred[0], S.xpow[5 + lg + 6]) ^ S.crcred[1];
    uint32_t c23 = gf_mul16(S.crcred[2], S.xpow[5 + lg + 6]) ^ S.crcred[3];
    uint32_t cc = gf_mul16(c01, S.xpow[5 + lg + 7]) ^ c23;
    // fold: crc = crc * x^(32*nfull) ^ cc
    uint32_t f = S.crc;
    for (int b = 0; b < 20; b++)
      if ((nfull >> b) & 1) f = gf_mul16(f, S.xpow[5 + b]);
    S.crc = f ^ cc;
  }
}

template <int SRC, bool B32>
__global__ void __launch_bounds__(kThreads) k_pack(JobArgs a) {
  __shared__ PackSmem S;
  const int g = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const FrameDev fr = a.frames[g];
  const StreamDev st = a.streams[fr.stream];
  const int n = fr.n;
  const NormParams np = norm_params(st, a.norm[fr.stream]);
  const uint64_t F = a.frame_off[g];
  uint8_t* out = a.out;

  // CRC tables
  {
    uint32_t dd = (uint32_t)t << 8;
    for (int b = 0; b < 8; b++) dd = (dd & 0x8000u) ? ((dd << 1) ^ 0x8005u) : (dd << 1);
    S.crctab[t] = (uint16_t)dd;
  }
  if (t == 0) {
    uint32_t xp = 2;  // x
    for (int i = 0; i < 40; i++) { S.xpow[i] = xp; xp = gf_mul16(xp, xp); }
    S.crc = 0;
    S.carry = 0;
    // frame header + CRC-8
    int hl = frame_header(S.hdr, st, fr);
    uint32_t c8 = 0;
    for (int i = 0; i < hl; i++) {
      c8 ^= S.hdr[i];
      for (int b = 0; b < 8; b++) c8 = (c8 & 0x80u) ? ((c8 << 1) ^ 0x07u) : (c8 << 1);
      c8 &= 0xFF;
    }
    S.hdr[hl] = (uint8_t)c8;
    S.hdr[23] = (uint8_t)(hl + 1);
  }
  for (int j = t; j < kBufWords; j += kThreads) S.buf[j] = 0;
  __syncthreads();
  const int hbytes = S.hdr[23];
  if (t < hbytes) {
    const int b = t;
    atomicOr(&S.buf[b >> 2], (uint32_t)S.hdr[b] << (24 - 8 * (b & 3)));
  }
  __syncthreads();
  uint32_t fbit = (uint32_t)hbytes * 8;
  flush_words(S, (int)(fbit >> 5), out, F, 0);
  if (t == 0) S.carry = (fbit & 31) ? S.buf[fbit >> 5] : 0;
  __syncthreads();

  for (int c = 0; c < st.channels; c++) {
    if (t == 0) S.desc = a.sf[(size_t)g * a.cmax + c];
    // load + normalise channel c
    for (int i = t; i < n; i += kThreads) S.smp[i] = fetch_sample<SRC>(a.raster, sample_elem(st, fr, c, i), np);
    __syncthreads();
    const SfDesc& d = S.desc;
    const int type = d.type, w = d.wasted, sbps = d.sbps, o = d.order;
    const uint32_t obit = fbit & 31, wbase = fbit >> 5;
    const uint32_t nw = (obit + d.bits + 31) >> 5;
    for (uint32_t j = t; j <= nw; j += kThreads) S.buf[j] = (j == 0) ? S.carry : 0u;
    if (type != 0 && w) {
      for (int i = t; i < n; i += kThreads) S.smp[i] = S.smp[i] >> w;
    }
    __syncthreads();
    const uint32_t smask = sbps >= 32 ? 0xFFFFFFFFu : ((1u << sbps) - 1u);
    const uint32_t hdrbits = 8u + (uint32_t)((type != 0 && w) ? w : 0);
    if (t == 0) {
      const int tcode = type == 0 ? 0 : type == 1 ? 1 : type == 2 ? 8 + o : 31 + o;
      lds_put(S.buf, obit, (uint32_t)(tcode << 1) | ((type != 0 && w) ? 1u : 0u), 8);
      if (type != 0 && w) lds_put(S.buf, obit + 8 + (uint32_t)(w - 1), 1u, 1);
      if (type == 0) lds_put(S.buf, obit + 8, (uint32_t)d.cval & smask, sbps);
    }
    if (type == 1) {
      for (int i = t; i < n; i += kThreads)
        lds_put(S.buf, obit + hdrbits + (uint32_t)i * sbps, (uint32_t)S.smp[i] & smask, sbps);
    } else if (type >= 2) {
      for (int i = t; i < o; i += kThreads)
        lds_put(S.buf, obit + hdrbits + (uint32_t)i * sbps, (uint32_t)S.smp[i] & smask, sbps);
      uint32_t pos = obit + hdrbits + (uint32_t)o * sbps;
      if (type == 3) {
        if (t == 0) {
          lds_put(S.buf, pos, (uint32_t)(d.precision - 1), 4);
          lds_put(S.buf, pos + 4, (uint32_t)d.shift & 31u, 5);
        }
        if (t < o)
          lds_put(S.buf, pos + 9 + (uint32_t)t * d.precision, (uint32_t)d.coef[t] & ((1u << d.precision) - 1u),
                  d.precision);
        pos += 9 + (uint32_t)o * d.precision;
      }
      if (t == 0) lds_put(S.buf, pos, ((uint32_t)d.method << 4) | d.porder, 6);
      pos += 6;
      // residual codes: thread owns samples [16t, 16t+16)
      const int pb = d.method ? 5 : 4;
      const int pz = n >> d.porder;
      const int i0 = t * kChunk;
      int32_t x[12 + kChunk];
#pragma unroll
      for (int j = 0; j < 12 + kChunk; j++) {
        int i = i0 - 12 + j;
        x[j] = (i >= 0 && i < n) ? S.smp[i] : 0;
      }
      int32_t q[kMaxLpc];
#pragma unroll
      for (int j = 0; j < kMaxLpc; j++) q[j] = d.coef[j];
      uint32_t u[kChunk];
      uint32_t len[kChunk];
      uint32_t tot = 0;
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) {
        const int i = i0 + jj;
        u[jj] = 0;
        len[jj] = 0;
        if (i < n && i >= o) {
          const int pidx = i / pz;
          const int k = d.k[pidx];
          const uint64_t uu = zz64(model_residual<B32>(x, jj, type, o, q, d.shift));
          u[jj] = (uint32_t)uu;
          const bool pstart = (pidx == 0) ? (i == o) : (i == pidx * pz);
          len[jj] = (uint32_t)(uu >> k) + 1u + (uint32_t)k + (pstart ? (uint32_t)pb : 0u);
          tot += len[jj];
        }
      }
      // block exclusive scan of tot
      uint32_t inc = tot;
      for (int off = 1; off < 64; off <<= 1) {
        uint32_t v = __shfl_up(inc, off, 64);
        if (lane >= off) inc += v;
      }
      if (lane == 63) S.scan[wv] = inc;
      __syncthreads();
      uint32_t base = inc - tot;
      for (int ww = 0; ww < wv; ww++) base += S.scan[ww];
      uint32_t p = pos + base;
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) {
        const int i = i0 + jj;
        if (i < n && i >= o) {
          const int pidx = i / pz;
          const int k = d.k[pidx];
          const bool pstart = (pidx == 0) ? (i == o) : (i == pidx * pz);
          uint32_t pp = p;
          if (pstart) { lds_put(S.buf, pp, (uint32_t)k, pb); pp += pb; }
          const uint32_t qv = u[jj] >> k;
          const uint32_t code = (k == 0) ? 1u : ((1u << k) | (u[jj] & ((1u << k) - 1u)));
          lds_put(S.buf, pp + qv, code, k + 1);
          p += len[jj];
        }
      }
    }
    __syncthreads();
    const uint32_t endbit = obit + d.bits;
    flush_words(S, (int)(endbit >> 5), out, F, (int)wbase);
    __syncthreads();
    if (t == 0) S.carry = (endbit & 31) ? S.buf[endbit >> 5] : 0u;
    fbit += d.bits;
    __syncthreads();
  }
  // pad to byte, flush the tail bytes of the carry word, append CRC-16
  if (t == 0) {
    const uint32_t fend = (fbit + 7) & ~7u;
    const uint32_t wb = fbit >> 5;
    const int nb = (int)((fend >> 3) - 4 * wb);
    uint32_t crc = S.crc;
    const uint32_t cw = S.carry;
    for (int b = 0; b < nb; b++) {
      const uint8_t by = (uint8_t)(cw >> (24 - 8 * b));
      out[F + 4ull * wb + b] = by;
      crc = ((crc << 8) ^ S.crctab[((crc >> 8) ^ by) & 0xFF]) & 0xFFFF;
    }
    out[F + (fend >> 3)] = (uint8_t)(crc >> 8);
    out[F + (fend >> 3) + 1] = (uint8_t)crc;
  }
}

// ============================================================================ launchers
#define FRA_SRC_CASES(M) M(ST_U8) M(ST_I8) M(ST_U16) M(ST_I16) M(ST_U32) M(ST_I32) M(ST_F32) M(ST_F64)

__global__ void k_norm_finalize(const StreamDev* streams, NormDev* nd, int nstreams) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nstreams) return;
  NormParams p = norm_params(streams[i], nd[i]);
  nd[i].mn = p.mn;
  nd[i].mx = nd[i].mnkey == ~0ull ? p.mn : unkey(nd[i].mxkey);
  nd[i].range = p.range;
}

hipError_t launch_norm_finalize(const JobArgs& a, int nstreams, hipStream_t s) {
  k_norm_finalize<<<(nstreams + 255) / 256, 256, 0, s>>>(a.streams, a.norm, nstreams);
  return hipGetLastError();
}

hipError_t launch_minmax(int src, const JobArgs& a, int nstreams, int max_segs, hipStream_t s) {
  k_norm_init<<<(nstreams + 255) / 256, 256, 0, s>>>(a.norm, nstreams);
  dim3 grid((unsigned)max_segs, (unsigned)nstreams);
  switch (src) {
#define M(S_) case S_: k_minmax<S_><<<grid, 256, 0, s>>>(a.raster, a.streams, a.norm); break;
    FRA_SRC_CASES(M)
#undef M
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_analyze(int src, bool b32, const JobArgs& a, hipStream_t s) {
  dim3 grid((unsigned)a.nframes_total, (unsigned)a.cmax);
  switch (src) {
#define M(S_)                                                          \
  case S_:                                                             \
    if (b32) k_analyze<S_, true><<<grid, kThreads, 0, s>>>(a);         \
    else k_analyze<S_, false><<<grid, kThreads, 0, s>>>(a);            \
    break;
    FRA_SRC_CASES(M)
#undef M
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_frame_bytes(const JobArgs& a, hipStream_t s) {
  k_frame_bytes<<<(a.nframes_total + 1 + 255) / 256, 256, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_pack(int src, bool b32, const JobArgs& a, hipStream_t s) {
  dim3 grid((unsigned)a.nframes_total);
  switch (src) {
#define M(S_)                                                       \
  case S_:                                                          \
    if (b32) k_pack<S_, true><<<grid, kThreads, 0, s>>>(a);         \
    else k_pack<S_, false><<<grid, kThreads, 0, s>>>(a);            \
    break;
    FRA_SRC_CASES(M)
#undef M
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace fra
