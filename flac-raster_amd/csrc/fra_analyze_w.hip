// fra_analyze_w.hip -- k_analyze_w: the 16-bit analysis with one subframe per WAVE.
//
// Replaces, like k_analyze (fra_analyze.hip), libFLAC 1.4.3's per-channel analysis inside
// FLAC__stream_encoder_process_interleaved (driven by pyflac at src/flac_raster/converter.py:153 /
// spatial_encoder.py:303), fused with normalize_to_audio (normalization.py:126-202) and the band
// interleave (converter.py:99-110).  Decision rule FRA-1 == oracle/fr_oracle.c
// analyze_subframe(), bit for bit the same bytes as k_analyze.
//
// Scope: full 4096-sample frames of a <= 16-bit integer raster whose normalisation goes through the
// per-tile table (k_norm_lut), 8-byte sample vectors, levels 0-6 (lag <= 8, <= 3 apodization windows):
// the C3/C4 workloads.  Everything else (partial last frames, raw int16 input, levels 7-8, 32-bps and
// the mid-side virtual channels) stays on k_analyze; the launcher routes the partial frames there
// through a frame list.
//
// Why a wave and not a workgroup: k_analyze's 256-thread workgroup spends 43 % of its wave cycles
// parked at s_waitcnt / s_barrier -- eight barriers per subframe, Levinson-Durbin on 16
// lanes of one wave and the partition search on one wave while the others wait.  Here a wave owns its
// subframe end to end: no workgroup barrier, no single-wave phase, no per-wave duplicated bookkeeping.
// Lane l processes the 16-sample chunks t = 64 j + l, j = 0..3: iteration j is exactly wave j of
// k_analyze, so every FRA-1 reduction order (the chunk-partial tree per 64 chunks, then
// (G0 + G1) + (G2 + G3)) is unchanged.
//
// LDS per wave (9.6 KiB, 64-thread workgroups): the int16 samples in chunks of 8 dwords, dword d of chunk
// t at 8 + 8t + 2 (t >> 3) + d (2 pad dwords per 8 chunks: the 8-byte reads of 32 lanes at a 32-byte
// stride hit 64 distinct banks; d stays an immediate offset), a zero chunk in front (samples before the block)
// and a spare one behind (look-ahead of the last chunk, multiplied by zero window coefficients); the
// encoded subframe's bit buffer aliases the samples once the winner's residuals are in registers; a
// 1.25 KiB scratch holds partition sums and the partition-search nodes.
#include "fra_device.h"

namespace fra {

namespace {

constexpr int kWChunks = kMaxBlock / kChunk;  // 256
constexpr int kWIters = kWChunks / 64;        // chunks per lane

struct WaveSmem {
  uint32_t sw[8 + 8 * (kWChunks + 1) + 2 * (kWChunks / 8)];  // zero chunk, 256 chunks (+ pads), spare chunk
  unsigned long long scr[160];          // FIXED partition sums (u32 [5][64]) / LPC sums / search nodes
};
// the bit buffer: <= 2,049 words (exact < verbatim = 8 + 65,536 bits) + one spare zeroed word
static_assert(sizeof(WaveSmem::sw) >= 4 * 2050, "bit buffer inside the sample array");

__device__ __forceinline__ int sdw(int t, int d) { return 8 + 8 * t + 2 * (t >> 3) + d; }
__device__ __forceinline__ int32_t wsample(const uint32_t* sw, int s) {
  const uint32_t v = sw[sdw(s >> 4, (s & 15) >> 1)];
  return (s & 1) ? hi16(v) : lo16(v);
}
__device__ __forceinline__ void wsync() {  // this wave's LDS stores -> its own reads
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
}
// D[0..5] = the last 12 samples of chunk t - 1, D[6..13] = chunk t (int16 pairs, sample 16t - 12 + 2k in
// the low half of D[k]) -- the layout read_d14 gives k_analyze
__device__ __forceinline__ void wread_d14(const uint32_t* sw, int t, uint32_t (&D)[14]) {
#pragma unroll
  for (int p = 0; p < 3; p++) {
    const uint2 v = *reinterpret_cast<const uint2*>(&sw[sdw(t - 1, 2 + 2 * p)]);
    D[2 * p] = v.x;
    D[2 * p + 1] = v.y;
  }
#pragma unroll
  for (int p = 0; p < 4; p++) {
    const uint2 v = *reinterpret_cast<const uint2*>(&sw[sdw(t, 2 * p)]);
    D[6 + 2 * p] = v.x;
    D[7 + 2 * p] = v.y;
  }
}
__device__ __forceinline__ void unpack28(const uint32_t (&D)[14], int32_t (&x)[28]) {
#pragma unroll
  for (int k = 0; k < 14; k++) {
    x[2 * k] = lo16(D[k]);
    x[2 * k + 1] = hi16(D[k]);
  }
}
// upper-lane group sums over aligned groups of 2^ls lanes (ls <= 6, runtime), result at the group's
// last lane
__device__ __forceinline__ uint32_t group_sum32(uint32_t v, int ls) {
  if (ls > 0) v = up_add32<0>(v);
  if (ls > 1) v = up_add32<1>(v);
  if (ls > 2) v = up_add32<2>(v);
  if (ls > 3) v = up_add32<3>(v);
  if (ls > 4) v = up_add32<4>(v);
  if (ls > 5) v = up_add32<5>(v);
  return v;
}
__device__ __forceinline__ uint64_t group_sum64(uint64_t v, int ls) {
  if (ls > 0) v = up_add64<0>(v);
  if (ls > 1) v = up_add64<1>(v);
  if (ls > 2) v = up_add64<2>(v);
  if (ls > 3) v = up_add64<3>(v);
  if (ls > 4) v = up_add64<4>(v);
  if (ls > 5) v = up_add64<5>(v);
  return v;
}
// group sums of per-lane values that may exceed 32 bits together: 32-bit adds when no group can
// overflow (every lane below 2^(32 - ls)), else 64-bit
__device__ __forceinline__ uint64_t group_sum_auto(uint64_t v, int ls) {
  if (__all(v < (1ull << (32 - ls)))) return group_sum32((uint32_t)v, ls);
  return group_sum64(v, ls);
}
__device__ __forceinline__ double rdlane_f64(double v, int l) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// autocorr_reduce_wave (fra_device.h) without the store: the same reduce-scatter, the lag sums left in
// z[k] at lanes 16r + 15; kLagK / kLagR say where lag L ends up
template <int NL>
__device__ __forceinline__ void autocorr_reduce_regs(const double (&acc)[NL], double (&z)[((NL + 1) / 2 + 1) / 2]) {
  constexpr int N32 = (NL + 1) / 2, N16 = (N32 + 1) / 2;
  double w[N32];
#pragma unroll
  for (int k = 0; k < N32; k++) {
    double x = acc[2 * k], y = (2 * k + 1 < NL) ? acc[2 * k + 1] : acc[2 * k];
    swap32_f64(x, y);
    w[k] = x + y;
  }
#pragma unroll
  for (int k = 0; k < N16; k++) {
    double x = w[2 * k], y = (2 * k + 1 < N32) ? w[2 * k + 1] : w[2 * k];
    swap16_f64(x, y);
    double v = x + y;
    v = v + dppf64<DPP_SHR8, 0xF>(v);
    v = v + dppf64<DPP_SHR4, 0xF>(v);
    v = v + dppf64<DPP_SHR2, 0xF>(v);
    v = v + dppf64<DPP_SHR1, 0xF>(v);
    z[k] = v;
  }
}
template <int NL>
__host__ __device__ constexpr int lag_slot(int lag) {  // (k << 2) | r of the first slot holding lag
  constexpr int N32 = (NL + 1) / 2, N16 = (N32 + 1) / 2;
  for (int k = 0; k < N16; k++)
    for (int r = 0; r < 4; r++) {
      const int wi = (2 * k + 1 < N32) ? 2 * k + (r & 1) : 2 * k;
      const int l = (2 * wi + 1 < NL) ? 2 * wi + (r >> 1) : 2 * wi;
      if (l == lag) return (k << 2) | r;
    }
  return -1;
}

// Levinson-Durbin (op sequence of levinson_wave / oracle ora_levinson) where each lane also keeps the
// coefficient row of ITS order lo (row of order lo = lpc after step lo - 1), so the rows need no LDS
template <int MAXLAG>
__device__ inline int levinson_keep(const double (&ac)[MAXLAG + 1], int max_order, double (&errv)[MAXLAG],
                                    double (&row)[MAXLAG], int lo) {
  double lpc[MAXLAG];
#pragma unroll
  for (int j = 0; j < MAXLAG; j++) { lpc[j] = 0.0; errv[j] = 0.0; row[j] = 0.0; }
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
      const bool mine = lo == i + 1;
#pragma unroll
      for (int j = 0; j <= i; j++) row[j] = mine ? lpc[j] : row[j];
      errv[i] = err;
      if (!(err > 0.0)) {
        result = (err == 0.0) ? i + 1 : i;
        done = true;
      }
    }
  }
  return result;
}

// FRA-1 3.7 FIXED candidates from register partition sums (lane p < 2^P: partition p of order k) ==
// fixed_guess2 (fra_analyze.hip) with every order valid (n = 4096)
__device__ __forceinline__ void fixed_guess2_w(const uint32_t (&ps)[5], int P, int lane, int& g1, int& g2) {
  uint64_t T[5];
  bool small = true;
  uint32_t pv[5];
#pragma unroll
  for (int k = 0; k < 5; k++) {
    pv[k] = lane < (1 << P) ? ps[k] : 0u;
    small = small && pv[k] < (1u << 25);
  }
  if (__all(small)) {
#pragma unroll
    for (int k = 0; k < 5; k++) T[k] = wave_sum32(pv[k]);
  } else {
#pragma unroll
    for (int k = 0; k < 5; k++) {
      uint64_t v = pv[k];
      v = up_add64<0>(v); v = up_add64<1>(v); v = up_add64<2>(v);
      v = up_add64<3>(v); v = up_add64<4>(v); v = up_add64<5>(v);
      T[k] = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    }
  }
  int h1 = -1, h2 = -1;
  uint64_t b1 = 0, b2 = 0;
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const bool lt1 = h1 < 0 || T[k] < b1;
    const bool lt2 = !lt1 && (h2 < 0 || T[k] < b2);
    b2 = lt1 ? b1 : (lt2 ? T[k] : b2);
    h2 = lt1 ? h1 : (lt2 ? k : h2);
    b1 = lt1 ? T[k] : b1;
    h1 = lt1 ? k : h1;
  }
  g1 = __builtin_amdgcn_readfirstlane(h1);
  g2 = __builtin_amdgcn_readfirstlane(h2);
}

// porder_search (fra_analyze.hip) on a register of finest partition sums (lane p < 2^P), node sums in the
// wave's scratch; returns the best total, its order and, in kreg lane j < 2^bp, partition j's Rice parameter
__device__ __forceinline__ void porder_search_w(uint64_t Sv, unsigned long long* node, int P, int pm, int n, int o,
                                                int lane, uint64_t& best_out, int& bp_out, uint32_t& kreg) {
  const bool narrow = __all(Sv < (1ull << 23));
  uint32_t bits32 = 0;
  bool big = false;
  int kn = 0;
  const int p = lane ? 31 - __clz(lane) : 0;
  uint32_t tot6 = 0;
  bool big6 = false;
  int k6 = 0;
  if (narrow) {  // every node sum < 2^29: 32-bit arithmetic (rice_pick32), bit-identical
    uint32_t* nd = reinterpret_cast<uint32_t*>(node);
    uint32_t S = (uint32_t)Sv;
    if (lane < (1 << P)) nd[(1 << P) + lane] = S;
#define FRA_NODE_STEP32(S_)                                                        \
  if (P > S_) {                                                                    \
    S = up_add32<S_>(S);                                                           \
    if (lane < (1 << P) && ((lane + 1) & ((2 << S_) - 1)) == 0)                    \
      nd[(1 << (P - S_ - 1)) + (lane >> (S_ + 1))] = S;                            \
  }
    FRA_NODE_STEP32(0) FRA_NODE_STEP32(1) FRA_NODE_STEP32(2)
    FRA_NODE_STEP32(3) FRA_NODE_STEP32(4) FRA_NODE_STEP32(5)
#undef FRA_NODE_STEP32
    wsync();
    if (lane >= 1 && p <= P && p <= pm) {
      const int j = lane - (1 << p);
      rice_pick32((uint32_t)((n >> p) - (j == 0 ? o : 0)), nd[lane], kn, bits32);
      big = kn > 14;
    }
    if (P == 6 && pm == 6) {
      uint32_t b6;
      rice_pick32((uint32_t)((n >> 6) - (lane == 0 ? o : 0)), nd[64 + lane], k6, b6);
      tot6 = wave_sum32(b6);
      big6 = __any(k6 > 14);
    }
  } else {
    uint64_t S = Sv;
    if (lane < (1 << P)) node[(1 << P) + lane] = S;
#define FRA_NODE_STEP(S_)                                                          \
  if (P > S_) {                                                                    \
    S = up_add64<S_>(S);                                                           \
    if (lane < (1 << P) && ((lane + 1) & ((2 << S_) - 1)) == 0)                    \
      node[(1 << (P - S_ - 1)) + (lane >> (S_ + 1))] = S;                          \
  }
    FRA_NODE_STEP(0) FRA_NODE_STEP(1) FRA_NODE_STEP(2)
    FRA_NODE_STEP(3) FRA_NODE_STEP(4) FRA_NODE_STEP(5)
#undef FRA_NODE_STEP
    wsync();
    if (lane >= 1 && p <= P && p <= pm) {
      const int j = lane - (1 << p);
      uint64_t bits;
      rice_pick((uint64_t)((n >> p) - (j == 0 ? o : 0)), node[lane], kn, bits);
      bits32 = (uint32_t)bits;
      big = kn > 14;
    }
    if (P == 6 && pm == 6) {
      uint64_t b6;
      rice_pick((uint64_t)((n >> 6) - (lane == 0 ? o : 0)), node[64 + lane], k6, b6);
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
  uint64_t best = 0;
  int bp = pm;
  for (int q = pm; q >= 0; q--) {
    const bool bq = q == 6 ? big6 : ((bigm >> (1u << q)) & ((1ull << (1u << q)) - 1)) != 0;
    const uint64_t t = (uint64_t)tot[q] + (uint64_t)(1u << q) * (bq ? 5 : 4) + 6;
    if (q == pm || t <= best) { best = t; bp = q; }
  }
  best_out = best;
  bp_out = bp;
  // partition j's parameter at order bp: node (bp, j) sits at lane 2^bp + j (level 6: k6 at lane j)
  const int kl = __shfl(kn, ((1 << (bp < 6 ? bp : 0)) + lane) & 63, 64);
  kreg = (uint32_t)(bp == 6 ? k6 : kl);
  wsync();  // the node reads are done before the next search reuses the scratch
}

// LUT fast load of one channel of a full frame into the swizzled chunks (load_lut_full_t, per wave):
// lane l loads the 8-byte vectors l + 64k (all issued before the first use), gathers each sample's audio
// value from the tile's table, packs int16 pairs and stores 4 samples per ds_write_b64
template <int SRC>
__device__ __forceinline__ void wload_lut(const void* base, const StreamDev& st, const FrameDev& fr, int c,
                                          const int32_t* lut, uint32_t* sw, int lane, uint32_t& orv, int32_t& vmin,
                                          int32_t& vmax) {
  using T = typename RawType<SRC>::T;
  constexpr int V = 8 / (int)sizeof(T);
  constexpr int NV = kMaxBlock / 64 / V;
  constexpr int step = 64 * V;
  using VT = VecT<T, V>;
  const int w = st.width;
  const char* b0 = (const char*)((const T*)base + st.base_off + (int64_t)c * st.band_stride + (int64_t)fr.row0 * st.row_stride);
  const uint32_t rsb = (uint32_t)st.row_stride * (uint32_t)sizeof(T);
  int col = fr.col0 + lane * V;
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
  uint32_t orp = 0;
  i16x2 pmin = {32767, 32767}, pmax = {-32768, -32768};
#pragma unroll
  for (int kv = 0; kv < NV; kv++) {
    int32_t g[V];
#pragma unroll
    for (int e = 0; e < V; e++) g[e] = lut[lut_index<SRC>(x[kv].v[e])];
    const int i = (lane + 64 * kv) * V;
#pragma unroll
    for (int h = 0; h < V / 4; h++) {
      const int s = i + 4 * h;
      const uint32_t p0 = __builtin_amdgcn_perm((uint32_t)g[4 * h + 1], (uint32_t)g[4 * h], 0x05040100u);
      const uint32_t p1 = __builtin_amdgcn_perm((uint32_t)g[4 * h + 3], (uint32_t)g[4 * h + 2], 0x05040100u);
      *reinterpret_cast<uint2*>(&sw[sdw(s >> 4, (s & 15) >> 1)]) = make_uint2(p0, p1);
      orp |= p0 | p1;
      const i16x2 a0 = __builtin_bit_cast(i16x2, p0), a1 = __builtin_bit_cast(i16x2, p1);
      pmin = __builtin_elementwise_min(pmin, __builtin_elementwise_min(a0, a1));
      pmax = __builtin_elementwise_max(pmax, __builtin_elementwise_max(a0, a1));
    }
  }
  orv |= (orp | (orp >> 16)) & 0xFFFFu;
  vmin = min(vmin, min((int32_t)pmin.x, (int32_t)pmin.y));
  vmax = max(vmax, max((int32_t)pmax.x, (int32_t)pmax.y));
}

// 16-bit path: sum of |LPC residual| of order O over one chunk (lpc_abs16_raw without the kept residuals)
template <int O>
__device__ __forceinline__ uint32_t lpc_abs16_w(const uint32_t (&D)[14], const int32_t* q, int sh, bool head) {
  constexpr int NP = (O + 1) / 2;
  fra_short2 Q[NP];
  q_pairs_rev<NP>(q, Q);
  uint32_t acc = 0;
#pragma unroll
  for (int jj = 0; jj < kChunk; jj++) {
    const int32_t r = sample_at(D, 12 + jj) - (pred_raw<NP>(D, 12 + jj, Q) >> sh);
    const uint32_t rb = (uint32_t)r ^ kBias;
    acc = sad_acc(rb, (jj < O && head) ? rb : kBias, acc);
  }
  return acc;
}

}  // namespace

template <int MAXLAG>
__global__ void __launch_bounds__(64, 4) k_analyze_w(JobArgs a, int src) {
  static_assert(MAXLAG == 0 || MAXLAG == 8, "levels 0-6");
  __shared__ WaveSmem S;
  uint32_t* const sw = S.sw;
  const int lane = (int)threadIdx.x;
  const int g = a.frame_base + (int)blockIdx.x;
  const int c = (int)blockIdx.y;
  const FrameDev fr = a.frames[g];
  if (fr.n != kMaxBlock) return;  // partial frames: k_analyze over the frame list
  const StreamDev st = a.streams[fr.stream];
  if (c >= (st.ms ? 2 : st.channels)) return;
  constexpr int n = kMaxBlock;
  const int bps = st.bps;
  const LevelCfg cfg = level_cfg(a.level);
  SfDesc* d = &a.sf[(size_t)g * a.cmax + c];
  uint32_t* const slot = a.tmp + ((size_t)g * a.cmax + c) * a.tmp_stride;

  // ---- 1. load + normalise (table gather), OR / min / max
  uint32_t orv = 0;
  int32_t vmin = INT32_MAX, vmax = INT32_MIN;
  {
    const int32_t* lut = a.lut + (int64_t)fr.stream * a.lut_stride;
    if (lane < 8) sw[lane] = 0u;  // zero chunk
    switch (src) {  // wave-uniform
      case ST_U8: wload_lut<ST_U8>(a.raster, st, fr, c, lut, sw, lane, orv, vmin, vmax); break;
      case ST_I8: wload_lut<ST_I8>(a.raster, st, fr, c, lut, sw, lane, orv, vmin, vmax); break;
      case ST_U16: wload_lut<ST_U16>(a.raster, st, fr, c, lut, sw, lane, orv, vmin, vmax); break;
      default: wload_lut<ST_I16>(a.raster, st, fr, c, lut, sw, lane, orv, vmin, vmax); break;
    }
  }
  orv = wave_or32(orv);
  vmin = (int32_t)(wave_min32((uint32_t)vmin ^ 0x80000000u) ^ 0x80000000u);
  vmax = (int32_t)(~wave_min32(~((uint32_t)vmax ^ 0x80000000u)) ^ 0x80000000u);

  // ---- 2. CONSTANT / wasted bits (3.2, 3.3)
  if (vmin == vmax) {
    if (lane == 0) {
      d->type = 0; d->order = 0; d->wasted = 0; d->sbps = (uint8_t)bps; d->cval = vmin;
      d->bits = 8u + (uint32_t)bps; d->porder = 0; d->method = 0; d->precision = 0; d->shift = 0;
      const uint64_t v = (uint64_t)(uint32_t)vmin & ((1ull << bps) - 1);
      const uint64_t blob = v << (64 - 8 - bps);
      slot[0] = (uint32_t)(blob >> 32);
      slot[1] = (uint32_t)blob;
    }
    return;
  }
  const int w = __builtin_ctz(orv);
  const int sbps = bps - w;
  if (w) {  // samples >>= w (int16 pairs, arithmetic; the pad dwords too)
    for (int k = lane; k < sdw(kWChunks, 0) - 8; k += 64) {
      const uint32_t v = sw[8 + k];
      const uint32_t lo = (uint32_t)(lo16(v) >> w) & 0xFFFFu, hi = (uint32_t)(hi16(v) >> w);
      sw[8 + k] = lo | (hi << 16);
    }
  }
  wsync();
  const uint32_t hdr = 8u + (uint32_t)w;
  const uint32_t verb = hdr + (uint32_t)n * (uint32_t)sbps;
  const int P = max_porder(n, 0, cfg.max_porder);  // = cfg.max_porder (3..6)
  const int gsl = 8 - P;                             // lanes per finest partition: 2^gsl (chunks of 16)
  const int prec = qlp_precision(bps, n);
  const int lmax = cfg.max_lpc;                      // < n - 1

  // ---- 3a. FIXED residual sums (3.8) by finite differences, per finest partition
  uint32_t* const scr32 = reinterpret_cast<uint32_t*>(S.scr);
  for (int j = 0; j < kWIters; j++) {
    const int t = 64 * j + lane;
    const bool head = t == 0;
    uint32_t D[14];
    wread_d14(sw, t, D);
    int32_t x[28];
    unpack28(D, x);
#pragma unroll
    for (int k = 0; k <= 4; k++) {
      if (k > 1) {
#pragma unroll
        for (int jx = 12 + kChunk - 1; jx >= 7 + k; jx--) x[jx] = x[jx] - x[jx - 1];
      }
      uint32_t s32 = 0;
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) {
        const uint32_t ab = (uint32_t)x[12 + jj] ^ kBias;
        const uint32_t bb = k == 0 ? kBias : ((jj < k && head) ? ab : (uint32_t)x[11 + jj] ^ kBias);
        s32 = sad_acc(ab, bb, s32);
      }
      // a partition of <= 512 samples: 2 sum |r| < 2^30
      const uint32_t gs = group_sum32(s32, gsl);
      if ((lane & ((1 << gsl) - 1)) == (1 << gsl) - 1) scr32[k * 64 + (t >> gsl)] = 2u * gs;
    }
  }
  wsync();
  uint32_t pfix[5];
#pragma unroll
  for (int k = 0; k < 5; k++) pfix[k] = lane < (1 << P) ? scr32[k * 64 + lane] : 0u;
  wsync();

  // ---- running winner (FRA-1 3.8: first minimal estimate in model order)
  uint32_t west = 0xFFFFFFFFu;
  int wm = 99, wtype = 2, wo = 0, wsh = 0, wps = 0;
  int32_t wq[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t wk = 0;
  auto offer = [&](uint32_t est, int m, int type, int o, int sh, const int32_t* q, int ps, uint32_t kreg) {
    if (est < west || (est == west && m < wm)) {
      west = est; wm = m; wtype = type; wo = o; wsh = sh; wps = ps; wk = kreg;
#pragma unroll
      for (int jq = 0; jq < 8; jq++) wq[jq] = q ? q[jq] : 0;
    }
  };

  // ---- 5a. FIXED candidates (3.7) and their partition search
  {
    int g1, g2;
    fixed_guess2_w(pfix, P, lane, g1, g2);
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const int m = r == 0 ? g1 : g2;
      if (m < 0) continue;
      uint32_t pm_sum = 0;
#pragma unroll
      for (int k = 0; k < 5; k++) pm_sum = k == m ? pfix[k] : pm_sum;
      const int pm = max_porder(n, m, cfg.max_porder);
      uint64_t best;
      int bp;
      uint32_t kreg;
      porder_search_w(pm_sum, S.scr, P, pm, n, m, lane, best, bp, kreg);
      offer((uint32_t)(hdr + (uint64_t)m * sbps + best), m, 2, m, 0, nullptr, bp, kreg);
    }
  }

  // ---- 3. LPC analysis per apodization window (3.4-3.7)
  if constexpr (MAXLAG > 0) {
    if (cfg.nsub > 0 && lmax > 0) {
      const int nwin = a.nwin;
      constexpr int NL = MAXLAG + 1, N16 = ((NL + 1) / 2 + 1) / 2;
      double acl[NL];
#pragma unroll
      for (int l = 0; l < NL; l++) acl[l] = 0.0;
      for (int wi = 0; wi < nwin; wi++) {
        const int32_t* wr = a.wrange + 2 * ((size_t)fr.win * a.nwin + wi);
        const int32_t* wp = a.wplat + 2 * ((size_t)fr.win * a.nwin + wi);
        const int lo = wr[0], hi = wr[1], plo = wp[0], phi = wp[1];
        const float* win = a.win + ((size_t)fr.win * a.nwin + wi) * a.blocksize;
        double s01[N16], s[N16];
#pragma unroll
        for (int k = 0; k < N16; k++) { s01[k] = 0.0; s[k] = 0.0; }
        for (int j = 0; j < kWIters; j++) {
          double z[N16];
          // an iteration whose samples + look-ahead miss the window's nonzero extent sums exact zeros:
          // every chunk partial is +0.0 (k_analyze's inactive wave)
          if (lo < 1024 * j + 1024 + MAXLAG && hi > 1024 * j) {
            const int t = 64 * j + lane, i0 = kChunk * t;
            // coefficients: exactly 1.0f inside the plateau (the product is the sample itself); else
            // loaded, entries at or past n are 0.0f (load_window)
            float wc[kChunk + MAXLAG];
            const bool plat = i0 >= plo && i0 + kChunk + MAXLAG <= phi;
            if (plat) {
#pragma unroll
              for (int jx = 0; jx < kChunk + MAXLAG; jx++) wc[jx] = 1.0f;
            } else {
              load_window<MAXLAG>(win, i0, n, wc);
            }
            int32_t y[kChunk + MAXLAG];  // samples 16t .. 16t + 15 + MAXLAG (dword pairs: ds_read_b64)
#pragma unroll
            for (int p = 0; p < (kChunk + MAXLAG) / 4; p++) {
              const int tt = p < kChunk / 4 ? t : t + 1, dd = 2 * (p % (kChunk / 4));
              const uint2 v = *reinterpret_cast<const uint2*>(&sw[sdw(tt, dd)]);
              y[4 * p] = lo16(v.x);
              y[4 * p + 1] = hi16(v.x);
              y[4 * p + 2] = lo16(v.y);
              y[4 * p + 3] = hi16(v.y);
            }
            float wf[kChunk + MAXLAG];
#pragma unroll
            for (int jx = 0; jx < kChunk + MAXLAG; jx++) wf[jx] = plat ? (float)y[jx] : (float)y[jx] * wc[jx];
            f32x2 pacc[NL];
#pragma unroll
            for (int l = 0; l < NL; l++) pacc[l] = f32x2{0.0f, 0.0f};
#pragma unroll
            for (int pp = 0; pp < kChunk / 2; pp++) {
              const f32x2 a2 = {wf[2 * pp], wf[2 * pp + 1]};
#pragma unroll
              for (int l = 0; l < NL; l++) {
                const f32x2 b2 = {wf[2 * pp + l], wf[2 * pp + l + 1]};
                pacc[l] = __builtin_elementwise_fma(a2, b2, pacc[l]);
              }
            }
            double acc[NL];
#pragma unroll
            for (int l = 0; l < NL; l++) acc[l] = (double)(pacc[l].x + pacc[l].y);
            autocorr_reduce_regs<NL>(acc, z);
          } else {
#pragma unroll
            for (int k = 0; k < N16; k++) z[k] = 0.0;
          }
          // (G0 + G1) + (G2 + G3) per lag, the order of k_analyze's cross-wave sum
          if (j == 2) {
#pragma unroll
            for (int k = 0; k < N16; k++) s01[k] = s[k];
          }
#pragma unroll
          for (int k = 0; k < N16; k++) s[k] = (j & 1) ? s[k] + z[k] : z[k];
        }
        const int gw = lane >> 4;
#pragma unroll
        for (int l = 0; l < NL; l++) {
          const int sl = lag_slot<NL>(l);
          const double tot = rdlane_f64(s01[sl >> 2] + s[sl >> 2], 16 * (sl & 3) + 15);
          acl[l] = gw == wi ? tot : acl[l];
        }
      }
      // Levinson-Durbin, order choice and quantisation of up to 4 windows at once: window wi on lanes
      // 16 wi .. +15 (the same op sequence per lane); lane 16 wi + o holds order o's row and quantisation
      const int gw = lane >> 4, lo = lane & 15;
      const bool gon = gw < nwin;
      double row[MAXLAG], errv[MAXLAG];
      int nord = 0;
      if (gon && acl[0] != 0.0) nord = levinson_keep<MAXLAG>(acl, lmax, errv, row, lo);
      double e = errv[0];
#pragma unroll
      for (int jx = 1; jx < MAXLAG; jx++)
        if (lo == jx + 1) e = errv[jx];
      const bool on = nord > 0 && lo >= 1 && lo <= nord;
      const uint64_t key = on ? (uint64_t)__double_as_longlong(order_bits(e, n, lo, prec + sbps)) : ~0ull;
      uint64_t rk = min(key, dpp64_old<DPP_SHR1, 0xF>(key, ~0ull));
      rk = min(rk, dpp64_old<DPP_SHR2, 0xF>(rk, ~0ull));
      rk = min(rk, dpp64_old<DPP_SHR4, 0xF>(rk, ~0ull));
      rk = min(rk, dpp64_old<DPP_SHR8, 0xF>(rk, ~0ull));
      const uint64_t kmin = __shfl(rk, (lane & 48) | 15, 64);
      const uint64_t bal = __ballot(on && key == kmin);
      const uint32_t rowbits = (uint32_t)(bal >> (16 * gw)) & 0xFFFFu;
      // every lane quantises its own order's row; the window's model is lane 16 wi + o
      bool ok = false;
      int qsh = 0;
      int32_t q[MAXLAG];
#pragma unroll
      for (int jx = 0; jx < MAXLAG; jx++) q[jx] = 0;
      {
        double lpo[MAXLAG];
#pragma unroll
        for (int jx = 0; jx < MAXLAG; jx++) lpo[jx] = jx < lo ? -row[jx] : 0.0;  // lp = -lpc
        if (on) ok = quantize<MAXLAG>(lpo, lo, prec, q, qsh);
      }
      const int o_l = nord > 0 ? (int)__builtin_ctz(rowbits | 0x10000u) : 0;
      // ---- 4+5. per window: residual sums of the model at the finest partitions, partition search
      for (int wi = 0; wi < nwin; wi++) {
        const int o = __builtin_amdgcn_readlane(o_l, 16 * wi);
        if (o == 0) continue;  // LD found no order (nord 0)
        const int L = 16 * wi + o;
        if (!__builtin_amdgcn_readlane((int)ok, L)) continue;
        const int sh = __builtin_amdgcn_readlane(qsh, L);
        int32_t qm[8];
#pragma unroll
        for (int jx = 0; jx < 8; jx++) qm[jx] = jx < MAXLAG ? __builtin_amdgcn_readlane(q[jx < MAXLAG ? jx : 0], L) : 0;
        for (int j = 0; j < kWIters; j++) {
          const int t = 64 * j + lane;
          const bool head = t == 0;
          uint32_t D[14];
          wread_d14(sw, t, D);
          uint32_t acc = 0;
          switch (o) {
#define FRA_CASE(O_) \
  case O_: acc = lpc_abs16_w<O_>(D, qm, sh, head); break;
            FRA_CASE(1) FRA_CASE(2) FRA_CASE(3) FRA_CASE(4) FRA_CASE(5) FRA_CASE(6) FRA_CASE(7) FRA_CASE(8)
#undef FRA_CASE
          }
          const uint64_t gs = group_sum_auto(2ull * acc, gsl);
          if ((lane & ((1 << gsl) - 1)) == (1 << gsl) - 1) S.scr[t >> gsl] = gs;
        }
        wsync();
        const uint64_t ps = lane < (1 << P) ? S.scr[lane] : 0ull;
        wsync();
        const int pm = max_porder(n, o, cfg.max_porder);
        uint64_t best;
        int bp;
        uint32_t kreg;
        porder_search_w(ps, S.scr, P, pm, n, o, lane, best, bp, kreg);
        offer((uint32_t)(hdr + (uint64_t)o * sbps + 9 + (uint64_t)o * prec + best), 5 + wi, 3, o, sh, qm, bp, kreg);
      }
    }
  }

  // ---- 6. the winner's residuals (zig-zag, warm-up samples 0), exact Rice bits with k refined (3.9)
  const int type = wtype, o = wo, sh = wsh, ps = wps;
  const int pz = n >> ps;
  const int tl = 8 - ps;                  // log2 chunks per partition (2..8)
  const int ls = tl < 6 ? tl : 6;         // lanes per partition group inside one iteration
  const int npp = 1 << ps;
  int32_t warm = 0;
  if (lane < o) warm = wsample(sw, lane);
  fra_short2 Q[4];
  q_pairs_rev<4>(wq, Q);
  // zig-zag residuals of the winner for chunk 64 j + lane (warm-up positions 0)
  auto residuals = [&](int j, uint32_t (&un)[kChunk]) {
    const int t = 64 * j + lane;
    uint32_t D[14];
    wread_d14(sw, t, D);
    if (type == 3) {
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) un[jj] = zz32(sample_at(D, 12 + jj) - (pred_raw<4>(D, 12 + jj, Q) >> sh));
    } else {  // FIXED: the o-th finite difference in place
      int32_t x[28];
      unpack28(D, x);
#pragma unroll
      for (int k = 1; k <= 4; k++) {
        if (k <= o) {
#pragma unroll
          for (int jx = 12 + kChunk - 1; jx >= 8 + k; jx--) x[jx] = x[jx] - x[jx - 1];
        }
      }
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) un[jj] = zz32(x[12 + jj]);
    }
    if (t == 0) {
#pragma unroll
      for (int jj = 0; jj < 12; jj++)
        if (jj < o) un[jj] = 0u;
    }
  };
  // per iteration (runtime j, explicit selects: no dynamically indexed registers)
  auto sel4 = [](const uint32_t (&v)[kWIters], int j) -> uint32_t {
    return j == 0 ? v[0] : j == 1 ? v[1] : j == 2 ? v[2] : v[3];
  };
  auto set4 = [](uint32_t (&v)[kWIters], int j, uint32_t x) {
#pragma unroll
    for (int jx = 0; jx < kWIters; jx++) v[jx] = jx == j ? x : v[jx];
  };
  uint32_t kc[kWIters] = {0, 0, 0, 0};    // Rice parameter of the lane's chunk of iteration j
  uint32_t fk[kWIters][3];                // sums of u >> (k0 - 1), u >> k0, u >> (k0 + 1) of that chunk
  uint32_t k0r[kWIters] = {0, 0, 0, 0};
  uint32_t bitsl = 0;                     // exact bits of the partitions this lane leads
  bool bigl = false;
  uint64_t E[3] = {0, 0, 0};              // partitions spanning iterations (ps <= 1): running sums
#pragma unroll 1
  for (int j = 0; j < kWIters; j++) {
    const int t = 64 * j + lane;
    uint32_t un[kChunk];
    residuals(j, un);
    const int pidx = t >> tl;
    const int k0 = __shfl((int)wk, pidx & 63, 64);
    const int km = k0 > 0 ? k0 - 1 : 0;
    uint32_t f0 = 0, f1 = 0, f2 = 0;  // u < 2^28: 16 of them fit 32 bits
#pragma unroll
    for (int jj = 0; jj < kChunk; jj++) {
      f0 += un[jj] >> km;
      f1 += un[jj] >> k0;
      f2 += un[jj] >> (k0 + 1);
    }
#pragma unroll
    for (int jx = 0; jx < kWIters; jx++) {
      fk[jx][0] = jx == j ? f0 : fk[jx][0];
      fk[jx][1] = jx == j ? f1 : fk[jx][1];
      fk[jx][2] = jx == j ? f2 : fk[jx][2];
    }
    set4(k0r, j, (uint32_t)k0);
    uint64_t v0, v1, v2;
    if (__all(f0 <= (0xFFFFFFFFu >> ls))) {
      v0 = group_sum32(f0, ls); v1 = group_sum32(f1, ls); v2 = group_sum32(f2, ls);
    } else {
      v0 = group_sum64(f0, ls); v1 = group_sum64(f1, ls); v2 = group_sum64(f2, ls);
    }
    if (tl <= 6) {  // the partition lies inside this iteration: its last lane decides
      int bk = 0;
      if ((lane & ((1 << ls) - 1)) == (1 << ls) - 1) {
        const uint64_t cnt = (uint64_t)(pz - (pidx == 0 ? o : 0));
        const uint64_t ev[3] = {v0, v1, v2};
        uint64_t best = 0;
        bool first = true;
#pragma unroll
        for (int dk = -1; dk <= 1; dk++) {
          const int kk = k0 + dk;
          if (kk < 0 || kk > 30) continue;
          const uint64_t e = cnt * (uint64_t)(kk + 1) + ev[dk + 1];
          if (first || e < best) { best = e; bk = kk; first = false; }
        }
        bitsl += (uint32_t)best;
        bigl = bigl || bk > 14;
        d->k[pidx] = (uint8_t)bk;
      }
      set4(kc, j, (uint32_t)__shfl(bk, lane | ((1 << ls) - 1), 64));
    } else {  // ps <= 1: whole-iteration sums accumulate into the partition's running sums
      auto rl64 = [](uint64_t v) -> uint64_t {
        return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63) |
               ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63) << 32);
      };
      E[0] += rl64(v0);
      E[1] += rl64(v1);
      E[2] += rl64(v2);
      const int span = 1 << (tl - 6);  // iterations per partition (2 or 4)
      if (((j + 1) & (span - 1)) == 0) {  // partition complete: decide its parameter (uniform)
        const int pq = j >> (tl - 6);
        const uint64_t cnt = (uint64_t)(pz - (pq == 0 ? o : 0));
        int bk = 0;
        uint64_t best = 0;
        bool first = true;
#pragma unroll
        for (int dk = -1; dk <= 1; dk++) {
          const int kk = k0 + dk;
          if (kk < 0 || kk > 30) continue;
          const uint64_t e = cnt * (uint64_t)(kk + 1) + E[dk + 1];
          if (first || e < best) { best = e; bk = kk; first = false; }
        }
        if (lane == 0) {
          bitsl += (uint32_t)best;
          d->k[pq] = (uint8_t)bk;
        }
        bigl = bigl || bk > 14;
#pragma unroll
        for (int jx = 0; jx < kWIters; jx++)
          if (jx <= j && jx > j - span) kc[jx] = (uint32_t)bk;
        E[0] = E[1] = E[2] = 0;
      }
    }
  }
  const bool big = __any(bigl);
  const uint64_t rtot = (uint64_t)wave_sum32(bitsl) + (uint64_t)npp * (big ? 5 : 4) + 6;
  const uint64_t exact = hdr + (uint64_t)o * sbps + (type == 3 ? 9 + (uint64_t)o * prec : 0) + rtot;
  const bool verbatim = exact >= verb;
  if (lane < kMaxLpc) {
    int32_t cv = 0;
#pragma unroll
    for (int jq = 0; jq < 8; jq++) cv = lane == jq ? wq[jq] : cv;
    d->coef[lane] = type == 3 ? cv : 0;
  }
  if (lane == 0) {
    d->wasted = (uint8_t)w;
    d->sbps = (uint8_t)sbps;
    d->cval = 0;
    if (verbatim) {
      d->type = 1; d->order = 0; d->porder = 0; d->method = 0; d->precision = 0; d->shift = 0;
      d->bits = verb;
    } else {
      d->type = (uint8_t)type; d->order = (uint8_t)o; d->porder = (uint8_t)ps; d->method = big ? 1 : 0;
      d->precision = (uint8_t)(type == 3 ? prec : 0); d->shift = (int8_t)sh;
      d->bits = (uint32_t)exact;
    }
  }
  const uint32_t smask = (1u << sbps) - 1u;  // sbps <= 16
  if (verbatim) {  // straight from the samples to the slot (the bit buffer is not touched)
    const uint32_t nw = (verb + 31) >> 5;
    for (uint32_t jw = lane; jw < nw; jw += 64) {
      const uint64_t hv = ((uint64_t)(2u | (w ? 1u : 0u)) << 56) | (w ? (1ull << (63 - (8 + w - 1))) : 0ull);
      const int64_t wb = 32 * (int64_t)jw;
      uint32_t word = jw == 0 ? (uint32_t)(hv >> 32) : (jw == 1 ? (uint32_t)hv : 0u);
      const int s0 = wb > (int64_t)hdr ? (int)((wb - (int64_t)hdr) / sbps) : 0;
      for (int s = s0; s < n && (int64_t)hdr + (int64_t)s * sbps < wb + 32; s++) {
        const int64_t rel = (int64_t)hdr + (int64_t)s * sbps - wb;
        const int sft = 32 - (int)rel - sbps;
        const uint64_t v = (uint64_t)((uint32_t)wsample(sw, s) & smask);
        word |= sft >= 0 ? (uint32_t)(v << sft) : (uint32_t)(v >> -sft);
      }
      slot[jw] = word;
    }
    return;
  }

  // ---- 7. encode (RFC 9639 9.2).  Code bits of each chunk from the exact pass's sums; bit position of
  // every iteration's first code (B[j]) known up front
  const uint32_t fbits = (uint32_t)exact;
  const uint32_t nw = (fbits + 31) >> 5;
  const int pb = big ? 5 : 4;
  uint32_t pos = hdr + (uint32_t)o * sbps + (type == 3 ? 9u + (uint32_t)o * prec : 0u);
  uint32_t totl[kWIters];
  uint32_t B[kWIters + 1];
  B[0] = pos + 6;
#pragma unroll
  for (int j = 0; j < kWIters; j++) {
    const int t = 64 * j + lane;
    const uint32_t kcur = kc[j], k0 = k0r[j];
    const uint32_t f = kcur + 1 == k0 ? fk[j][0] : kcur == k0 ? fk[j][1] : fk[j][2];
    const bool pstart = ((t << 4) & (pz - 1)) == 0;
    totl[j] = f + (uint32_t)(kChunk - (t == 0 ? o : 0)) * (kcur + 1u) + (pstart ? (uint32_t)pb : 0u);
    B[j + 1] = B[j] + wave_sum32(totl[j]);
  }
  // The bit buffer aliases the samples and is filled iteration by iteration, each iteration's samples
  // read (its residuals in registers) before its words are zeroed and written.  Iteration j must leave
  // chunk 64 j + 63 intact (iteration j + 1 looks back into it): its last word + the spare one stay below
  // that chunk's first word.  Otherwise (an incompressible start before a compressible rest)
  // the codes go straight to the slot in global memory by atomic ORs.
  bool safe = true;
#pragma unroll
  for (int j = 0; j + 1 < kWIters; j++) safe = safe && (B[j + 1] - 1) / 32 + 2 <= (uint32_t)sdw(64 * j + 63, 0);
  auto put_header = [&](uint32_t* buf) {
    if (lane == 0) {
      const int tcode = type == 2 ? 8 + o : 31 + o;
      lds_put(buf, 0, (uint32_t)(tcode << 1) | (w ? 1u : 0u), 8);
      if (w) lds_put(buf, 8 + (uint32_t)(w - 1), 1u, 1);
    }
    if (lane < o) lds_put(buf, hdr + (uint32_t)lane * sbps, (uint32_t)warm & smask, sbps);
    uint32_t ph = hdr + (uint32_t)o * sbps;
    if (type == 3) {
      if (lane == 0) {
        lds_put(buf, ph, (uint32_t)(prec - 1), 4);
        lds_put(buf, ph + 4, (uint32_t)sh & 31u, 5);
      }
      if (lane < o) {
        int32_t cv = 0;
#pragma unroll
        for (int jq = 0; jq < 8; jq++) cv = lane == jq ? wq[jq] : cv;
        lds_put(buf, ph + 9 + (uint32_t)lane * prec, (uint32_t)cv & ((1u << prec) - 1u), prec);
      }
    }
    if (lane == 0) lds_put(buf, pos, ((uint32_t)(big ? 1 : 0) << 4) | (uint32_t)ps, 6);
  };
  auto put_codes = [&](uint32_t* buf, int j, const uint32_t (&un)[kChunk]) {
    const int t = 64 * j + lane;
    const bool head = t == 0;
    const uint32_t kcur = sel4(kc, j), tot = sel4(totl, j);
    const bool pstart = ((t << 4) & (pz - 1)) == 0;
    const uint32_t Bj = j == 0 ? B[0] : j == 1 ? B[1] : j == 2 ? B[2] : B[3];
    uint32_t p = Bj + wave_incl_scan32(tot) - tot;
    if (pstart) { lds_put(buf, p, kcur, pb); p += (uint32_t)pb; }
    const uint32_t sal = 31u - kcur;
#pragma unroll
    for (int jj = 0; jj < kChunk; jj++) {
      if (!(jj < 12 && head && jj < o)) {
        const uint32_t Pp = p + (un[jj] >> kcur);
        lds_put_al(buf, Pp, (un[jj] << sal) | 0x80000000u);
        p = Pp + 1u + kcur;
      }
    }
  };
  if (safe) {
    uint32_t Z = 0;  // words [0, Z) are zeroed (and possibly written)
#pragma unroll 1
    for (int j = 0; j < kWIters; j++) {
      uint32_t un[kChunk];
      residuals(j, un);
      wsync();  // every lane's reads of this iteration's samples are done
      const uint32_t Bn = j == 0 ? B[1] : j == 1 ? B[2] : j == 2 ? B[3] : B[4];
      const uint32_t Zend = j == kWIters - 1 ? nw + 1 : (Bn - 1) / 32 + 2;
      for (uint32_t jw = Z + lane; jw < Zend; jw += 64) sw[jw] = 0u;
      Z = Zend > Z ? Zend : Z;
      wsync();
      if (j == 0) put_header(sw);
      put_codes(sw, j, un);
    }
    wsync();
    for (uint32_t jw = lane; jw < nw; jw += 64) slot[jw] = sw[jw];
  } else {
    for (uint32_t jw = lane; jw <= nw; jw += 64) slot[jw] = 0u;  // (nw + 1 <= tmp_stride)
    __threadfence();
    put_header(slot);
#pragma unroll 1
    for (int j = 0; j < kWIters; j++) {
      uint32_t un[kChunk];
      residuals(j, un);
      put_codes(slot, j, un);
    }
  }
}

hipError_t launch_analyze_w(int src, int level, const JobArgs& a, int cw, hipStream_t s) {
  if (a.frame_count <= 0) return hipSuccess;
  const dim3 grid((unsigned)a.frame_count, (unsigned)cw);
  const LevelCfg cfg = level_cfg(level);
  if (cfg.nsub == 0) k_analyze_w<0><<<grid, 64, 0, s>>>(a, src);
  else k_analyze_w<8><<<grid, 64, 0, s>>>(a, src);
  return hipGetLastError();
}

}  // namespace fra
