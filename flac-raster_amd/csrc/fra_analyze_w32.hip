// fra_analyze_w32.hip -- k_analyze_w32: the 32-bps analysis with one subframe per WAVE (r05).
//
// Replaces, like k_analyze<true, 12> (fra_analyze.hip), libFLAC 1.4.3's per-channel analysis of a 32-bps stream
// (the int32 audio pyflac receives for float rasters: normalize_to_audio(bits=24), normalization.py:180-187,
// encoded at src/flac_raster/converter.py:139-154), fused with the normalisation and the band interleave.
// Decision rule FRA-1 == oracle/fr_oracle.c analyze_subframe(): the same bytes as
// k_analyze.
//
// Scope: full 4096-sample frames of a float32 raster normalised to 24 bits (norm 24: every sample within
// +-8,388,607), 8-byte sample vectors, levels 7-8 (lag 12, <= 6 apodization windows, partition order 6): the C5
// workload.  Partial last frames and everything else stay on k_analyze (the plan's partial-subframe list).
//
// Why a wave: k_analyze's 256-thread workgroup parks 30 % of its wave cycles at barriers and runs
// Levinson-Durbin and the partition searches on single waves; here one wave owns its subframe end to end, as
// k_analyze_w does for 16-bit rasters.  Lane l processes chunks t = 64 j + l, j = 0..3, so every FRA-1
// reduction order (chunk partials per 64 chunks, then (G0 + G1) + (G2 + G3)) is unchanged.
//
// LDS per wave: the 4,096 int32 samples (16 KiB: 10 waves per CU; the register budget is then up to 168
// VGPRs).  Chunk t = 16 dwords, its four 16-byte quads swizzled q -> q ^ ((t >> 1) & 3), so eight consecutive
// lanes reading the same quad of their chunks hit eight distinct bank quads (no padding words).  After the
// model search the winner's zig-zag residuals overwrite the samples; the encoded subframe's bit buffer then
// aliases them, filled iteration by iteration.
#include "fra_device.h"

namespace fra {

namespace {

constexpr int kVChunks = kMaxBlock / kChunk;   // 256
constexpr int kVIters = kVChunks / 64;          // chunks per lane
constexpr uint32_t kVWords = 16 * kVChunks;     // 4,096 dwords
constexpr int kVWin = 6;                        // apodization windows of levels 7-8
constexpr int kVLag = 12;

struct V32Smem {
  int32_t s[kVWords];
};

__device__ __forceinline__ int vq(int t, int q) { return 16 * t + 4 * (q ^ ((t >> 1) & 3)); }
__device__ __forceinline__ int4 vld(const int32_t* s, int t, int q) { return *reinterpret_cast<const int4*>(s + vq(t, q)); }
__device__ __forceinline__ void vst(int32_t* s, int t, int q, int4 v) { *reinterpret_cast<int4*>(s + vq(t, q)) = v; }
__device__ __forceinline__ int32_t vsample(const int32_t* s, int i) { return s[vq(i >> 4, (i >> 2) & 3) + (i & 3)]; }
__device__ __forceinline__ void vsync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// x[0..11] = samples 16t - 12 .. 16t - 1 (0 before the block), x[12..27] = chunk t
__device__ __forceinline__ void vread_x28(const int32_t* s, int t, int32_t (&x)[28]) {
  const bool first = t == 0;
  const int tp = first ? 0 : t - 1;
  const int4 a1 = vld(s, tp, 1), a2 = vld(s, tp, 2), a3 = vld(s, tp, 3);
  const int4 b0 = vld(s, t, 0), b1 = vld(s, t, 1), b2 = vld(s, t, 2), b3 = vld(s, t, 3);
  const int32_t xa[12] = {a1.x, a1.y, a1.z, a1.w, a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
#pragma unroll
  for (int k = 0; k < 12; k++) x[k] = first ? 0 : xa[k];
  const int32_t xb[16] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w, b2.x, b2.y, b2.z, b2.w, b3.x, b3.y, b3.z, b3.w};
#pragma unroll
  for (int k = 0; k < 16; k++) x[12 + k] = xb[k];
}
// y[0..15] = chunk t, y[16..27] = samples 16t + 16 .. 16t + 27 (0 past the block: t == 255)
__device__ __forceinline__ void vread_y28(const int32_t* s, int t, int32_t (&y)[28]) {
  const bool last = t == kVChunks - 1;
  const int tn = last ? t : t + 1;
  const int4 b0 = vld(s, t, 0), b1 = vld(s, t, 1), b2 = vld(s, t, 2), b3 = vld(s, t, 3);
  const int4 c0 = vld(s, tn, 0), c1 = vld(s, tn, 1), c2 = vld(s, tn, 2);
  const int32_t yb[16] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w, b2.x, b2.y, b2.z, b2.w, b3.x, b3.y, b3.z, b3.w};
#pragma unroll
  for (int k = 0; k < 16; k++) y[k] = yb[k];
  const int32_t yc[12] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c2.x, c2.y, c2.z, c2.w};
#pragma unroll
  for (int k = 0; k < 12; k++) y[16 + k] = last ? 0 : yc[k];
}

// normalize_to_audio (bits 24) of one channel of a full frame of a float32 raster, norm_sample's op sequence
// (the f64 chain numpy evaluates): lane l takes the 8-byte vectors l + 64 k (2 samples), 16 loads in flight
// per batch; the row walk adds the uniform step qs w + rs (no division per vector)
__device__ __forceinline__ void vload_f32(const void* base, const StreamDev& st, const FrameDev& fr, int c,
                                          const NormParams& np, int32_t* s, int lane, uint32_t& orv, int32_t& vmin,
                                          int32_t& vmax) {
  constexpr int V = 2, NV = kMaxBlock / 64 / V, NB = 16;
  constexpr uint32_t step = 64 * V;
  using VT = VecT<float, V>;
  const uint32_t w = (uint32_t)st.width;
  const char* b0 = (const char*)((const float*)base + st.base_off + (int64_t)c * st.band_stride + (int64_t)fr.row0 * st.row_stride);
  const uint32_t rsb = (uint32_t)st.row_stride * 4u;
  const uint32_t qs = step / w, rs = step - qs * w, rstep = qs * rsb;
  uint32_t col = (uint32_t)fr.col0 + (uint32_t)lane * V;
  uint32_t roff = 0;
  if (col >= w) {
    const uint32_t q = col / w;
    col -= q * w;
    roff = q * rsb;
  }
#pragma unroll
  for (int b = 0; b < NV / NB; b++) {
    VT x[NB];
#pragma unroll
    for (int k = 0; k < NB; k++) {
      x[k] = *(const VT*)(b0 + (roff + col * 4u));
      col += rs;
      roff += rstep;
      if (col >= w) { col -= w; roff += rsb; }
    }
#pragma unroll
    for (int k = 0; k < NB; k++) {
      const int i = 2 * (lane + 64 * (NB * b + k));
      const int32_t v0 = norm_sample<ST_F32>((double)x[k].v[0], np), v1 = norm_sample<ST_F32>((double)x[k].v[1], np);
      *reinterpret_cast<int2*>(s + vq(i >> 4, (i >> 2) & 3) + (i & 3)) = make_int2(v0, v1);
      orv |= (uint32_t)v0 | (uint32_t)v1;
      vmin = min(vmin, min(v0, v1));
      vmax = max(vmax, max(v0, v1));
    }
  }
}

// upper-lane group sums over aligned groups of 2^LS lanes (compile-time LS), result at the group's last lane
template <int LS>
__device__ __forceinline__ uint64_t vgroup_sum64(uint64_t v) {
  if constexpr (LS > 0) v = up_add64<0>(v);
  if constexpr (LS > 1) v = up_add64<1>(v);
  if constexpr (LS > 2) v = up_add64<2>(v);
  if constexpr (LS > 3) v = up_add64<3>(v);
  if constexpr (LS > 4) v = up_add64<4>(v);
  if constexpr (LS > 5) v = up_add64<5>(v);
  return v;
}
__device__ __forceinline__ uint64_t vgroup_sum64_rt(uint64_t v, int ls) {
  if (ls > 0) v = up_add64<0>(v);
  if (ls > 1) v = up_add64<1>(v);
  if (ls > 2) v = up_add64<2>(v);
  if (ls > 3) v = up_add64<3>(v);
  if (ls > 4) v = up_add64<4>(v);
  if (ls > 5) v = up_add64<5>(v);
  return v;
}
__device__ __forceinline__ double vrdlane_f64(double v, int l) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
}

// FRA-1 3.7 FIXED candidates from 64-bit register partition sums (lane p < 2^P: partition p of order k)
__device__ __forceinline__ void vfixed_guess2(const uint64_t (&ps)[5], int P, int lane, int& g1, int& g2) {
  uint64_t T[5];
#pragma unroll
  for (int k = 0; k < 5; k++) {
    uint64_t v = lane < (1 << P) ? ps[k] : 0ull;
    v = up_add64<0>(v); v = up_add64<1>(v); v = up_add64<2>(v);
    v = up_add64<3>(v); v = up_add64<4>(v); v = up_add64<5>(v);
    T[k] = rl64(v, 63);
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

// Levinson-Durbin keeping only this lane's order lo (the op sequence of levinson_wave / oracle ora_levinson)
template <int MAXLAG>
__device__ inline int vlevinson_keep(const double (&ac)[MAXLAG + 1], int max_order, double& e, double (&lp)[MAXLAG],
                                     int lo) {
  double lpc[MAXLAG];
#pragma unroll
  for (int j = 0; j < MAXLAG; j++) { lpc[j] = 0.0; lp[j] = 0.0; }
  e = 0.0;
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
      for (int j = 0; j <= i; j++) lp[j] = mine ? -lpc[j] : lp[j];
      e = (mine || (i == 0 && lo == 0)) ? err : e;
      if (!(err > 0.0)) {
        result = (err == 0.0) ? i + 1 : i;
        done = true;
      }
    }
  }
  return result;
}

// the lag sums of one autocorrelation reduce-scatter (autocorr_reduce_wave without the store)
template <int NL>
__device__ __forceinline__ void vreduce_regs(const double (&acc)[NL], double (&z)[((NL + 1) / 2 + 1) / 2]) {
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
__host__ __device__ constexpr int vlag_slot(int lag) {  // (k << 2) | r of the first slot holding lag
  constexpr int N32 = (NL + 1) / 2, N16 = (N32 + 1) / 2;
  for (int k = 0; k < N16; k++)
    for (int r = 0; r < 4; r++) {
      const int wi = (2 * k + 1 < N32) ? 2 * k + (r & 1) : 2 * k;
      const int l = (2 * wi + 1 < NL) ? 2 * wi + (r >> 1) : 2 * wi;
      if (l == lag) return (k << 2) | r;
    }
  return -1;
}

// 32-bps residuals of a 12-tap predictor evaluated exactly in f64 (lpc_abs2_f64: |q| < 2^14, |x| < 2^24, so every
// product and partial sum is an integer below 2^53 and floor(sum * 2^-sh) is the int64 arithmetic shift).
// Lower orders carry zero coefficients: a +-0 product leaves the exact integer sum unchanged.
__device__ __forceinline__ void vres12(const double (&xd)[28], const double (&qd)[kVLag], double scale,
                                       double (&r)[kChunk]) {
#pragma unroll
  for (int jj = 0; jj < kChunk; jj++) {
    double sum = 0.0;
#pragma unroll
    for (int j = 0; j < kVLag; j++) sum = fma(qd[j], xd[11 + jj - j], sum);
    r[jj] = xd[12 + jj] - floor(sum * scale);
  }
}

}  // namespace

// occupancy: 16 KiB of LDS -> 10 waves per CU (2-3 per SIMD): registers up to 168 keep 3 per SIMD possible
template <int MAXLAG, int PCAP>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 3)))
k_analyze_w32(JobArgs a, int src) {
  static_assert(MAXLAG == kVLag && PCAP == 6, "levels 7-8");
  __shared__ V32Smem S;
  int32_t* const sw = S.s;
  const int lane = (int)threadIdx.x;
  const int g = a.frame_base + (int)blockIdx.x;
  const int c = (int)blockIdx.y;
  const FrameDev fr = a.frames[g];
  const StreamDev st = a.streams[fr.stream];
  if (c >= st.channels) return;
  if (fr.n != kMaxBlock) return;  // partial last frames: k_analyze, over the plan's list of them
  constexpr int n = kMaxBlock;
  const int bps = st.bps;  // 32
  const LevelCfg cfg = level_cfg(a.level);
  SfDesc* d = &a.sf[(size_t)g * a.cmax + c];
  uint32_t* const slot = a.tmp + ((size_t)g * a.cmax + c) * a.tmp_stride;

  // ---- 1. load + normalise, OR / min / max
  const void* const raster = a.raster;
  const NormParams np = norm_params(st, a.norm[fr.stream]);
  auto load_samples = [&](uint32_t& ov, int32_t& mn, int32_t& mx) {
    vload_f32(raster, st, fr, c, np, sw, lane, ov, mn, mx);
  };
  uint32_t orv = 0;
  int32_t vmin = INT32_MAX, vmax = INT32_MIN;
  load_samples(orv, vmin, vmax);
  orv = wave_or32(orv);
  vsync();
  vmin = (int32_t)(wave_min32((uint32_t)vmin ^ 0x80000000u) ^ 0x80000000u);
  vmax = (int32_t)(~wave_min32(~((uint32_t)vmax ^ 0x80000000u)) ^ 0x80000000u);

#ifdef W32_STOP
#define W32_STOP_AT(k_, keep_)                        \
  if (W32_STOP == (k_)) {                             \
    if (lane == 0) d->cval = (int32_t)(keep_);        \
    return;                                           \
  }
#else
#define W32_STOP_AT(k_, keep_)
#endif
  W32_STOP_AT(1, orv ^ (uint32_t)vmin ^ (uint32_t)vmax)
  // ---- 2. CONSTANT / wasted bits (3.2, 3.3)
  if (vmin == vmax) {
    if (lane == 0) {
      d->type = 0; d->order = 0; d->wasted = 0; d->sbps = (uint8_t)bps; d->cval = vmin;
      d->bits = 8u + (uint32_t)bps; d->porder = 0; d->method = 0; d->precision = 0; d->shift = 0;
      const uint64_t v = (uint64_t)(uint32_t)vmin & (bps >= 32 ? 0xFFFFFFFFull : ((1ull << bps) - 1));
      const uint64_t blob = v << (64 - 8 - bps);
      slot[0] = (uint32_t)(blob >> 32);
      slot[1] = (uint32_t)blob;
    }
    return;
  }
  const int w = __builtin_ctz(orv);
  const int sbps = bps - w;
  auto shift_wasted = [&]() {
    for (int k = lane; k < (int)kVWords; k += 64) sw[k] = sw[k] >> w;
  };
  if (w) shift_wasted();
  vsync();
  const uint32_t hdr = 8u + (uint32_t)w;
  const uint32_t verb = hdr + (uint32_t)n * (uint32_t)sbps;
  constexpr int P = PCAP;          // = max_porder(n, 0, cfg.max_porder)
  constexpr int gsl = 8 - P;       // lanes per finest partition (chunks of 16)
  constexpr int npl = 6 - gsl;     // log2 finest partitions per iteration
  const int prec = qlp_precision(bps, n);
  const int lmax = cfg.max_lpc;    // 12 < n - 1
  const int pj = lane >> npl;
  const int psrc = ((lane & ((1 << npl) - 1)) << gsl) | ((1 << gsl) - 1);

  // ---- 3a. FIXED residual sums by 32-bit finite differences (|samples| < 2^23: |4th difference| < 2^27, 16 of
  // them < 2^31), per finest partition: group sums gathered so that lane p holds partition p (64-bit)
  uint64_t pfix[5] = {0, 0, 0, 0, 0};
  for (int j = 0; j < kVIters; j++) {
    const int t = 64 * j + lane;
    const bool head = t == 0;
    int32_t x[28];
    vread_x28(sw, t, x);
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
      const uint64_t gs = bperm64(vgroup_sum64<gsl>(2ull * s32), psrc);
      pfix[k] = pj == j ? gs : pfix[k];
    }
  }

  W32_STOP_AT(2, (uint32_t)(pfix[0] ^ pfix[1] ^ pfix[2] ^ pfix[3] ^ pfix[4]))
  // ---- running winner (FRA-1 3.8: first minimal estimate in model order)
  uint32_t west = 0xFFFFFFFFu;
  int wm = 99, wtype = 2, wo = 0, wsh = 0, wps = 0;
  uint32_t wk = 0;
  auto offer = [&](uint32_t est, int m, int type, int o, int sh, int ps, uint32_t kreg) {
    if (est < west || (est == west && m < wm)) {
      west = est; wm = m; wtype = type; wo = o; wsh = sh; wps = ps; wk = kreg;
    }
  };
  int g1, g2;
  vfixed_guess2(pfix, P, lane, g1, g2);
  uint64_t pf1 = 0, pf2 = 0;
#pragma unroll
  for (int k = 0; k < 5; k++) {
    pf1 = k == g1 ? pfix[k] : pf1;
    pf2 = k == g2 ? pfix[k] : pf2;
  }

  // ---- 3. LPC analysis per apodization window (3.4-3.7).  Models lane-distributed: mvA lane 12 wi + jx = qlp
  // coefficient jx of window wi < 5, mvB lane jx = coefficient jx of window 5, mvB lane 16 + wi = window wi's
  // shift | usable order << 8 (0: none / not quantisable)
  uint32_t mvA = 0, mvB = 0;
  int nlpc = 0;
  if (cfg.nsub > 0 && lmax > 0) {
    const int nwin = a.nwin;
    nlpc = nwin;
    constexpr int NL = MAXLAG + 1, N16 = ((NL + 1) / 2 + 1) / 2;
    const int gw = lane >> 4, lo = lane & 15;
    const int dA = lane < 60 ? lane / 12 : -1, jA = lane < 60 ? lane % 12 : 0;  // mvA lane: window, coefficient
    const int dB = lane < 12 ? 5 : (lane >= 16 && lane < 22 ? lane - 16 : -1);   // mvB lane: window
    // rounds of <= 4 windows: their autocorrelations (window wi's lag sums to lane group wi % 4), then
    // Levinson-Durbin, order choice and quantisation of the round's windows at once (window wi on lanes
    // 16 (wi % 4) .. +15), each model gathered into mvA / mvB -- one round's sums live at a time
#pragma unroll 1
    for (int r = 0; r * 4 < nwin; r++) {
      double acl[NL];
#pragma unroll
      for (int l = 0; l < NL; l++) acl[l] = 0.0;
      const int wend = min(nwin, 4 * r + 4);
#pragma unroll 1
      for (int wi = 4 * r; wi < wend; wi++) {
        const int32_t* wr = a.wrange + 2 * ((size_t)fr.win * a.nwin + wi);
        const int32_t* wp = a.wplat + 2 * ((size_t)fr.win * a.nwin + wi);
        const int wlo = wr[0], whi = wr[1], plo = wp[0], phi = wp[1];
        const float* win = a.win + ((size_t)fr.win * a.nwin + wi) * a.blocksize;
        double s01[N16], sacc[N16];
#pragma unroll
        for (int k = 0; k < N16; k++) { s01[k] = 0.0; sacc[k] = 0.0; }
        int lnw = lane;
        asm volatile("" : "+v"(lnw));
#pragma unroll 1
        for (int j = 0; j < kVIters; j++) {
          double z[N16];
          if (wlo < 1024 * j + 1024 + MAXLAG && whi > 1024 * j) {
            const int t = 64 * j + lnw, i0 = kChunk * t;
            int32_t y[kChunk + MAXLAG];
            vread_y28(sw, t, y);
            // the last chunk's look-ahead is zero (vread_y28): its coefficients are read without a bound (the
            // window table has slack past its last row) and every product past n is still +-0
            const bool plat = i0 >= plo && i0 + kChunk + MAXLAG <= phi;
            float wf[kChunk + MAXLAG];
            if (__all(plat)) {
#pragma unroll
              for (int jx = 0; jx < kChunk + MAXLAG; jx++) wf[jx] = (float)y[jx];
            } else {
#pragma unroll
              for (int jx = 0; jx < kChunk + MAXLAG; jx++) wf[jx] = (float)y[jx] * (plat ? 1.0f : win[i0 + jx]);
            }
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
            vreduce_regs<NL>(acc, z);
          } else {
#pragma unroll
            for (int k = 0; k < N16; k++) z[k] = 0.0;
          }
          if (j == 2) {
#pragma unroll
            for (int k = 0; k < N16; k++) s01[k] = sacc[k];
          }
#pragma unroll
          for (int k = 0; k < N16; k++) sacc[k] = (j & 1) ? sacc[k] + z[k] : z[k];
        }
#pragma unroll
        for (int l = 0; l < NL; l++) {
          const int sl = vlag_slot<NL>(l);
          const double tot = vrdlane_f64(s01[sl >> 2] + sacc[sl >> 2], 16 * (sl & 3) + 15);
          acl[l] = gw == wi - 4 * r ? tot : acl[l];
        }
      }
      const bool gon = 4 * r + gw < nwin;
      double lpo[MAXLAG], e = 0.0;
      int nord = 0;
      if (gon && acl[0] != 0.0) nord = vlevinson_keep<MAXLAG>(acl, lmax, e, lpo, lo);
      const bool on = nord > 0 && lo >= 1 && lo <= nord;
      const uint64_t key = on ? (uint64_t)__double_as_longlong(order_bits(e, n, lo, prec + sbps)) : ~0ull;
      uint64_t rk = min(key, dpp64_old<DPP_SHR1, 0xF>(key, ~0ull));
      rk = min(rk, dpp64_old<DPP_SHR2, 0xF>(rk, ~0ull));
      rk = min(rk, dpp64_old<DPP_SHR4, 0xF>(rk, ~0ull));
      rk = min(rk, dpp64_old<DPP_SHR8, 0xF>(rk, ~0ull));
      const uint64_t kmin = __shfl(rk, (lane & 48) | 15, 64);
      const uint64_t bal = __ballot(on && key == kmin);
      const uint32_t rowbits = (uint32_t)(bal >> (16 * gw)) & 0xFFFFu;
      int32_t q[MAXLAG];
#pragma unroll
      for (int jx = 0; jx < MAXLAG; jx++) q[jx] = 0;
      bool ok = false;
      int qsh = 0;
      if (on) ok = quantize<MAXLAG>(lpo, lo, prec, q, qsh);
      const int o_l = nord > 0 ? (int)__builtin_ctz(rowbits | 0x10000u) : 0;
      // source lane of a window of this round: 16 g + o_g (every ds_bpermute on all 64 lanes)
      const int ga = dA - 4 * r, gb = dB - 4 * r;
      const bool inA = dA >= 0 && ga >= 0 && ga < 4 && dA < nwin, inB = dB >= 0 && gb >= 0 && gb < 4 && dB < nwin;
      const int gA = inA ? ga : 0, gB = inB ? gb : 0;
      const int owA = (int)bperm32((uint32_t)o_l, 16 * gA), owB = (int)bperm32((uint32_t)o_l, 16 * gB);
      const int LA = 16 * gA + owA, LB = 16 * gB + owB;
      // (info computed at the SOURCE lane from its own values: its order o_l == lo there)
      const uint32_t info = (uint32_t)qsh | ((o_l > 0 && ok) ? (uint32_t)o_l << 8 : 0u);
      const uint32_t vinfo = bperm32(info, LB);
#pragma unroll
      for (int jx = 0; jx < MAXLAG; jx++) {
        const uint32_t va = bperm32((uint32_t)q[jx], LA), vb = bperm32((uint32_t)q[jx], LB);
        mvA = (inA && jA == jx) ? va : mvA;
        mvB = (inB && lane < 12 && lane == jx) ? vb : mvB;
      }
      mvB = (inB && lane >= 16) ? vinfo : mvB;
    }
  }
  W32_STOP_AT(3, mvA ^ mvB)
  // windows with a usable model (lanes 16 + wi of mvB with an order)
  const uint32_t okm = (uint32_t)(__ballot(lane >= 16 && lane < 16 + kVWin && (mvB >> 8) != 0) >> 16);
  auto coef = [&](int wi, int jx) -> int32_t {  // uniform wi, jx
    return wi < 5 ? __builtin_amdgcn_readlane((int)mvA, 12 * wi + jx) : __builtin_amdgcn_readlane((int)mvB, jx);
  };

  // ---- 4+5. the candidates in model order -- FIXED g1, g2, then each window's LPC model -- one partition search
  // each; an LPC model first gets its residual sums at the finest partitions (exact f64 predictor); a model whose
  // residual leaves int32 is not a candidate (as the oracle's compute_residual)
#pragma unroll 1
  for (int ci = 0; ci < 2 + nlpc; ci++) {
    int m, o, sh = 0, type = 2;
    uint64_t psum = 0;
    if (ci < 2) {
      m = o = ci == 0 ? g1 : g2;
      psum = ci == 0 ? pf1 : pf2;
    } else {
      const int wi = ci - 2;
      if (!((okm >> wi) & 1u)) continue;
      const uint32_t inf = (uint32_t)__builtin_amdgcn_readlane((int)mvB, 16 + wi);
      o = (int)(inf >> 8);
      m = 5 + wi;
      type = 3;
      sh = (int)(inf & 0xFFu);
      double qd[kVLag];
#pragma unroll
      for (int jx = 0; jx < kVLag; jx++) qd[jx] = (double)coef(wi, jx);
      const double scale = ldexp(1.0, -sh);
      bool ovf = false;
#pragma unroll 1
      for (int j = 0; j < kVIters; j++) {
        const int t = 64 * j + lane;
        const bool head = t == 0;
        int32_t x[28];
        vread_x28(sw, t, x);
        double xd[28];
#pragma unroll
        for (int k = 0; k < 28; k++) xd[k] = (double)x[k];
        double acc = 0.0;  // exact: sum of 16 |r| < 2^36 whenever no residual overflowed
        // the model's own order (lpc_abs2_f64's exact-order bodies): a 12-tap body for every order cost twice the
        // f64 FMAs of the level-8 models
        switch (o) {
#define FRA_CASE(O_)                                                                   \
  case O_:                                                                             \
    _Pragma("unroll") for (int jj = 0; jj < kChunk; jj++) {                            \
      double sum = 0.0;                                                                \
      _Pragma("unroll") for (int jq = 0; jq < O_; jq++) sum = fma(qd[jq], xd[11 + jj - jq], sum); \
      const double rr = xd[12 + jj] - floor(sum * scale);                              \
      const bool on = !(jj < O_ && head);                                              \
      ovf |= on && (rr > 2147483647.0 || rr < -2147483648.0);                          \
      acc += on ? fabs(rr) : 0.0;                                                      \
    }                                                                                  \
    break;
          FRA_CASE(1) FRA_CASE(2) FRA_CASE(3) FRA_CASE(4) FRA_CASE(5) FRA_CASE(6)
          FRA_CASE(7) FRA_CASE(8) FRA_CASE(9) FRA_CASE(10) FRA_CASE(11) FRA_CASE(12)
#undef FRA_CASE
        }
        const uint64_t a2 = 2ull * (uint64_t)acc;
        const uint64_t gs = bperm64(vgroup_sum64<gsl>(a2), psrc);
        psum = pj == j ? gs : psum;
      }
      if (__any(ovf)) continue;
    }
    constexpr int pm = P;  // max_porder(n, o, cfg.max_porder) == P for n = 4096, o <= 12
    uint64_t best;
    int bp;
    uint32_t kreg;
    porder_search_reg(psum, P, pm, n, o, lane, best, bp, kreg);
    const uint64_t est = hdr + (uint64_t)o * sbps + (type == 3 ? 9 + (uint64_t)o * prec : 0) + best;
    offer((uint32_t)est, m, type, o, sh, bp, kreg);
  }

  W32_STOP_AT(4, west ^ (uint32_t)wm ^ wk)
  // ---- 6. the winner's zig-zag residuals (written over the samples), exact Rice bits with each partition's
  // parameter refined (3.9), VERBATIM if not smaller (the samples loaded again), else encode (RFC 9639 9.2) into
  // the LDS bit buffer aliasing the residuals (or, when a poorly compressible start would overrun them, straight
  // into the slot with global ORs)
  const int type = wtype, o = wo, sh = wsh, ps = wps;
  const int wwi = wm - 5;
  double qd[kVLag];
#pragma unroll
  for (int jx = 0; jx < kVLag; jx++) qd[jx] = type == 3 ? (double)coef(wwi, jx) : 0.0;
  const double scale = ldexp(1.0, -sh);
  const int32_t warm = lane < o ? vsample(sw, lane) : 0;  // warm-up sample `lane` (before the overwrite)
  const int pz = n >> ps;
  const int tl = 8 - ps;                  // log2 chunks per partition (2..8)
  const int ls = tl < 6 ? tl : 6;         // lanes per partition group inside one iteration
  const int npp = 1 << ps;
  uint32_t kc[kVIters];
  uint64_t fk[kVIters][3];
  uint32_t k0r[kVIters];
  uint32_t bitsl = 0;
  bool bigl = false;
  uint64_t E[3] = {0, 0, 0};
  int32_t cy[12];
#pragma unroll
  for (int k = 0; k < 12; k++) cy[k] = 0;
#pragma unroll
  for (int j = 0; j < kVIters; j++) {
    const int t = 64 * j + lane;
    const bool head = t == 0;
    int32_t x[28];
    vread_x28(sw, t, x);
    if (j > 0) {  // chunk 64 j - 1 already holds residuals: its last 12 samples came from lane 63
#pragma unroll
      for (int k = 0; k < 12; k++) x[k] = lane == 0 ? cy[k] : x[k];
    }
#pragma unroll
    for (int k = 0; k < 12; k++) cy[k] = __builtin_amdgcn_readlane(x[16 + k], 63);
    uint32_t u[kChunk];
    if (type == 3) {
      double xd[28];
#pragma unroll
      for (int k = 0; k < 28; k++) xd[k] = (double)x[k];
      double r[kChunk];
      vres12(xd, qd, scale, r);
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) u[jj] = zz32((int32_t)r[jj]);
    } else {  // FIXED: the o-th finite difference in place (32-bit: |samples| < 2^23)
#pragma unroll
      for (int k = 1; k <= 4; k++) {
        if (k <= o) {
#pragma unroll
          for (int jx = 12 + kChunk - 1; jx >= 8 + k; jx--) x[jx] = x[jx] - x[jx - 1];
        }
      }
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) u[jj] = zz32(x[12 + jj]);
    }
#pragma unroll
    for (int jj = 0; jj < kVLag; jj++)
      if (head && jj < o) u[jj] = 0u;
    vsync();  // every lane's sample reads of this iteration precede the stores
#pragma unroll
    for (int qq = 0; qq < 4; qq++)
      vst(sw, t, qq, make_int4((int)u[4 * qq], (int)u[4 * qq + 1], (int)u[4 * qq + 2], (int)u[4 * qq + 3]));
    const int pidx = t >> tl;
    const int k0 = __shfl((int)wk, pidx & 63, 64);
    const int km = k0 > 0 ? k0 - 1 : 0;
    uint64_t f0 = 0, f1 = 0, f2 = 0;
#pragma unroll
    for (int jj = 0; jj < kChunk; jj++) {
      f0 += u[jj] >> km;
      f1 += u[jj] >> k0;
      f2 += u[jj] >> (k0 + 1);
    }
    fk[j][0] = f0;
    fk[j][1] = f1;
    fk[j][2] = f2;
    k0r[j] = (uint32_t)k0;
    const uint64_t v0 = vgroup_sum64_rt(f0, ls), v1 = vgroup_sum64_rt(f1, ls), v2 = vgroup_sum64_rt(f2, ls);
    if (tl <= 6) {  // the partition lies inside this iteration: its last lane decides
      const uint32_t cnt = (uint32_t)(pz - (pidx == 0 ? o : 0));
      const uint64_t ev[3] = {v0, v1, v2};
      uint64_t best = 0;
      int bk = 0;
      bool first = true;
#pragma unroll
      for (int dk = -1; dk <= 1; dk++) {
        const int kk = k0 + dk;
        const uint64_t e = (uint64_t)(cnt * (uint32_t)(kk + 1)) + ev[dk + 1];
        const bool take = kk >= 0 && kk <= 30 && (first || e < best);
        best = take ? e : best;
        bk = take ? kk : bk;
        first = first && !(kk >= 0 && kk <= 30);
      }
      const bool leader = (lane & ((1 << ls) - 1)) == (1 << ls) - 1;
      bk = leader ? bk : 0;
      bitsl += leader ? (uint32_t)best : 0u;
      bigl = bigl || bk > 14;
      if (leader) d->k[pidx] = (uint8_t)bk;
      kc[j] = (uint32_t)__shfl(bk, lane | ((1 << ls) - 1), 64);
    } else {  // ps <= 1: whole-iteration sums accumulate into the partition's running sums (uniform)
      E[0] += rl64(v0, 63);
      E[1] += rl64(v1, 63);
      E[2] += rl64(v2, 63);
      const int span = 1 << (tl - 6);  // iterations per partition (2 or 4)
      kc[j] = 0;
      if (((j + 1) & (span - 1)) == 0) {  // partition complete: decide its parameter
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
        for (int jx = 0; jx < kVIters; jx++)
          if (jx <= j && jx > j - span) kc[jx] = (uint32_t)bk;
        E[0] = E[1] = E[2] = 0;
      }
    }
  }
  W32_STOP_AT(5, bitsl ^ (uint32_t)fk[1][1])
  const bool big = __any(bigl);
  const uint64_t rtot = (uint64_t)wave_sum32(bitsl) + (uint64_t)npp * (big ? 5 : 4) + 6;
  const uint64_t exact = hdr + (uint64_t)o * sbps + (type == 3 ? 9 + (uint64_t)o * prec : 0) + rtot;
  const uint32_t smask = sbps >= 32 ? 0xFFFFFFFFu : (1u << sbps) - 1u;
  if (exact >= verb) {  // VERBATIM: the samples loaded again, written straight to the slot
    vsync();
    {
      uint32_t ov = 0;
      int32_t mn = 0, mx = 0;
      load_samples(ov, mn, mx);
    }
    vsync();
    if (w) shift_wasted();
    vsync();
    if (lane == 0) {
      d->type = 1; d->order = 0; d->wasted = (uint8_t)w; d->sbps = (uint8_t)sbps; d->cval = 0; d->porder = 0;
      d->method = 0; d->precision = 0; d->shift = 0; d->bits = verb;
    }
    const uint32_t nwv = (verb + 31) >> 5;
    const uint64_t hv = ((uint64_t)(2u | (w ? 1u : 0u)) << 56) | (w ? (1ull << (63 - (8 + w - 1))) : 0ull);
    for (uint32_t jw = lane; jw < nwv; jw += 64) {
      const int64_t wb = 32 * (int64_t)jw;
      uint32_t word = jw == 0 ? (uint32_t)(hv >> 32) : (jw == 1 ? (uint32_t)hv : 0u);
      const int s0 = wb > (int64_t)hdr ? (int)((wb - (int64_t)hdr) / sbps) : 0;
      for (int si = s0; si < n && (int64_t)hdr + (int64_t)si * sbps < wb + 32; si++) {
        const int64_t rel = (int64_t)hdr + (int64_t)si * sbps - wb;
        const int sft = 32 - (int)rel - sbps;
        const uint64_t v = (uint64_t)((uint32_t)vsample(sw, si) & smask);
        word |= sft >= 0 ? (uint32_t)(v << sft) : (uint32_t)(v >> -sft);
      }
      slot[jw] = word;
    }
    return;
  }
  // code bits of each chunk from the exact pass's sums; the bit position of every iteration's first code
  const uint32_t fbits = (uint32_t)exact;
  const uint32_t nw = (fbits + 31) >> 5;
  const int pb = big ? 5 : 4;
  const uint32_t pos = hdr + (uint32_t)o * sbps + (type == 3 ? 9u + (uint32_t)o * prec : 0u);
  uint32_t totl[kVIters];
  uint32_t B[kVIters + 1];
  B[0] = pos + 6;
#pragma unroll
  for (int j = 0; j < kVIters; j++) {
    const int t = 64 * j + lane;
    const uint32_t kcur = kc[j], k0 = k0r[j];
    const uint64_t f = kcur + 1 == k0 ? fk[j][0] : kcur == k0 ? fk[j][1] : fk[j][2];
    const bool pstart = ((t << 4) & (pz - 1)) == 0;
    totl[j] = (uint32_t)f + (uint32_t)(kChunk - (t == 0 ? o : 0)) * (kcur + 1u) + (pstart ? (uint32_t)pb : 0u);
    B[j + 1] = B[j] + wave_sum32(totl[j]);
  }
  // iteration j's words (+ the spare one) must stay below chunk 64 (j + 1)'s first word
  bool inlds = nw + 1 <= kVWords;
#pragma unroll
  for (int j = 0; j + 1 < kVIters; j++) inlds = inlds && (B[j + 1] - 1) / 32 + 2 <= 16u * 64u * (uint32_t)(j + 1);
  // the winner's coefficient `lane` (descriptor and header)
  const int32_t cvl = type == 3 ? (int32_t)__shfl((int)(wwi < 5 ? mvA : mvB),
                                                  (wwi < 5 ? 12 * (wwi < 0 ? 0 : wwi) : 0) + (lane < kVLag ? lane : 0), 64)
                                : 0;
  if (lane < kMaxLpc) d->coef[lane] = cvl;
  if (lane == 0) {
    d->wasted = (uint8_t)w; d->sbps = (uint8_t)sbps; d->cval = 0;
    d->type = (uint8_t)type; d->order = (uint8_t)o; d->porder = (uint8_t)ps; d->method = big ? 1 : 0;
    d->precision = (uint8_t)(type == 3 ? prec : 0); d->shift = (int8_t)sh; d->bits = (uint32_t)exact;
  }
  auto put_header = [&](uint32_t* buf) {
    if (lane == 0) {
      lds_put(buf, 0, (uint32_t)((type == 3 ? 31 + o : 8 + o) << 1) | (w ? 1u : 0u), 8);
      if (w) lds_put(buf, 8 + (uint32_t)(w - 1), 1u, 1);
    }
    if (lane < o) lds_put(buf, hdr + (uint32_t)lane * sbps, (uint32_t)warm & smask, sbps);
    const uint32_t ph = hdr + (uint32_t)o * sbps;
    if (type == 3 && lane == 0) {
      lds_put(buf, ph, (uint32_t)(prec - 1), 4);
      lds_put(buf, ph + 4, (uint32_t)sh & 31u, 5);
    }
    if (type == 3 && lane < o) lds_put(buf, ph + 9 + (uint32_t)lane * prec, (uint32_t)cvl & ((1u << prec) - 1u), prec);
    if (lane == 0) lds_put(buf, pos, ((uint32_t)(big ? 1 : 0) << 4) | (uint32_t)ps, 6);
  };
  auto put_codes = [&](uint32_t* buf, int j, const uint32_t (&un)[kChunk]) {
    const int t = 64 * j + lane;
    const bool head = t == 0;
    const uint32_t kcur = kc[j], tot = totl[j];
    const bool pstart = ((t << 4) & (pz - 1)) == 0;
    uint32_t p = B[j] + wave_incl_scan32(tot) - tot;
    if (pstart) { lds_put(buf, p, kcur, pb); p += (uint32_t)pb; }
    const uint32_t sal = 31u - kcur;
#pragma unroll
    for (int jj = 0; jj < kChunk; jj++) {
      const bool skip = jj < kVLag && head && jj < o;
      const uint32_t Pp = p + (un[jj] >> kcur);
      lds_put_al(buf, Pp, skip ? 0u : ((un[jj] << sal) | 0x80000000u));
      p = skip ? p : Pp + 1u + kcur;
    }
  };
  auto read_u = [&](int j, uint32_t (&un)[kChunk]) {
    const int t = 64 * j + lane;
#pragma unroll
    for (int qq = 0; qq < 4; qq++) {
      const int4 v = vld(sw, t, qq);
      un[4 * qq] = (uint32_t)v.x; un[4 * qq + 1] = (uint32_t)v.y; un[4 * qq + 2] = (uint32_t)v.z; un[4 * qq + 3] = (uint32_t)v.w;
    }
  };
  if (inlds) {
    uint32_t* const buf = reinterpret_cast<uint32_t*>(sw);
    uint32_t Z = 0;  // words [0, Z) are zeroed (and possibly written)
#pragma unroll
    for (int j = 0; j < kVIters; j++) {
      uint32_t un[kChunk];
      read_u(j, un);
      vsync();  // every lane's reads of this iteration's residuals precede the zeroing
      const uint32_t Zend = j == kVIters - 1 ? nw + 1 : (B[j + 1] - 1) / 32 + 2;
      for (uint32_t jw = Z + lane; jw < Zend; jw += 64) buf[jw] = 0u;
      Z = Zend > Z ? Zend : Z;
      vsync();
      if (j == 0) put_header(buf);
      put_codes(buf, j, un);
    }
    vsync();
    for (uint32_t jw = lane; jw < nw; jw += 64) slot[jw] = buf[jw];
  } else {  // codes ORed into the zeroed slot (global atomics); the residuals stay intact in LDS
    for (uint32_t jw = lane; jw <= nw; jw += 64) slot[jw] = 0u;  // (nw + 1 <= tmp_stride)
    __threadfence();
    put_header(slot);
#pragma unroll 1
    for (int j = 0; j < kVIters; j++) {
      uint32_t un[kChunk];
      read_u(j, un);
      put_codes(slot, j, un);
    }
  }
}

bool analyze_w32_ok(int src, int level, int norm) { return src == ST_F32 && norm == 24 && level >= 7 && level <= 8; }

hipError_t launch_analyze_w32(int src, int level, const JobArgs& a, int cw, hipStream_t s) {
  if (a.frame_count <= 0) return hipSuccess;
  const LevelCfg cfg = level_cfg(level);
  if (src != ST_F32 || cfg.max_lpc != 12 || cfg.max_porder != 6 || a.nwin > kVWin) return hipErrorInvalidValue;
  const dim3 grid((unsigned)a.frame_count, (unsigned)cw);
  k_analyze_w32<12, 6><<<grid, 64, 0, s>>>(a, src);
  return hipGetLastError();
}

}  // namespace fra
