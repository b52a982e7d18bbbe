// fra_analyze_w.hip -- k_analyze_w: the 16-bit analysis with one subframe per WAVE.
//
// Replaces, like k_analyze (fra_analyze.hip), libFLAC 1.4.3's per-channel analysis inside
// FLAC__stream_encoder_process_interleaved (driven by pyflac at src/flac_raster/converter.py:153 /
// spatial_encoder.py:303), fused with normalize_to_audio (normalization.py:126-202) and the band
// interleave (converter.py:99-110).  Decision rule FRA-1 == oracle/fr_oracle.c
// analyze_subframe(), bit for bit the same bytes as k_analyze.
//
// Scope: full 4096-sample frames of a <= 16-bit integer raster whose normalisation goes through the
// per-tile table (k_norm_lut), 8-byte sample vectors, levels 3-6 (lag <= 8, <= 3 apodization windows):
// the C3/C4 workloads.  Everything else (partial last frames, raw int16 input, levels 7-8, 32-bps and
// the mid-side virtual channels) stays on k_analyze; the launcher runs it over the plan's list of partial
// subframes (known at plan creation), so this kernel finishes every subframe it starts.
//
// Why a wave and not a workgroup: k_analyze's 256-thread workgroup spends 43 % of its wave cycles
// parked at s_waitcnt / s_barrier -- eight barriers per subframe, Levinson-Durbin on 16
// lanes of one wave and the partition search on one wave while the others wait.  Here a wave owns its
// subframe end to end: no workgroup barrier, no single-wave phase, no per-wave duplicated bookkeeping.
// Lane l processes the 16-sample chunks t = 64 j + l, j = 0..3: iteration j is exactly wave j of
// k_analyze, so every FRA-1 reduction order (the chunk-partial tree per 64 chunks, then
// (G0 + G1) + (G2 + G3)) is unchanged.
//
// LDS per wave: only the 4,096 int16 samples (8 KiB, so 20 waves fit a CU); partition sums and the
// partition-search tree move between lanes by ds_bpermute / DPP, the LPC models live in scalar registers.
// The winner's zig-zag residuals overwrite the samples in place (16-bit pairs), and the encoded subframe's
// bit buffer then aliases them, filled iteration by iteration.
#include <type_traits>

#include "fra_device.h"

namespace fra {

namespace {

constexpr int kWChunks = kMaxBlock / kChunk;  // 256
constexpr int kWIters = kWChunks / 64;        // chunks per lane

// LDS per wave: exactly the 4,096 int16 samples (8 KiB: 20 waves per CU), chunk t (16 samples) at dwords
// [8t, 8t + 8).  The bit buffer aliases them (<= 2,047 words + one spare; a longer subframe takes the sample path)
struct WaveSmem {
  uint32_t sw[8 * kWChunks];
  double acf[3][9];      // FRA-1 3.5b: each window's autocorrelation (lags 0..8), read back per lane group
};
constexpr uint32_t kBufWords = 8 * kWChunks;

__device__ __forceinline__ int sdw(int t, int d) { return 8 * t + d; }
__device__ __forceinline__ int32_t wsample(const uint32_t* sw, int s) {
  const uint32_t v = sw[sdw(s >> 4, (s & 15) >> 1)];
  return (s & 1) ? hi16(v) : lo16(v);
}
// this wave's LDS stores -> its own reads (and reads before later stores): the DS instructions of one wave
// execute in order, so only the compiler must not move LDS accesses across this point -- no s_waitcnt
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
// Chunk t = 64 j + lane starts at dword 8 lane + 512 j: every sample read is a per-lane base + 512 j + an
// immediate offset, 16 bytes at a time (ds_read_b128: 16 lanes per LDS cycle at a 32-byte stride, 2-way)
constexpr int kWIterDw = 8 * 64;
constexpr int kWinW = 3;  // apodization windows of levels 3-6
__device__ __forceinline__ uint4 lds4(const uint32_t* p) { return *reinterpret_cast<const uint4*>(p); }
// D[0..5] = the last 12 samples of chunk t - 1 (zeros before the block: t == 0), D[6..13] = chunk t (int16
// pairs, sample 16t - 12 + 2k in the low half of D[k]) -- the layout read_d14 gives k_analyze
__device__ __forceinline__ void wread_d14(const uint32_t* sw, int lane, int j, uint32_t (&D)[14]) {
  const uint32_t* po = sw + 8 * lane + kWIterDw * j;
  const bool first = j == 0 && lane == 0;
  const uint32_t* pp = first ? po : po - 8;  // (a valid address; zeroed below)
  const uint4 p0 = lds4(pp), p1 = lds4(pp + 4), o0 = lds4(po), o1 = lds4(po + 4);
  D[0] = first ? 0u : p0.z; D[1] = first ? 0u : p0.w;
  D[2] = first ? 0u : p1.x; D[3] = first ? 0u : p1.y; D[4] = first ? 0u : p1.z; D[5] = first ? 0u : p1.w;
  D[6] = o0.x; D[7] = o0.y; D[8] = o0.z; D[9] = o0.w;
  D[10] = o1.x; D[11] = o1.y; D[12] = o1.z; D[13] = o1.w;
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


// Levinson-Durbin (op sequence of levinson_wave / oracle ora_levinson) where each lane keeps only what its
// order lo needs: the prediction error after step lo - 1 (e, step 0's for lo = 0) and that step's row,
// negated (lp = -lpc, the quantiser's input), so neither the rows nor the errors go through LDS
template <int MAXLAG>
__device__ inline int levinson_keep(const double (&ac)[MAXLAG + 1], int max_order, double& e, double (&lp)[MAXLAG],
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

// FRA-1 3.7 FIXED candidates from register partition sums (lane p < 2^P: partition p of order k) ==
// fixed_guess2 (fra_analyze.hip) with every order valid (n = 4096)
__device__ __forceinline__ void fixed_guess2_w(const uint32_t (&ps)[5], int P, int lane, int& g1, int& g2,
                                               uint64_t& t1, uint64_t& t2) {
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
  t1 = b1;  // their block totals (FRA-1 3.7c)
  t2 = b2;
}

// LUT fast load of one channel of a full frame into the swizzled chunks (load_lut_full_t, per wave):
// lane l loads the 8-byte vectors l + 64k (all issued before the first use), gathers each sample's audio
// value from the tile's table, packs int16 pairs and stores 4 samples per ds_write_b64.  Templated on the
// element size only: the table index is the raw bit pattern (lut_index), the same for u8/i8 and u16/i16.
// The row walk adds the uniform step = qs w + rs per vector (col < w, so at most one more wrap): no
// division per vector for any width (a per-vector division was 14 KiB of this kernel's code)
// FRA_W_ARITH (A/B knob): 0 every sample through the table; 1 every sample by normalize_to_audio's f64 op
// sequence in registers (norm_sample: the table's own entries, so bit-identical) -- 9 VALU per sample instead of
// a gather; 2 the odd vectors arithmetic, the even ones gathered
#ifndef FRA_W_ARITH
#define FRA_W_ARITH 0
#endif
struct WNorm {
  double two_mn, range, rcp;  // (-2 mn: the exact 2 (x - mn) as one fma)
  uint32_t flip;               // 0x8000 / 0x80: signed raster (raw bits -> value by (r ^ flip) - flip)
};
template <typename T>
__device__ __forceinline__ int32_t wnorm(uint32_t r, const WNorm& q) {
  const int32_t v = (int32_t)((r ^ q.flip) - q.flip);
  const double t = fma((double)v, 2.0, q.two_mn);  // 2 (x - mn), exact
  const double q0 = t * q.rcp;                     // Markstein: the correctly rounded t / range
  const double rr = fma(-q0, q.range, t);
  double u = fma(rr, q.rcp, q0);
  u = u - 1.0;
  u = u * 32767.0;
  return (int32_t)u;  // (in [-32767, 32767]: the clamps of norm_sample never act on the tile's own values)
}
template <typename T>
__device__ __forceinline__ void wload_lut(const void* base, const WaveDev& wd, int c,
                                          const int32_t* lut, uint32_t* sw, int lane, uint32_t& orv, int32_t& vmin,
                                          int32_t& vmax, bool stamp, const WNorm& wn) {
  constexpr int V = 8 / (int)sizeof(T);
  constexpr int NV = kMaxBlock / 64 / V;
  constexpr uint32_t step = 64 * V;
  using VT = VecT<T, V>;
  const uint32_t w = wd.width;
  const char* b0 = (const char*)((const T*)base + wd.off0 + (int64_t)c * wd.band_stride);
  const uint32_t rsb = wd.row_stride * (uint32_t)sizeof(T);
  const uint32_t qs = step / w, rs = step - qs * w, rstep = qs * rsb;  // uniform
  uint32_t col = wd.col0 + (uint32_t)lane * V;
  uint32_t roff = 0;
  if (col >= w) {
    const uint32_t q = col / w;
    col -= q * w;
    roff = q * rsb;
  }
  VT x[NV];
#pragma unroll
  for (int kv = 0; kv < NV; kv++) {
    x[kv] = *(const VT*)(b0 + (roff + col * (uint32_t)sizeof(T)));
    col += rs;
    roff += rstep;
    if (col >= w) { col -= w; roff += rsb; }
  }
  if (stamp) FRA_WSTAMP_WAIT(11)
  uint32_t orp = 0;
  i16x2 pmin = {32767, 32767}, pmax = {-32768, -32768};
#pragma unroll
  for (int kv = 0; kv < NV; kv++) {
    int32_t g[V];
    const bool arith = FRA_W_ARITH == 1 || (FRA_W_ARITH == 2 && (kv & 1));
    // table byte offsets from the vector's two dwords in 32 bits (r06): indexing by the element of the 8-byte
    // vector let the compiler form half of the gather addresses with 64-bit adds (v_lshl_add_u64) instead of the
    // uniform-base + 32-bit-offset form
    const uint2 xw = __builtin_bit_cast(uint2, x[kv]);
#pragma unroll
    for (int e = 0; e < V; e++) {
      constexpr int EB = 8 * (int)sizeof(T);
      const uint32_t wsrc = e < V / 2 ? xw.x : xw.y;
      const uint32_t raw = (wsrc >> (EB * (e % (V / 2)))) & ((1u << EB) - 1u);
      g[e] = arith ? wnorm<T>(raw, wn) : *(const int32_t*)((const char*)lut + (raw << 2));
    }
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
  if (stamp) FRA_WSTAMP_WAIT(12)
}

// 16-bit path: sum of |LPC residual| of order O over one chunk (lpc_abs16_raw without the kept residuals),
// warm-up positions (< O, chunk 0) masked
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

// the same sum, plus the chunk's zig-zag residuals packed two per dword (u[2p] low, u[2p+1] high: their low 16
// bits) and bit 16 of each in `hb` (bit jj; r05): exact whenever every u < 2^17, which `um`, the OR of all u, tells
template <int O, bool K17>
__device__ __forceinline__ uint32_t lpc_abs16_pk(const uint32_t (&D)[14], const int32_t* q, int sh, bool head,
                                                 uint32_t (&pk)[kChunk / 2], uint32_t& um, uint32_t& hb) {
  constexpr int NP = (O + 1) / 2;
  fra_short2 Q[NP];
  q_pairs_rev<NP>(q, Q);
  uint32_t acc = 0;
  uint32_t u[kChunk];
  hb = 0;
#pragma unroll
  for (int jj = 0; jj < kChunk; jj++) {
    const int32_t r = sample_at(D, 12 + jj) - (pred_raw<NP>(D, 12 + jj, Q) >> sh);
    const uint32_t rb = (uint32_t)r ^ kBias;
    const bool warm = jj < O && head;
    acc = sad_acc(rb, warm ? rb : kBias, acc);
    u[jj] = warm ? 0u : zz32(r);
    um |= u[jj];
  }
#pragma unroll
  for (int p = 0; p < kChunk / 2; p++) pk[p] = (u[2 * p + 1] << 16) | (u[2 * p] & 0xFFFFu);
  // bit 16 of each residual only when some lane has one (a wave-uniform branch: rare on most rasters); u >> 16 is
  // 0 or 1 whenever the kept residuals are used at all (every u < 2^17)
  if (K17 && __any(um > 0xFFFFu)) {
#pragma unroll
    for (int jj = 0; jj < kChunk; jj++) hb |= (u[jj] >> 16) << jj;
  }
  return acc;
}

}  // namespace


// (no L2 prefetch of a later wave's rows, unlike k_analyze: measured slower here at every distance,
// profiles/r04_ab_wave_prefetch_distance.txt)
// PCAP: the level's max partition order (levels 3-4: 4, 5: 5, 6: 6) as a template argument (r05): full frames
// always search orders PCAP..0 (4096 >> 7 > 8 = max order), so the group / node loops of the FIXED sums, the LPC
// sums and the partition search are straight code instead of uniform branches on a runtime order -- branches
// that also split the blocks the scheduler could otherwise overlap the ds_bpermute round trips in
// K17 (r05): kept residuals up to 17 bits (true) or 16 (false: the bit-16 masks and their corrections compiled out,
// 97 instead of 110 VGPRs, which leaves the background kernels of a pipelined execute room beside the analysis).
// The plan picks the instance per execute from the count of waves whose kept residuals needed bit 16 in an earlier
// execute (JobArgs::cnt17, both instances count them); the bytes are the same either way (FRA-1)
template <int MAXLAG, int PCAP, bool K17>
// occupancy target: 4 waves per SIMD (r05).  8 KiB of LDS would let 20 waves share a CU and <= 96 VGPRs make it 5 per
// SIMD, but at 4 (97 VGPRs here) the CU keeps 32 KiB of LDS and a wave slot per SIMD for the norm stage and the
// assembly of the neighbouring executes, which then run beside the analysis instead of in its gaps: C4 step
// 1.535-1.539 -> 1.516-1.525 ms, C3 1.062-1.068 -> 1.043-1.045, C4 8-way share 0.243-0.247 -> 0.234-0.239 same box
// (profiles/r05_ab_four_waves.txt; r04 measured this cap neutral on its kernel).  The attribute lets the compiler
// take more than 96 VGPRs, which it does for levels 5-6 (97); the level 3-4 instance stays at 95 and 5 per SIMD.
// FRA_W_WAVES=5 builds the old target
#ifndef FRA_W_WAVES
#define FRA_W_WAVES 4
#endif
#ifndef FRA_W_ACF_ITERS  // diagnostic builds only: autocorrelation over the first k 1024-sample iterations
#define FRA_W_ACF_ITERS 4
#endif
#ifndef FRA_W_VGPR_FLOOR
#define FRA_W_VGPR_FLOOR 1
#endif
#ifndef FRA_W_WAVES_MAX
#define FRA_W_WAVES_MAX 8
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(FRA_W_WAVES, FRA_W_WAVES_MAX)))
k_analyze_w(JobArgs a, int src) {
  static_assert(MAXLAG == 8 && PCAP >= 4 && PCAP <= 6, "levels 3-6");
  __shared__ WaveSmem S;
  uint32_t* const sw = S.sw;
  const int lane = (int)threadIdx.x;
#if FRA_W_VGPR_FLOOR
  // occupancy 4 waves per SIMD by register count (r06): FRA-1 3.7d brought the kernel to 93 VGPRs, which lets a
  // fifth wave per SIMD in and takes the room the pipelined step's background kernels co-run in (C4 step 1.374 ->
  // 1.42 ms, C3 0.905 -> 0.96, profiles/r06_ab_fixed_sampled.txt); a clobbered v103 keeps the allocation at 104
  asm volatile("" ::: "v103");
#endif
  FRA_WSTAMP(0)
#ifndef FRA_W_XCD
#define FRA_W_XCD 1
#endif
  // XCD-aware frame order (FRA_W_XCD): the dispatcher sends workgroup i (x fastest) to XCD i mod 8, so consecutive
  // frames -- the same tile's streams and tables -- would spread over all eight L2s; remapped, XCD k takes a
  // contiguous eighth of each channel's frames (grids of whole multiples of 8 frames; others in order).  r05: step
  // neutral on C4 / C3, C3's serial analysis -2 % (profiles/r05_ab_xcd_order.txt)
  int bx = (int)blockIdx.x;
  if (FRA_W_XCD) {
    const int nx = (int)gridDim.x, n8 = nx & ~7;
    const int lin = bx + (int)blockIdx.y * nx;  // dispatch order
    if ((nx & 7) == 0 && bx < n8) bx = (lin & 7) * (n8 >> 3) + (bx >> 3);
  }
  const int g = a.frame_base + bx;
  const int c = (int)blockIdx.y;
  const WaveDev wd = a.wave[g];
  if (c >= wd.nch) return;
  FRA_WSTAMP_WAIT(10)
  if (wd.n != kMaxBlock) return;  // partial last frames: k_analyze, over the plan's list of them
  constexpr int n = kMaxBlock;
  const int bps = wd.bps;
  const LevelCfg cfg = level_cfg(a.level);
  SfDesc* d = &a.sf[(size_t)g * a.cmax + c];
  uint32_t* const slot = a.tmp + ((size_t)g * a.cmax + c) * a.tmp_stride;
#ifdef FRA_WSTOP
  if (lane == 0) {
    d->type = 1; d->order = 0; d->wasted = 0; d->sbps = (uint8_t)bps; d->cval = 0; d->porder = 0;
    d->method = 0; d->precision = 0; d->shift = 0; d->bits = 8u + (uint32_t)n * (uint32_t)bps;
  }
#endif

  // ---- 1. load + normalise (table gather), OR / min / max
  uint32_t orv = 0;
  int32_t vmin = INT32_MAX, vmax = INT32_MIN;
  // (the lambdas capture these locals, not the kernel arguments: taking the arguments' address costs registers)
  const void* const raster = a.raster;
  const int32_t* const lut = a.lut + (int64_t)wd.stream * a.lut_stride;
  WNorm wn{};
  if (FRA_W_ARITH) {
    const NormParams np = norm_params(a.streams[wd.stream], a.norm[wd.stream]);
    wn.two_mn = -2.0 * np.mn;
    wn.range = np.range;
    wn.rcp = np.rcp;
    wn.flip = src == ST_I16 ? 0x8000u : (src == ST_I8 ? 0x80u : 0u);
  }
  auto load_samples = [&](uint32_t& ov, int32_t& mn, int32_t& mx, bool first) {
    if (src == ST_U8 || src == ST_I8) wload_lut<uint8_t>(raster, wd, c, lut, sw, lane, ov, mn, mx, first, wn);  // uniform
    else wload_lut<uint16_t>(raster, wd, c, lut, sw, lane, ov, mn, mx, first, wn);
  };
  load_samples(orv, vmin, vmax, true);
  orv = wave_or32(orv);
  wsync();  // every lane's sample stores before any lane's reads
  FRA_WSTAMP(1)
  vmin = (int32_t)(wave_min32((uint32_t)vmin ^ 0x80000000u) ^ 0x80000000u);
  vmax = (int32_t)(~wave_min32(~((uint32_t)vmax ^ 0x80000000u)) ^ 0x80000000u);
  FRA_WSTOP_AT(1, orv ^ (uint32_t)vmin ^ (uint32_t)vmax ^ sw[lane] ^ sw[2047 - lane])

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
  auto shift_wasted = [&]() {  // samples >>= w (int16 pairs, arithmetic; the pad dwords too)
    for (int k = lane; k < (int)kBufWords; k += 64) {
      const uint32_t v = sw[k];
      const uint32_t lo = (uint32_t)(lo16(v) >> w) & 0xFFFFu, hi = (uint32_t)(hi16(v) >> w);
      sw[k] = lo | (hi << 16);
    }
  };
  if (w) shift_wasted();
  wsync();
  const uint32_t hdr = 8u + (uint32_t)w;
  const uint32_t verb = hdr + (uint32_t)n * (uint32_t)sbps;
  constexpr int P = PCAP;                            // = max_porder(n, 0, cfg.max_porder)
  constexpr int gsl = 8 - P;                         // lanes per finest partition: 2^gsl (chunks of 16)
  const int prec = qlp_precision(bps, n);
  const int lmax = cfg.max_lpc;                      // < n - 1

  // ---- 3a. FIXED residual sums (3.8) by finite differences, per finest partition: group sums of the lanes
  // of a partition, gathered so that lane p holds partition p (ds_bpermute from the group's last lane)
  constexpr int npl = 6 - gsl;  // log2 finest partitions per iteration
  const int pj = lane >> npl;  // the iteration of partition `lane` (>= 4: lane >= 2^P, none)
  const int psrc = ((lane & ((1 << npl) - 1)) << gsl) | ((1 << gsl) - 1);  // its group's last lane
  // FRA-1 3.7d (r06): the five orders' sums over the even quarters of the block only (iterations j = 0, 2: chunks
  // 0-63 and 128-191 = samples [0, 1024) and [2048, 3072)) choose the two candidates; their sums over iterations 1
  // and 3 follow for those two orders alone (pass B below)
  uint32_t pfix[5] = {0, 0, 0, 0, 0};
  for (int j = 0; j < kWIters; j += 2) {
    const int t = 64 * j + lane;
    const bool head = t == 0;
    uint32_t D[14];
    wread_d14(sw, lane, j, D);
    int32_t x[28];
    unpack28(D, x);
    // biased throughout (r05): v = x + 2^31, then each difference order by one v_xad_u32 -- (a ^ 0x7FFFFFFF) + b =
    // b - a + 2^31 - 1, the next order plus a (new) constant bias that the SAD of two neighbours cancels (|values| <
    // 2^21: no wrap) -- instead of a subtract and a re-bias per sample and order
    uint32_t v[28];
#pragma unroll
    for (int jx = 8; jx < 28; jx++) v[jx] = (uint32_t)x[jx] ^ kBias;
#pragma unroll
    for (int k = 0; k <= 4; k++) {
      if (k > 1) {
#pragma unroll
        for (int jx = 12 + kChunk - 1; jx >= 7 + k; jx--) v[jx] = xad_bias(v[jx - 1], v[jx]);
      }
      uint32_t s32 = 0;
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) {
        const uint32_t ab = v[12 + jj];
        const uint32_t bb = k == 0 ? kBias : ((jj < k && head) ? ab : v[11 + jj]);
        s32 = sad_acc(ab, bb, s32);
      }
      // a partition of <= 512 samples: 2 sum |r| < 2^30
      const uint32_t gs = bperm32(group_sum32(s32, gsl), psrc);
      pfix[k] = pj == j ? 2u * gs : pfix[k];
    }
  }
  FRA_WSTAMP(2)
  FRA_WSTOP_AT(2, pfix[0] ^ pfix[1] ^ pfix[2] ^ pfix[3] ^ pfix[4])

  // ---- running winner (FRA-1 3.8: first minimal estimate in model order)
  uint32_t west = 0xFFFFFFFFu;
  int wm = 99, wtype = 2, wo = 0, wsh = 0, wps = 0;
  uint32_t wk = 0;
  // (an LPC winner's coefficients stay in mv: model m = 5 + window)
  auto offer = [&](uint32_t est, int m, int type, int o, int sh, int ps, uint32_t kreg) {
    if (est < west || (est == west && m < wm)) {
      west = est; wm = m; wtype = type; wo = o; wsh = sh; wps = ps; wk = kreg;
    }
  };

  // ---- 5a. FIXED candidates (3.7): the two orders with the smallest totals; their partition sums stay
  // in registers for the candidate loop below
  int g1, g2;
  uint64_t gt1, gt2;
  fixed_guess2_w(pfix, P, lane, g1, g2, gt1, gt2);
  uint32_t pf1 = 0, pf2 = 0;
#pragma unroll
  for (int k = 0; k < 5; k++) {
    pf1 = k == g1 ? pfix[k] : pf1;
    pf2 = k == g2 ? pfix[k] : pf2;
  }
  // pass B (3.7d): orders g1 and g2 over iterations 1 and 3 (the odd quarters), the same difference chain and SADs
  {
    const int kmax = g1 > g2 ? g1 : g2;  // (uniform)
#pragma unroll 1
    for (int j = 1; j < kWIters; j += 2) {
      uint32_t D[14];
      wread_d14(sw, lane, j, D);
      int32_t x[28];
      unpack28(D, x);
      uint32_t v[28];
#pragma unroll
      for (int jx = 8; jx < 28; jx++) v[jx] = (uint32_t)x[jx] ^ kBias;
      uint32_t s1 = 0, s2 = 0;
#pragma unroll
      for (int k = 0; k <= 4; k++) {
        if (k > kmax) break;  // (uniform)
        if (k > 1) {
#pragma unroll
          for (int jx = 12 + kChunk - 1; jx >= 7 + k; jx--) v[jx] = xad_bias(v[jx - 1], v[jx]);
        }
        if (k == g1 || k == g2) {  // (uniform; no warm-up positions here: chunk 64 j + lane > 0)
          uint32_t s32 = 0;
#pragma unroll
          for (int jj = 0; jj < kChunk; jj++) s32 = sad_acc(v[12 + jj], k == 0 ? kBias : v[11 + jj], s32);
          if (k == g1) s1 = s32;
          else s2 = s32;
        }
      }
      const uint32_t gs1 = bperm32(group_sum32(s1, gsl), psrc), gs2 = bperm32(group_sum32(s2, gsl), psrc);
      pf1 = pj == j ? 2u * gs1 : pf1;
      pf2 = pj == j ? 2u * gs2 : pf2;
    }
    // the two candidates' FULL block totals, for the gate (3.7c)
    gt1 = (uint64_t)wave_sum32(pf1);
    gt2 = (uint64_t)wave_sum32(pf2);
  }
#if defined(FRA_WPAD) && FRA_WPAD > 0
  {  // diagnostic build only (tools/gpu_r04_pad.sh): FRA_WPAD extra independent VALU instructions per wave
    uint32_t p0 = lane, p1 = lane + 1, p2 = lane + 2, p3 = lane + 3;
#pragma unroll
    for (int k = 0; k < FRA_WPAD / 4; k++) {
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(p0) : "v"(p1));
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(p1) : "v"(p2));
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(p2) : "v"(p3));
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(p3) : "v"(p0));
    }
    asm volatile("" ::"v"(p0 ^ p1 ^ p2 ^ p3));  // keep the chains alive
  }
#endif
  FRA_WSTAMP(3)
  FRA_WSTOP_AT(3, pf1 ^ pf2 ^ (uint32_t)(g1 * 8 + g2))
  // ---- 3. LPC analysis per apodization window (3.4-3.7): lane 16 wi + o_l of window wi's lane group holds
  // that window's model (order o_l, quantised q, shift qsh, ok)
  int nlpc = 0;
  // LPC model per window (levels 3-6: <= 3 windows), lane-distributed in ONE VGPR instead of 33 scalars
  // (scalar copies of every model spilled to VGPR lanes: 153 SGPR spill slots): lane 8 wi + jx = qlp
  // coefficient jx of window wi, lane 24 + wi = its shift | usable order << 8 (0: none / not quantisable).
  // Read back per candidate by v_readlane with a uniform lane index
  uint32_t mv = 0;
  if constexpr (MAXLAG > 0) {
    if (cfg.nsub > 0 && lmax > 0) {
      nlpc = a.nwin;
      const int nwin = a.nwin;
      constexpr int NL = MAXLAG + 1;
      double acl[NL];
      for (int wi = 0; wi < nwin; wi++) {
        const int32_t* wr = a.wrange + 2 * ((size_t)wd.win * a.nwin + wi);
        const int32_t* wp = a.wplat + 2 * ((size_t)wd.win * a.nwin + wi);
        const int lo = wr[0], hi = wr[1], plo = wp[0], phi = wp[1];
        const float* win = a.win + ((size_t)wd.win * a.nwin + wi) * a.blocksize;
        // FRA-1 3.5b on the matrix cores.  The windowed integer samples v (|v| < 2^15) as a 256 x 16 matrix
        // Y[k][i] = v[16 k + i] (k = 16 g + e per 1024-sample block: lane 16 g + i holds rows k of its group in
        // its 16 bytes, e = 0..15, and the next row k + 1 for the shifted copy): C0 = Y^T Y and C1 = Y^T Y'
        // (Y' = the rows one down) give R[L] = sum_{i <= 15-L} C0[i][i+L] + sum_{i >= 16-L} C1[i][i+L-16].
        // Each v = 256 h + (l + 128) with h = v >> 8 and l = (v & 255) - 128 signed bytes, the products
        // h h', h l' + l h', l l' accumulated exactly in int32 by v_mfma_i32_16x16x64_i8 (|sums| < 2^23), and
        // R[L] = 65536 HH + 256 HL + LL + 256 sum(v) - 128 sum_{m<L} v[m] - 2^26 (the offsets of the 4,096
        // pairs, samples past n being v = 0) -- exact, like the oracle's int64 sums
        const int ri = lane & 15, g4 = lane >> 4;
        i32x4 c0h = {0, 0, 0, 0}, c0m = c0h, c0l = c0h, c1h = c0h, c1m = c0h, c1l = c0h;
        int32_t ysh = 0, ysl = 0, yfirst = 0;  // sums of the samples' h and l bytes; sample of lane ri (< 16)
        const int16_t* const sh16 = reinterpret_cast<const int16_t*>(sw);
        for (int blk = 0; blk < kWIters; blk++) {
          const int b0 = 1024 * blk;
          // elements 0..15: samples b0 + 256 g4 + 16 e + ri; element 16: the next row (past n: 0).  The lane's
          // offset is opaque per block, so the per-element addresses stay immediate offsets of one base instead
          // of 17 x 4 hoisted 64-bit addresses (which spilled)
          int sb = b0 + 256 * g4 + ri;
          asm volatile("" : "+v"(sb));
          const int16_t* const sp = sh16 + sb;
          const float* const wp = win + sb;
          const int kind = (!(lo < b0 + 1024 && hi > b0) || blk >= FRA_W_ACF_ITERS) ? 0
                           : (b0 >= plo && b0 + 1024 <= phi) ? 1 : 2;  // zero / plateau (1.0f) / windowed
          uint32_t H[5], L[5];
          // two halves of 8 elements, loaded, windowed and packed in turn (all 16 in flight at once needed
          // more than the kernel's 104 VGPRs)
#pragma unroll
          for (int hf = 0; hf < 2; hf++) {
            int32_t y[8];
            if (kind == 0) {
#pragma unroll
              for (int e = 0; e < 8; e++) y[e] = 0;
            } else if (kind == 1) {
#pragma unroll
              for (int e = 0; e < 8; e++) y[e] = sp[16 * (8 * hf + e)];
            } else {
              float wc[8];
#pragma unroll
              for (int e = 0; e < 8; e++) wc[e] = wp[16 * (8 * hf + e)];
#pragma unroll
              for (int e = 0; e < 8; e++) y[e] = (int32_t)__builtin_rintf((float)sp[16 * (8 * hf + e)] * wc[e]);
            }
            if (blk == 0 && hf == 0) yfirst = y[0];
#pragma unroll
            for (int dd = 0; dd < 2; dd++) {
              const uint32_t p01 = __builtin_amdgcn_perm((uint32_t)y[4 * dd + 1], (uint32_t)y[4 * dd], 0x05010400u);
              const uint32_t p23 = __builtin_amdgcn_perm((uint32_t)y[4 * dd + 3], (uint32_t)y[4 * dd + 2], 0x05010400u);
              L[2 * hf + dd] = __builtin_amdgcn_perm(p23, p01, 0x05040100u) ^ 0x80808080u;
              H[2 * hf + dd] = __builtin_amdgcn_perm(p23, p01, 0x07060302u);
              // sum(v) from the bytes (v = 256 h + l + 128): no sample stays live past its packing
              ysh = __builtin_amdgcn_sdot4((int)H[2 * hf + dd], 0x01010101, ysh, false);
              ysl = __builtin_amdgcn_sdot4((int)L[2 * hf + dd], 0x01010101, ysl, false);
            }
            if (hf == 0) asm volatile("" ::: "memory");
          }
          int32_t y16;
          {
            const bool in = blk < kWIters - 1 || g4 < 3;  // the next row lies inside the block of n samples
            const float x16 = in ? (float)sp[256] : 0.0f;
            y16 = (int32_t)__builtin_rintf(x16 * (in ? wp[256] : 0.0f));
          }
          H[4] = (uint32_t)y16 >> 8;
          L[4] = (uint32_t)y16 ^ 0x80u;
          const i32x4 xh = {(int)H[0], (int)H[1], (int)H[2], (int)H[3]};
          const i32x4 xl = {(int)L[0], (int)L[1], (int)L[2], (int)L[3]};
          const i32x4 sh = {(int)__builtin_amdgcn_alignbyte(H[1], H[0], 1), (int)__builtin_amdgcn_alignbyte(H[2], H[1], 1),
                            (int)__builtin_amdgcn_alignbyte(H[3], H[2], 1), (int)__builtin_amdgcn_alignbyte(H[4], H[3], 1)};
          const i32x4 sl = {(int)__builtin_amdgcn_alignbyte(L[1], L[0], 1), (int)__builtin_amdgcn_alignbyte(L[2], L[1], 1),
                            (int)__builtin_amdgcn_alignbyte(L[3], L[2], 1), (int)__builtin_amdgcn_alignbyte(L[4], L[3], 1)};
          c0h = __builtin_amdgcn_mfma_i32_16x16x64_i8(xh, xh, c0h, 0, 0, 0);
          c0m = __builtin_amdgcn_mfma_i32_16x16x64_i8(xh, xl, c0m, 0, 0, 0);
          c0m = __builtin_amdgcn_mfma_i32_16x16x64_i8(xl, xh, c0m, 0, 0, 0);
          c0l = __builtin_amdgcn_mfma_i32_16x16x64_i8(xl, xl, c0l, 0, 0, 0);
          c1h = __builtin_amdgcn_mfma_i32_16x16x64_i8(xh, sh, c1h, 0, 0, 0);
          c1m = __builtin_amdgcn_mfma_i32_16x16x64_i8(xh, sl, c1m, 0, 0, 0);
          c1m = __builtin_amdgcn_mfma_i32_16x16x64_i8(xl, sh, c1m, 0, 0, 0);
          c1l = __builtin_amdgcn_mfma_i32_16x16x64_i8(xl, sl, c1l, 0, 0, 0);
        }
        // C element (row 4 g4 + q, column ri) at lane 16 g4 + ri, register q: lag (ri - 4 g4 - q) mod 16, from C0
        // when ri >= row, else C1; rotated within the row so that lane 16 g4 + L holds lag L, rows summed
        double mq = 0.0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int dd = ri - 4 * g4 - q;
          const bool in0 = dd >= 0;
          const double v = fma((double)(in0 ? c0h[q] : c1h[q]), 65536.0,
                               fma((double)(in0 ? c0m[q] : c1m[q]), 256.0, (double)(in0 ? c0l[q] : c1l[q])));
          mq = mq + __shfl(v, 16 * g4 + ((ri + 4 * g4 + q) & 15), 64);
        }
        mq = mq + __shfl_xor(mq, 16, 64);
        mq = mq + __shfl_xor(mq, 32, 64);
        const int32_t ytot = (int32_t)wave_sum32((uint32_t)(256 * ysh + ysl)) + 128 * kMaxBlock;
        int32_t pre = 0;  // sum of v[m], m < L, at lane L (samples 0..7: lanes 0..7, block 0, element 0)
#pragma unroll
        for (int m = 0; m < MAXLAG; m++) {
          const int32_t vm = __builtin_amdgcn_readlane(yfirst, m);
          pre += ri > m ? vm : 0;
        }
        const double rl = mq + (256.0 * (double)ytot - 128.0 * (double)pre - 67108864.0);
        if (lane < NL) S.acf[wi][lane] = rl;  // (through LDS: nine doubles per lane kept live across the
                                              // windows would push the phase past 128 VGPRs)
      }
      wsync();
      {
        const int gw = min(lane >> 4, nwin - 1);
#pragma unroll
        for (int l = 0; l < NL; l++) acl[l] = S.acf[gw][l];
      }
      FRA_WSTAMP(4)
#ifdef FRA_WSTOP
      {
        uint64_t kx = 0;
#pragma unroll
        for (int l = 0; l < NL; l++) kx ^= (uint64_t)__double_as_longlong(acl[l]);
        FRA_WSTOP_AT(4, kx ^ (kx >> 32))
      }
#endif
      // Levinson-Durbin, order choice and quantisation of up to 4 windows at once: window wi on lanes
      // 16 wi .. +15 (the same op sequence per lane); lane 16 wi + o holds order o's row and quantisation
      const int gw = lane >> 4, lo = lane & 15;
      const bool gon = gw < nwin;
      double lpo[MAXLAG], e = 0.0;
      int nord = 0;
      if (gon && acl[0] != 0.0) nord = levinson_keep<MAXLAG>(acl, lmax, e, lpo, lo);
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
      int32_t q[MAXLAG];
#pragma unroll
      for (int jx = 0; jx < MAXLAG; jx++) q[jx] = 0;
      bool ok = false;
      int qsh = 0;
      if (on) ok = quantize<MAXLAG>(lpo, lo, prec, q, qsh);
      const int o_l = nord > 0 ? (int)__builtin_ctz(rowbits | 0x10000u) : 0;
      // each window's model (lane 16 wi + o_wi) gathered into mv (o = 0: none): lane l < 24 takes coefficient
      // l & 7 of window l >> 3, lane 24 + wi the shift and usable order (every ds_bpermute on all 64 lanes)
      const int dwi = lane < 24 ? lane >> 3 : (lane - 24) & 3;
      const int ow = (int)bperm32((uint32_t)o_l, 16 * dwi);
      const int L = 16 * dwi + ow;
      // (computed at the SOURCE lane 16 wi + o_wi from its own values: its order o_l == lo there)
      const uint32_t info = (uint32_t)qsh | ((o_l > 0 && ok) ? (uint32_t)o_l << 8 : 0u);
      const uint32_t vinfo = bperm32(info, L);
#pragma unroll
      for (int jx = 0; jx < 8; jx++) {
        const uint32_t vq = bperm32((uint32_t)q[jx], L);
        mv = (lane & 7) == jx ? vq : mv;
      }
      mv = lane >= 24 ? vinfo : mv;
      mv = (lane < 24 ? dwi : lane - 24) < nwin && lane < 27 ? mv : 0u;
    }
  }
  FRA_WSTAMP(5)
#ifdef FRA_WSTOP
  {
    const uint32_t kx = wave_or32(mv ^ (uint32_t)lane);
    FRA_WSTOP_AT(5, kx)
  }
#endif

  // ---- 4+5. the candidates -- each window's LPC model, then FIXED g1, g2 (r06: LPC first, so that FRA-1 3.7c can drop
  // a FIXED candidate whose block total is not below the LPC models' smallest one before its search; the winner is
  // still the first minimal estimate in model order, FIXED first: offer() compares (estimate, model index)) -- one
  // partition search each (one code body); an LPC model first gets its residual sums at the finest partitions.
  // The keep window's model is summed last among the LPC models: its pass replaces each chunk's samples in LDS by
  // the chunk's zig-zag residuals (int16 pairs), which the exact pass and the encoder then read instead of
  // recomputing the predictor twice (fallback: the samples are loaded again)
  // windows with a usable model (lanes 24 + wi of mv with an order)
  const uint32_t okm = (uint32_t)(__ballot(lane >= 24 && lane < 24 + kWinW && (mv >> 8) != 0) >> 24);
  // the window whose residuals are kept: the first usable one (FRA_W_KEEP=0; window 0, the whole-block tukey,
  // is the likeliest winner) or the last (FRA_W_KEEP=1); its sum pass runs last, after the other windows' passes
#ifndef FRA_W_KEEP
#define FRA_W_KEEP 0
#endif
  const int keep_wi = okm ? (FRA_W_KEEP ? 31 - __clz((int)okm) : __builtin_ctz(okm)) : -1;
  bool kept_fit = false;
  uint64_t hk = 0;  // bit 16 of the kept residuals: bit 16 j + jj = chunk 64 j + lane's residual jj
  bool hk_any = false;  // (wave-uniform) some kept residual has bit 16
  uint32_t w4[4] = {0, 0, 0, 0};  // samples 0..7 (the warm-up), saved before chunk 0 is overwritten
  uint64_t lpcT = ~0ull;  // the smallest block total of 2|r| of the LPC models summed (FRA-1 3.7c)
#pragma unroll 1
  for (int ci = 0; ci < nlpc + 2; ci++) {
    int m, o, sh = 0, type = 2;
    int32_t qm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t psum = 0;
    if (ci >= nlpc) {  // FIXED g1, g2 -- dropped when not below the LPC models' block total (3.7c)
      m = o = ci == nlpc ? g1 : g2;
      if (o < 0 || (lpcT != ~0ull && (ci == nlpc ? gt1 : gt2) >= lpcT)) continue;
      psum = ci == nlpc ? pf1 : pf2;
    } else {
      const int wi = (ci + keep_wi + 1) % nlpc;  // the keep window last (nlpc >= 1 here)
      if (!((okm >> wi) & 1u)) continue;  // no order / not quantisable
      const uint32_t inf = (uint32_t)__builtin_amdgcn_readlane((int)mv, 24 + wi);
      o = (int)(inf >> 8);
      m = 5 + wi;
      type = 3;
      sh = (int)(inf & 0xFFu);
#pragma unroll
      for (int jx = 0; jx < 8; jx++) qm[jx] = __builtin_amdgcn_readlane((int)mv, 8 * wi + jx);
      if (wi == keep_wi) {
        uint32_t um = 0, carry[6] = {0, 0, 0, 0, 0, 0};
        // iteration 0 (the only one holding the warm-up samples, lane 0) peeled: the others are compiled with head
        // false, without the warm-up selects (r05)
        auto keep_iter = [&](const int j, auto headc) {
          constexpr bool kHead = decltype(headc)::value;
          const bool head = kHead && lane == 0;
          uint32_t* const po = sw + 8 * lane + kWIterDw * j;
          uint32_t D[14];
          wread_d14(sw, lane, j, D);
          if (j > 0) {  // chunk 64 j - 1 already holds residuals: its last 12 samples came from lane 63
#pragma unroll
            for (int k = 0; k < 6; k++) D[k] = lane == 0 ? carry[k] : D[k];
          }
#pragma unroll
          for (int k = 0; k < 6; k++) carry[k] = (uint32_t)__builtin_amdgcn_readlane((int)D[8 + k], 63);
          if (j == 0) {
#pragma unroll
            for (int k = 0; k < 4; k++) w4[k] = (uint32_t)__builtin_amdgcn_readlane((int)D[6 + k], 0);
          }
          uint32_t acc = 0, pk[kChunk / 2], hb = 0;
          switch (o) {
#define FRA_CASE(O_) \
  case O_: acc = lpc_abs16_pk<O_, K17>(D, qm, sh, head, pk, um, hb); break;
            FRA_CASE(1) FRA_CASE(2) FRA_CASE(3) FRA_CASE(4) FRA_CASE(5) FRA_CASE(6) FRA_CASE(7) FRA_CASE(8)
#undef FRA_CASE
          }
          wsync();  // (all lanes' sample reads of this iteration precede the stores)
#pragma unroll
          for (int p = 0; p < kChunk / 4; p++) *reinterpret_cast<uint2*>(po + 2 * p) = make_uint2(pk[2 * p], pk[2 * p + 1]);
          hk |= (uint64_t)hb << (16 * j);
          const uint64_t gs = bperm64(group_sum_auto(2ull * acc, gsl), psrc);
          psum = pj == j ? gs : psum;
        };
        keep_iter(0, std::true_type{});
#pragma unroll 1
        for (int j = 1; j < kWIters; j++) keep_iter(j, std::false_type{});
        const bool need17 = __any(um > 0xFFFFu) && !__any(um > 0x1FFFFu);  // (wave-uniform)
        if (need17 && lane == 0 && a.cnt17) atomicAdd(a.cnt17, 1u);  // (a vector atomic: lane 0 only)
        if constexpr (K17) {
          kept_fit = !__any(um > 0x1FFFFu);  // 16 bits in LDS + bit 16 in hk
          hk_any = __any(hk != 0);
        } else {
          kept_fit = !__any(um > 0xFFFFu);
        }
      } else {
#pragma unroll 1
        for (int j = 0; j < kWIters; j++) {
          const int t = 64 * j + lane;
          const bool head = t == 0;
          uint32_t D[14];
          wread_d14(sw, lane, j, D);
          uint32_t acc = 0;
          switch (o) {
#define FRA_CASE(O_) \
  case O_: acc = lpc_abs16_w<O_>(D, qm, sh, head); break;
            FRA_CASE(1) FRA_CASE(2) FRA_CASE(3) FRA_CASE(4) FRA_CASE(5) FRA_CASE(6) FRA_CASE(7) FRA_CASE(8)
#undef FRA_CASE
          }
          const uint64_t gs = bperm64(group_sum_auto(2ull * acc, gsl), psrc);
          psum = pj == j ? gs : psum;
        }
      }
      // the model's block total (lanes >= 2^P hold 0)
      uint64_t tv = psum;
      tv = up_add64<0>(tv); tv = up_add64<1>(tv); tv = up_add64<2>(tv);
      tv = up_add64<3>(tv); tv = up_add64<4>(tv); tv = up_add64<5>(tv);
      const uint64_t T = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(tv >> 32), 63) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)tv, 63);
      lpcT = T < lpcT ? T : lpcT;
    }
    constexpr int pm = P;  // max_porder(n, o, cfg.max_porder) == P for n = 4096, o <= 8
    uint64_t best;
    int bp;
    uint32_t kreg;
    porder_search_reg(psum, P, pm, n, o, lane, best, bp, kreg);
    const uint64_t est = hdr + (uint64_t)o * sbps + (type == 3 ? 9 + (uint64_t)o * prec : 0) + best;
    offer((uint32_t)est, m, type, o, sh, bp, kreg);
  }

  FRA_WSTAMP(6)
  FRA_WSTOP_AT(6, west ^ (uint32_t)wm ^ (uint32_t)wps)
  // ---- 6. the winner's zig-zag residuals, exact Rice bits with each partition's parameter refined (3.9),
  // encode (RFC 9639 9.2).  Two instances:
  //  * kept (the common case): the winner is the LPC model of the keep pass and every residual fits 16 bits:
  //    residuals read as int16 pairs from the samples' place, the bit buffer in LDS aliasing them;
  //  * otherwise (a FIXED order, another window, residuals past 16 bits): the samples (loaded again if the keep
  //    pass overwrote them) and the winner's predictor, the codes ORed straight into the slot in global memory.
  // A kept subframe that is not smaller than VERBATIM, or whose encode would overrun its residuals in the
  // aliased buffer, takes the second instance after the samples are loaded again: every full frame ends here
  const int type = wtype, o = wo, sh = wsh, ps = wps;
  int32_t wq[8];
#pragma unroll
  for (int jq = 0; jq < 8; jq++) wq[jq] = type == 3 ? __builtin_amdgcn_readlane((int)mv, 8 * (wm - 5) + jq) : 0;
  const bool kept_w = type == 3 && wm == 5 + keep_wi && kept_fit;
  FRA_WSTAMP_VAL(9, kept_w ? 0 : (type != 3 ? 3 : (wm != 5 + keep_wi ? 4 : 5)))  // why the sample path
  auto reload = [&]() {  // the keep pass replaced the samples: load them once more
    wsync();
    uint32_t ov = 0;
    int32_t mn = 0, mx = 0;
    load_samples(ov, mn, mx, false);
    wsync();
    if (w) shift_wasted();
    wsync();
  };
  const int pz = n >> ps;
  const int tl = 8 - ps;                  // log2 chunks per partition (2..8)
  const int ls = tl < 6 ? tl : 6;         // lanes per partition group inside one iteration
  const int npp = 1 << ps;
  auto tail = [&](auto kept_tag) {
    constexpr bool kept = decltype(kept_tag)::value;
    int32_t warm = 0;  // warm-up sample `lane`
    if (kept) {
      const uint32_t wv2 = lane >= 6 ? w4[3] : lane >= 4 ? w4[2] : lane >= 2 ? w4[1] : w4[0];
      warm = lane < o ? ((lane & 1) ? hi16(wv2) : lo16(wv2)) : 0;
    } else if (lane < o) {
      warm = wsample(sw, lane);
    }
    fra_short2 Q[4];
    q_pairs_rev<4>(wq, Q);
    // the residuals of chunk 64 j + lane (warm-up positions 0).  Sample path: chunk 64 j - 1's last 12 samples
    // (lane 0's look-back) come from cy, lane 63's words of the previous call, so iteration j - 1's bit-buffer
    // words may already cover that chunk (calls in order j = 0..3)
    auto residuals = [&](int j, uint32_t (&un)[kChunk], uint32_t (&cy)[6]) {
      const int t = 64 * j + lane;
      if (kept) {  // 8 dwords of u16 pairs (+ bit 16 of each from hk when the wave has any)
        const uint32_t* po = sw + 8 * lane + kWIterDw * j;
#pragma unroll
        for (int p = 0; p < kChunk / 4; p++) {
          const uint2 v = *reinterpret_cast<const uint2*>(po + 2 * p);
          un[4 * p] = v.x & 0xFFFFu;
          un[4 * p + 1] = v.x >> 16;
          un[4 * p + 2] = v.y & 0xFFFFu;
          un[4 * p + 3] = v.y >> 16;
        }
        if (hk_any) {
          const uint32_t h = (uint32_t)(hk >> (16 * j));
#pragma unroll
          for (int jj = 0; jj < kChunk; jj++) un[jj] |= ((h >> jj) & 1u) << 16;
        }
        return;
      }
      uint32_t D[14];
      wread_d14(sw, lane, j, D);
      if (j > 0) {
#pragma unroll
        for (int k = 0; k < 6; k++) D[k] = lane == 0 ? cy[k] : D[k];
      }
#pragma unroll
      for (int k = 0; k < 6; k++) cy[k] = (uint32_t)__builtin_amdgcn_readlane((int)D[8 + k], 63);
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
#pragma unroll
      for (int jj = 0; jj < 12; jj++)
        if (t == 0 && jj < o) un[jj] = 0u;
    };
    uint32_t kc[kWIters];       // Rice parameter of the lane's chunk of iteration j
    uint32_t fk[kWIters][3];    // sums of u >> (k0 - 1), u >> k0, u >> (k0 + 1) of that chunk
    uint32_t k0r[kWIters];
    uint32_t bitsl = 0;         // exact bits of the partitions this lane leads
    bool bigl = false;
    uint64_t E[3] = {0, 0, 0};  // partitions spanning iterations (ps <= 1): running sums
    uint32_t cyx[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < kWIters; j++) {
      const int t = 64 * j + lane;
      const int pidx = t >> tl;
      const int k0 = __shfl((int)wk, pidx & 63, 64);
      const int km = k0 > 0 ? k0 - 1 : 0;
      uint32_t f0 = 0, f1 = 0, f2 = 0;  // u < 2^28: 16 of them fit 32 bits
      if constexpr (kept) {
        // the kept residuals are u16 pairs: one v_pk_lshrrev_b16 + one v_dot2_u32_u16 (both halves times 1, into
        // 32 bits) per pair and shift -- half the instructions of the per-sample shifts and adds
        const uint32_t* po = sw + 8 * lane + kWIterDw * j;
        // (a u16 shifted by >= 16 is 0: the shift is capped at 15 and the pair weighted 0 instead -- the hardware
        // takes the shift count mod 16)
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        auto sh = [](int k) -> u16x2 {
          const unsigned short c = (unsigned short)(k < 15 ? k : 15);
          return u16x2{c, c};
        };
        auto wt = [](int k) -> u16x2 {
          const unsigned short c = k < 16 ? 1 : 0;
          return u16x2{c, c};
        };
        const u16x2 sm = sh(km), s0 = sh(k0), s1 = sh(k0 + 1), mm = wt(km), m0 = wt(k0), m1 = wt(k0 + 1);
        // bit 16 of a residual adds 2^16 >> k to u >> k (k <= 16; 0 above: u < 2^17): c of them in this chunk
        if (hk_any) {
          const uint32_t c = (uint32_t)__builtin_popcount((uint32_t)(hk >> (16 * j)) & 0xFFFFu);
          f0 = km <= 16 ? c << (16 - km) : 0u;
          f1 = k0 <= 16 ? c << (16 - k0) : 0u;
          f2 = k0 + 1 <= 16 ? c << (15 - k0) : 0u;
        }
#pragma unroll
        for (int p = 0; p < kChunk / 4; p++) {
          const uint2 v = *reinterpret_cast<const uint2*>(po + 2 * p);
          const u16x2 w0 = __builtin_bit_cast(u16x2, v.x), w1 = __builtin_bit_cast(u16x2, v.y);
          f0 = __builtin_amdgcn_udot2(w0 >> sm, mm, f0, false);
          f0 = __builtin_amdgcn_udot2(w1 >> sm, mm, f0, false);
          f1 = __builtin_amdgcn_udot2(w0 >> s0, m0, f1, false);
          f1 = __builtin_amdgcn_udot2(w1 >> s0, m0, f1, false);
          f2 = __builtin_amdgcn_udot2(w0 >> s1, m1, f2, false);
          f2 = __builtin_amdgcn_udot2(w1 >> s1, m1, f2, false);
        }
      } else {
        uint32_t un[kChunk];
        residuals(j, un, cyx);
#pragma unroll
        for (int jj = 0; jj < kChunk; jj++) {
          f0 += un[jj] >> km;
          f1 += un[jj] >> k0;
          f2 += un[jj] >> (k0 + 1);
        }
      }
      fk[j][0] = f0;
      fk[j][1] = f1;
      fk[j][2] = f2;
      k0r[j] = (uint32_t)k0;
      uint64_t v0, v1, v2;
      if (kept || __all(f0 <= (0xFFFFFFFFu >> ls))) {  // (kept: u < 2^17, so <= 64 lanes fit 32 bits)
        v0 = group_sum32(f0, ls); v1 = group_sum32(f1, ls); v2 = group_sum32(f2, ls);
      } else {
        v0 = group_sum64(f0, ls); v1 = group_sum64(f1, ls); v2 = group_sum64(f2, ls);
      }
      if (tl <= 6) {  // the partition lies inside this iteration: its last lane decides
        // (evaluated on every lane -- no exec masking -- and kept on the partition's last lane)
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
        auto rl64 = [](uint64_t v) -> uint64_t {
          return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63) |
                 ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63) << 32);
        };
        E[0] += rl64(v0);
        E[1] += rl64(v1);
        E[2] += rl64(v2);
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
          for (int jx = 0; jx < kWIters; jx++)
            if (jx <= j && jx > j - span) kc[jx] = (uint32_t)bk;
          E[0] = E[1] = E[2] = 0;
        }
      }
    }
    FRA_WSTAMP(7)
    const bool big = __any(bigl);
    const uint64_t rtot = (uint64_t)wave_sum32(bitsl) + (uint64_t)npp * (big ? 5 : 4) + 6;
    const uint64_t exact = hdr + (uint64_t)o * sbps + (type == 3 ? 9 + (uint64_t)o * prec : 0) + rtot;
    FRA_WSTOP_AT_T(7, exact)
    const bool verbatim = exact >= verb;
    const uint32_t smask = (1u << sbps) - 1u;  // sbps <= 16
    if (kept && verbatim) {  // VERBATIM wants the samples: the sample path after a reload
      FRA_WSTAMP_VAL(9, 6)
      return false;
    }
    if (!kept && verbatim) {  // straight from the samples to the slot
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
        for (int s = s0; s < n && (int64_t)hdr + (int64_t)s * sbps < wb + 32; s++) {
          const int64_t rel = (int64_t)hdr + (int64_t)s * sbps - wb;
          const int sft = 32 - (int)rel - sbps;
          const uint64_t v = (uint64_t)((uint32_t)wsample(sw, s) & smask);
          word |= sft >= 0 ? (uint32_t)(v << sft) : (uint32_t)(v >> -sft);
        }
        slot[jw] = word;
      }
      return true;
    }
    // code bits of each chunk from the exact pass's sums; the bit position of every iteration's first code
    const uint32_t fbits = (uint32_t)exact;
    const uint32_t nw = (fbits + 31) >> 5;
    const int pb = big ? 5 : 4;
    const uint32_t pos = hdr + (uint32_t)o * sbps + (type == 3 ? 9u + (uint32_t)o * prec : 0u);
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
    // the LDS bit buffer aliases the residuals (kept) or samples and is filled iteration by iteration, each
    // iteration's residuals computed before its words are zeroed and written: iteration j's last word + the
    // spare one must stay below chunk 64 (j + 1)'s first word.  Else (a poorly compressible start before a
    // compressible rest) the kept instance hands over to the sample path, which ORs the codes into the slot
    // in global memory
    bool inlds = nw + 1 <= kBufWords;  // the whole subframe + the spare word fit the buffer
#pragma unroll
    for (int j = 0; j + 1 < kWIters; j++) inlds = inlds && (B[j + 1] - 1) / 32 + 2 <= (uint32_t)sdw(64 * (j + 1), 0);
    if (kept && !inlds) {
      FRA_WSTAMP_VAL(9, 7)
      return false;
    }
    if (lane < kMaxLpc) {
      int32_t cv = 0;
#pragma unroll
      for (int jq = 0; jq < 8; jq++) cv = lane == jq ? wq[jq] : cv;
      d->coef[lane] = type == 3 ? cv : 0;
    }
    if (lane == 0) {
      d->wasted = (uint8_t)w; d->sbps = (uint8_t)sbps; d->cval = 0;
      d->type = (uint8_t)type; d->order = (uint8_t)o; d->porder = (uint8_t)ps; d->method = big ? 1 : 0;
      d->precision = (uint8_t)(type == 3 ? prec : 0); d->shift = (int8_t)sh; d->bits = (uint32_t)exact;
    }
    // subframe header, warm-up samples, qlp precision / shift / coefficients, residual coding method + order
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
      if (type == 3 && lane < o) {
        int32_t cv = 0;
#pragma unroll
        for (int jq = 0; jq < 8; jq++) cv = lane == jq ? wq[jq] : cv;
        lds_put(buf, ph + 9 + (uint32_t)lane * prec, (uint32_t)cv & ((1u << prec) - 1u), prec);
      }
      if (lane == 0) lds_put(buf, pos, ((uint32_t)(big ? 1 : 0) << 4) | (uint32_t)ps, 6);
    };
    // the partition parameter (in front of a partition's first chunk) and the lane's 16 Rice codes
    auto put_codes = [&](uint32_t* buf, int j, const uint32_t (&un)[kChunk]) {
      const int t = 64 * j + lane;
      const bool head = t == 0;
      const uint32_t kcur = kc[j], tot = totl[j];
      const bool pstart = ((t << 4) & (pz - 1)) == 0;
      uint32_t p = B[j] + wave_incl_scan32(tot) - tot;
      if (pstart) { lds_put(buf, p, kcur, pb); p += (uint32_t)pb; }
      // Rice code (stop bit + kcur low bits) left-aligned: bit 31 = the stop bit
      const uint32_t sal = 31u - kcur;
      // (warm-up positions -- lane 0 of iteration 0 -- OR nothing and do not advance: selects, not a branch)
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) {
        const bool skip = jj < 12 && head && jj < o;
        const uint32_t Pp = p + (un[jj] >> kcur);
        lds_put_al(buf, Pp, skip ? 0u : ((un[jj] << sal) | 0x80000000u));
        p = skip ? p : Pp + 1u + kcur;
      }
    };
    uint32_t cye[6] = {0, 0, 0, 0, 0, 0};
    if (kept || inlds) {
      uint32_t* const buf = sw;
      uint32_t Z = 0;  // words [0, Z) are zeroed (and possibly written)
#pragma unroll
      for (int j = 0; j < kWIters; j++) {
        uint32_t un[kChunk];
        residuals(j, un, cye);
        wsync();  // every lane's reads of this iteration's residuals precede the zeroing
        const uint32_t Zend = j == kWIters - 1 ? nw + 1 : (B[j + 1] - 1) / 32 + 2;
        for (uint32_t jw = Z + lane; jw < Zend; jw += 64) buf[jw] = 0u;
        Z = Zend > Z ? Zend : Z;
        wsync();
        if (j == 0) put_header(buf);
        put_codes(buf, j, un);
      }
      wsync();
      for (uint32_t jw = lane; jw < nw; jw += 64) slot[jw] = buf[jw];
      FRA_WSTAMP(8)
    } else {  // codes ORed into the zeroed slot (global atomics)
      for (uint32_t jw = lane; jw <= nw; jw += 64) slot[jw] = 0u;  // (nw + 1 <= tmp_stride)
      __threadfence();
      put_header(slot);
#pragma unroll 1
      for (int j = 0; j < kWIters; j++) {
        uint32_t un[kChunk];
        residuals(j, un, cye);
        put_codes(slot, j, un);
      }
    }
    return true;
  };
  // the kept instance hands a VERBATIM or overrunning subframe to the sample path (samples loaded again)
  // the kept instance hands a VERBATIM or overrunning subframe to the sample path (samples loaded again; one
  // call site of the reload)
  if (!kept_w || !tail(std::true_type{})) {
    if (keep_wi >= 0) reload();
    tail(std::false_type{});
  }
}

#ifdef FRA_STAMPS
}  // namespace fra
extern "C" __attribute__((visibility("default"))) int fra_diag_wstamps(void* host, unsigned long long bytes) {
  if (!host) {
    void* d = nullptr;
    if (hipGetSymbolAddress(&d, HIP_SYMBOL(fra::g_fra_wstamps)) != hipSuccess) return -1;
    return hipMemset(d, 0, sizeof(fra::g_fra_wstamps)) == hipSuccess ? 0 : -1;
  }
  const size_t nb = bytes < sizeof(fra::g_fra_wstamps) ? bytes : sizeof(fra::g_fra_wstamps);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(fra::g_fra_wstamps), nb, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
namespace fra {
#endif

hipError_t launch_analyze_w(int src, int level, const JobArgs& a, int cw, hipStream_t s) {
  const bool k17 = a.k17 != 0;
  if (a.frame_count <= 0) return hipSuccess;
  const dim3 grid((unsigned)a.frame_count, (unsigned)cw);
  const LevelCfg cfg = level_cfg(level);
  if (cfg.nsub == 0 || cfg.max_lpc > 8) return hipErrorInvalidValue;  // levels 3-6 only
  if (!a.wave) return hipErrorInvalidValue;  // the plan's per-frame descriptors (wave-path plans)
  switch (cfg.max_porder) {
    case 4: k17 ? k_analyze_w<8, 4, true><<<grid, 64, 0, s>>>(a, src) : k_analyze_w<8, 4, false><<<grid, 64, 0, s>>>(a, src); break;
    case 5: k17 ? k_analyze_w<8, 5, true><<<grid, 64, 0, s>>>(a, src) : k_analyze_w<8, 5, false><<<grid, 64, 0, s>>>(a, src); break;
    default: k17 ? k_analyze_w<8, 6, true><<<grid, 64, 0, s>>>(a, src) : k_analyze_w<8, 6, false><<<grid, 64, 0, s>>>(a, src); break;
  }
  return hipGetLastError();
}

}  // namespace fra
