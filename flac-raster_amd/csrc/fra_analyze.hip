// fra_analyze.hip -- k_analyze: one workgroup (256 threads, 4 waves) per subframe (frame x channel).
//
// Replaces libFLAC 1.4.3's per-channel analysis inside FLAC__stream_encoder_process_interleaved
// (driven by pyflac at src/flac_raster/converter.py:153 / spatial_encoder.py:303), fused with
// normalize_to_audio (normalization.py:126-202) and the band interleave (converter.py:99-110).
// Decision rule FRA-1 == oracle/fr_oracle.c analyze_subframe():
//
//   1. load + normalise the subframe (lane-contiguous HBM reads, all 16 per thread in flight;
//      Markstein division for integer dtypes), OR/min/max reductions
//   2. CONSTANT if min == max, else wasted bits = ctz(OR), shift
//   3. per apodization window: windowed float samples in registers -> 16-sample chunk partial
//      autocorrelations (fp64, exact products) -> the FRA-1 pairwise tree over the 256 chunks,
//      done with DPP row_shr / row_bcast (each pair summed at its upper lane: same two operands,
//      and IEEE addition is commutative) + a fixed cross-wave step -> Levinson-Durbin (lane 0) ->
//      qlp quantisation (one lane per order)
//   4. residual partition sums of every candidate model at the finest partition order.  All
//      models share ONE code body: FIXED order o is the integer predictor [1], [2,-1], [3,-3,1],
//      [4,-6,4,-1] with shift 0 (the same integers as the oracle's fixed formulas), LPC uses its
//      qlp coefficients; the 16-bit path multiplies with v_mad_i32_i24 (|x| < 2^16, |q| < 2^15).
//      One body keeps the executed code footprint inside the instruction cache.
//   5. all partition orders of a model in one pass (one wave per model): DPP upper-lane group
//      sums, Rice estimate per partition leader, per-order totals by DPP wave sums
//   6. winner = first minimal estimate (DPP argmin); exact Rice bits for the winner with k refined
//      over k-1..k+1; VERBATIM if not smaller
#include <algorithm>
#include <type_traits>

#if defined(FRA_STAMPS) && defined(FRA_STAMPS_FINE)
// finer load-phase stamps: thread 0 after the value `dep` has arrived (the data dependency orders the
// stamp after the load it depends on)
namespace fra { extern __device__ unsigned long long g_fra_stamps[]; }
#define FRA_LOAD_STAMP(k, dep)                                                                       \
  if (threadIdx.x == 0 && (dep) != 0x7FFFFFF1) {                                                     \
    const unsigned wgi_ = blockIdx.x * gridDim.y + blockIdx.y;                                       \
    if (wgi_ < (1u << 17)) g_fra_stamps[wgi_ * 20u + (k)] = __builtin_amdgcn_s_memtime();            \
  }
// lane 0 of the calling wave (per-role finish times inside a phase)
#define FRA_ROLE_STAMP(k)                                                                            \
  if ((threadIdx.x & 63) == 0) {                                                                     \
    const unsigned wgi_ = blockIdx.x * gridDim.y + blockIdx.y;                                       \
    if (wgi_ < (1u << 17)) g_fra_stamps[wgi_ * 20u + (k)] = __builtin_amdgcn_s_memtime();            \
  }
#else
#define FRA_ROLE_STAMP(k)
#endif
#include "fra_device.h"

namespace fra {

#ifdef FRA_STAMPS
// diagnostic build only (csrc/Makefile `stamps`, tools/stamp_phases.py): wave 0 of the first kStampWG
// workgroups stores s_memtime after each phase barrier, so phase durations are measured inside the
// real, mixed steady state (every other workgroup keeps running the full kernel)
constexpr unsigned kStampWG = 1u << 17, kStampN = 20;
__device__ unsigned long long g_fra_stamps[kStampWG * kStampN];
#define FRA_STAMP(k)                                                                          \
  if (threadIdx.x == 0) {                                                                      \
    const unsigned wgi_ = blockIdx.x * gridDim.y + blockIdx.y;                                 \
    if (wgi_ < kStampWG) g_fra_stamps[wgi_ * kStampN + (k)] = __builtin_amdgcn_s_memtime();   \
  }
#else
#define FRA_STAMP(k)
#endif

// encoded-subframe buffer: >= (max subframe bits + 31) / 32 + 1 words (VERBATIM bound)
template <bool B32>
constexpr int buf_words() { return B32 ? kMaxBlock + 16 : kMaxBlock / 2 + 16; }

// per-thread sample windows from the LDS array (chunk stride smp_stride<T>() elements):
//   read_x28: x[j] = sample 16t - 12 + j (the previous chunk's last 12, the zero chunk for t = 0)
//   read_y24: y[j] = sample 16t + j, j < 24 (this chunk + the next chunk's first 8)
// int16 storage is read as aligned dword pairs and sign-extended (2 samples per ds_read lane-dword)
__device__ __forceinline__ void read_x28(const int32_t* smp, int t, int32_t (&x)[28]) {
#pragma unroll
  for (int j = 0; j < 12; j++) x[j] = smp[t * smp_stride<int32_t>() + 4 + j];
#pragma unroll
  for (int j = 0; j < 16; j++) x[12 + j] = smp[(t + 1) * smp_stride<int32_t>() + j];
}
__device__ __forceinline__ void read_x28(const int16_t* smp, int t, int32_t (&x)[28]) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(smp);  // kSmpStride even: chunk starts dword-aligned
#pragma unroll
  for (int j = 0; j < 6; j++) {
    const uint32_t v = d[(t * kSmpStride + 4) / 2 + j];
    x[2 * j] = lo16(v);
    x[2 * j + 1] = hi16(v);
  }
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint32_t v = d[(t + 1) * kSmpStride / 2 + j];
    x[12 + 2 * j] = lo16(v);
    x[13 + 2 * j] = hi16(v);
  }
}
__device__ __forceinline__ void read_y24(const int32_t* smp, int t, int32_t (&y)[24]) {
#pragma unroll
  for (int j = 0; j < 16; j++) y[j] = smp[(t + 1) * smp_stride<int32_t>() + j];
#pragma unroll
  for (int j = 0; j < 8; j++) y[16 + j] = smp[(t + 2) * smp_stride<int32_t>() + j];
}
__device__ __forceinline__ void read_y24(const int16_t* smp, int t, int32_t (&y)[24]) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(smp);
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint32_t v = d[(t + 1) * kSmpStride / 2 + j];
    y[2 * j] = lo16(v);
    y[2 * j + 1] = hi16(v);
  }
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t v = d[(t + 2) * kSmpStride / 2 + j];
    y[16 + 2 * j] = lo16(v);
    y[17 + 2 * j] = hi16(v);
  }
}


// windows per block at this lag bound (levels 3-6: <= 3 with max_lpc 8; levels 7-8: <= 6)
template <int MAXLAG>
constexpr int kWinCap() { return MAXLAG == 0 ? 1 : (MAXLAG <= 8 ? 3 : kMaxWin); }

template <bool B32, int MAXLAG>
struct AnalyzeSmem {
  // sample i at sidx(i); [0, kSmpStride) = zero chunk.  16-bit path: int16 (every sample fits), which
  // keeps the workgroup at <= 32 KiB LDS (5 workgroups per CU at 96 VGPRs)
  using SmpT = typename std::conditional<B32, int32_t, int16_t>::type;
  SmpT smp[smp_words<SmpT>()];
  // the encoded subframe (big-endian words, MSB first) is built in smp, dead once the winner's residuals
  // are in registers (32-bps: <= 40 KiB, 4 workgroups per CU instead of 3; 16-bit: <= 22.75 KiB)
  union {
    unsigned long long psum[kMaxModels][kMaxPart];  // reused as esum[kMaxPart][3] for the winner
    // 32-bps: the autocorrelation partials and Levinson-Durbin rows live in the LPC models' sums, which are
    // zeroed again once the models are quantised (32 KiB of LDS: 5 workgroups per CU)
    struct {
      unsigned long long fixed[5][kMaxPart];
      double red[B32 ? kWinCap<MAXLAG>() : 1][4][MAXLAG + 1];
      double lp[B32 ? kWinCap<MAXLAG>() : 1][MAXLAG > 0 ? lp_row(MAXLAG) : 1];
    } ov;
  } u;
  int32_t warm[kMaxLpc];  // warm-up samples, saved before smp is reused as the bit buffer
  union {  // (a union of one since the partition search left LDS)
    struct {  // after the model search: winner's exact-pass sums / Rice parameters
      unsigned long long esum2[kMaxPart][3];  // fast frames: sums of u >> (k0-1), u >> k0, u >> (k0+1)
      int32_t kpart[kMaxPart];
      int32_t kfin[kMaxPart];
    } e;
  } nu;
  // 16-bit instances: per window, per wave: reduced chunk partials; LD rows per window (triangular)
  double red_[B32 ? 1 : kWinCap<MAXLAG>()][4][MAXLAG + 1];
  double lp_[B32 ? 1 : kWinCap<MAXLAG>()][MAXLAG > 0 ? lp_row(MAXLAG) : 1];
  __device__ auto& red() { if constexpr (B32) return u.ov.red; else return red_; }
  __device__ auto& lp() { if constexpr (B32) return u.ov.lp; else return lp_; }
  // model table in the narrowest types (16-bit path: 7 workgroups per CU need <= 22.5 KiB of LDS):
  // qlp coefficients < 2^15, orders/shifts/partition orders < 128
  int16_t mcoef[kMaxModels][kMaxLpc];
  int8_t mtype[kMaxModels], morder[kMaxModels], mshift[kMaxModels], mvalid[kMaxModels], mporder[kMaxModels];
  uint32_t mest[kMaxModels];
  unsigned long long mtot[kMaxModels];  // block total of 2|r| of each searched model (FRA-1 3.7c)
  unsigned long long ftot_s[5];  // FIXED orders' totals over the even 1024-sample quarters (FRA-1 3.7d)
  double mscore[MAXLAG > 8 ? kMaxModels : 1];  // FRA-1 3.7b window scores (levels 7-8)
  // 16-bit fast path: Rice parameter estimate of every partition at each searched model's best
  // partition order (written by porder_search, read by the winner's exact pass)
  uint8_t kbest[kMaxModels][kMaxPart];
  uint32_t ired[4][3];
  uint32_t scan[4];
  int32_t winner, ftype, fmethod;
  uint32_t fbits;
};

// ---- fast-path residual sums over the thread's 16 samples (one finest partition per thread);
// ---- samples jj < skip (warm-up: thread 0 only) are masked
template <bool B32>
__device__ __forceinline__ void acc_zz(int64_t r, bool on, uint64_t& acc, bool& ovf) {
  if constexpr (B32) {
    ovf |= on && (r > INT32_MAX || r < INT32_MIN);
    acc += on ? abs2_64(r) : 0ull;
  } else {
    acc += on ? abs2_64(r) : 0u;
  }
}
// FIXED orders 0..4 at once: the order-k residual is the k-th finite difference of the samples,
// the same integers as the oracle's closed forms (s, s-s1, s-2s1+s2, ...)
template <bool B32>
__device__ __forceinline__ void fixed_sums_fast(const int32_t* x, int i0, uint64_t (&acc)[5], bool (&ovf)[5]) {
  using T = typename std::conditional<B32, int64_t, int32_t>::type;
  T d[kChunk + 4];  // d[j] = current difference at x index j + 8
#pragma unroll
  for (int j = 0; j < kChunk + 4; j++) d[j] = (T)x[8 + j];
#pragma unroll
  for (int k = 0; k <= 4; k++) {
    if (k > 0) {
#pragma unroll
      for (int j = kChunk + 3; j >= k; j--) d[j] = d[j] - d[j - 1];
    }
    const int skip = k > i0 ? k - i0 : 0;
    uint64_t s = 0;
    bool o = false;
#pragma unroll
    for (int jj = 0; jj < kChunk; jj++) acc_zz<B32>((int64_t)d[jj + 4], jj >= skip, s, o);
    acc[k] = s;
    ovf[k] = o;
  }
}
template <bool B32, int O>
__device__ __forceinline__ uint64_t lpc_sum_fast(const int32_t* x, const int32_t* q, int sh, int skip, bool& ovf) {
  uint64_t acc = 0;
#pragma unroll
  for (int jj = 0; jj < kChunk; jj++) acc_zz<B32>(gres<B32, O>(x, jj, q, sh), jj >= skip, acc, ovf);
  return acc;
}

// 32-bps path: the predictor evaluated exactly in double precision: |q| < 2^14 (precision <= 15) and
// |x| < 2^31, so every product and partial sum is an integer below 2^50 (exact in f64);
// floor(sum * 2^-sh) is the int64 arithmetic shift and x - pred is exact.  Sum of 2|r| over the
// thread's samples (warm-up positions jj < skip masked); ovf if a residual leaves int32 (model invalid,
// as the oracle's compute_residual).  Replaces ~3 integer instructions per 64-bit multiply-add.
template <int O>
__device__ __forceinline__ uint64_t lpc_abs2_f64(const double* xd, const double* qd, int sh, int skip, bool& ovf) {
  const double scale = ldexp(1.0, -sh);
  double acc = 0.0;  // exact: sum of 16 |r| < 2^35 whenever no residual overflowed
#pragma unroll
  for (int jj = 0; jj < kChunk; jj++) {
    const int b = 12 + jj;
    double sum = 0.0;
#pragma unroll
    for (int j = 0; j < O; j++) sum = fma(qd[j], xd[b - 1 - j], sum);
    const double r = xd[b] - floor(sum * scale);
    const bool on = jj >= skip;
    ovf |= on && (r > 2147483647.0 || r < -2147483648.0);
    acc += on ? fabs(r) : 0.0;
  }
  return ovf ? 0ull : 2ull * (uint64_t)acc;
}

// 16-bit path LPC predictor with v_dot2c_i32_i16: samples fit int16 and |q| < 2^11, so the pairwise
// int16 products accumulate exactly in int32 (|sum| < 12 * 2^26); q pairs Q[p] = (q[2p], q[2p+1]),
// sample pairs A(m) = (x[m], x[m-1]) -> pred(b) = sum_p dot2(A(b - 1 - 2p), Q[p])
template <int NP>
__device__ __forceinline__ int32_t pred_dot2(const int32_t* x, int b, const fra_short2 (&Q)[NP]) {
  int32_t acc = 0;
#pragma unroll
  for (int p = 0; p < NP; p++) acc = __builtin_amdgcn_sdot2(pack_pair(x[b - 1 - 2 * p], x[b - 2 - 2 * p]), Q[p], acc, false);
  return acc;
}
template <int NP>
__device__ __forceinline__ void q_pairs(const int32_t* q, fra_short2 (&Q)[NP]) {
#pragma unroll
  for (int p = 0; p < NP; p++) Q[p] = pack_pair(q[2 * p], q[2 * p + 1]);
}
// 16-bit path straight from the LDS words: D[j] = samples (x[2j], x[2j+1]) as (lo, hi) int16, x[k] = sample
// i0 - 12 + k.  The dot2 operand pairs are taken in memory order (x[k], x[k+1]) -- a word itself for even k,
// one v_alignbit for odd k -- against coefficient pairs in reversed order (q[2p+1], q[2p]), so no sample
// is unpacked to 32 bits and re-packed
__device__ __forceinline__ void read_d14(const int16_t* smp, int t, uint32_t (&D)[14]) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(smp);  // kSmpStride even: chunks start dword-aligned
#pragma unroll
  for (int j = 0; j < 6; j++) D[j] = d[(t * kSmpStride + 4) / 2 + j];
#pragma unroll
  for (int j = 0; j < 8; j++) D[6 + j] = d[(t + 1) * kSmpStride / 2 + j];
}
// sum of |residual| of order O over the thread's 16 samples (warm-up positions jj < O of thread 0 masked),
// the residuals kept in r for the winner's encode
template <int O>
__device__ __forceinline__ uint32_t lpc_abs16_raw(const uint32_t (&D)[14], const int32_t* q, int sh, bool head,
                                                  int32_t (&r)[kChunk]) {
  constexpr int NP = (O + 1) / 2;
  fra_short2 Q[NP];
  q_pairs_rev<NP>(q, Q);
  uint32_t acc = 0;
#pragma unroll
  for (int jj = 0; jj < kChunk; jj++) {
    r[jj] = sample_at(D, 12 + jj) - (pred_raw<NP>(D, 12 + jj, Q) >> sh);
    const uint32_t rb = (uint32_t)r[jj] ^ kBias;
    acc = sad_acc(rb, (jj < O && head) ? rb : kBias, acc);
  }
  return acc;
}

// 16-bit path: sum of |LPC residual| over the thread's 16 samples (|r| < 2^27: fits 32 bits), warm-up
// positions jj < O masked for thread 0 only (compile-time bound); the caller doubles it (3.8)
template <int O>
__device__ __forceinline__ uint32_t lpc_abs16(const int32_t* x, const int32_t* q, int sh, bool head) {
  constexpr int NP = (O + 1) / 2;
  fra_short2 Q[NP];
  q_pairs<NP>(q, Q);
  uint32_t acc = 0;
#pragma unroll
  for (int jj = 0; jj < kChunk; jj++) {
    const int b = 12 + jj;
    const uint32_t xb = (uint32_t)x[b] ^ kBias;
    const uint32_t pb = (uint32_t)(pred_dot2<NP>(x, b, Q) >> sh) ^ kBias;
    acc = sad_acc(xb, (jj < O && head) ? xb : pb, acc);
  }
  return acc;
}

// wave-uniform sum of a 64-bit value over the wave (upper-lane DPP tree, lane 63's result broadcast)
__device__ __forceinline__ uint64_t wave_sum_u64_dpp(uint64_t v) {
  v = up_add64<0>(v); v = up_add64<1>(v); v = up_add64<2>(v);
  v = up_add64<3>(v); v = up_add64<4>(v); v = up_add64<5>(v);
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
}
// FRA-1 3.7 / 3.7d: the two FIXED orders with the smallest total of 2|r| over the even 1024-sample quarters of the
// block (ftot_s; first minimum first; invalid orders skipped) == oracle fg1/fg2.  Wave-uniform, every wave may run it.
__device__ __forceinline__ void fixed_guess2(const unsigned long long* ftot_s, const int8_t* mvalid, int lane,
                                             int& g1, int& g2) {
  uint64_t T[5];
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const uint64_t v = ftot_s[k];
    T[k] = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  }
  (void)lane;
  // branch-free selects on uniform values (a branchy form let the compiler merge g1/g2 into a
  // dynamically indexed private array, i.e. scratch memory)
  int h1 = -1, h2 = -1;
  uint64_t b1 = 0, b2 = 0;
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const bool valid = __builtin_amdgcn_readfirstlane(mvalid[k]) != 0;
    const bool lt1 = valid && (h1 < 0 || T[k] < b1);
    const bool lt2 = valid && !lt1 && (h2 < 0 || T[k] < b2);
    b2 = lt1 ? b1 : (lt2 ? T[k] : b2);
    h2 = lt1 ? h1 : (lt2 ? k : h2);
    b1 = lt1 ? T[k] : b1;
    h1 = lt1 ? k : h1;
  }
  g1 = __builtin_amdgcn_readfirstlane(h1);
  g2 = __builtin_amdgcn_readfirstlane(h2);
}

// FRA-1 3.7c (r06): a FIXED candidate whose block total of 2|r| is not below the smallest block total of the LPC
// models evaluated drops out of the winner choice (oracle analyze_subframe).  The totals are the root nodes of the
// models' partition searches (S.mtot; the FIXED searches may have run speculatively, during Levinson-Durbin).
// Wave-uniform: the mask of the FIXED models to drop.
__device__ __forceinline__ uint32_t fixed_gate(const unsigned long long* mtot, const int8_t* mvalid, int nmod) {
  unsigned long long lt = ~0ull;
  for (int m = 5; m < nmod; m++)
    if (__builtin_amdgcn_readfirstlane(mvalid[m]) && mtot[m] < lt) lt = mtot[m];
  uint32_t drop = 0;
  if (lt != ~0ull)
    for (int m = 0; m < 5; m++)
      if (__builtin_amdgcn_readfirstlane(mvalid[m]) && mtot[m] >= lt) drop |= 1u << m;
  return drop;
}

// Every partition order of one model's finest sums psum[0, 2^P) in one wave (porder_search_reg,
// fra_device.h: node sums by the upper-lane DPP tree and ds_bpermute, no LDS); kout[j], j < 2^bp, receives
// partition j's Rice parameter at the chosen order
__device__ __forceinline__ void porder_search(const unsigned long long* psum, int P, int pm, int n, int o, int lane,
                                              uint64_t& best_out, int& bp_out, uint8_t* kout = nullptr,
                                              unsigned long long* tot = nullptr) {
  const uint64_t Sv = lane < (1 << P) ? psum[lane] : 0ull;
  uint32_t kreg = 0;
  uint64_t total = 0;
  porder_search_reg(Sv, P, pm, n, o, lane, best_out, bp_out, kreg, &total);
  if (kout && (bp_out == 6 || lane < (1 << bp_out))) kout[lane] = (uint8_t)kreg;
  if (tot && lane == 0) *tot = total;  // the model's block total of 2|r| (FRA-1 3.7c)
}

// VERBATIM subframe written word by word straight to its slot (32-bps path, whose LDS bit buffer aliases
// the sample array): word j = the <= 3 samples (sbps >= 16 bits... any sbps >= 1) overlapping bits
// [32 j, 32 j + 32) of header (8 + w bits) + samples, MSB first -- the words lds_put would produce
template <typename SmpT>
__device__ __forceinline__ uint32_t verbatim_word(const SmpT* smp, int n, uint32_t hdr, int w, int sbps, uint32_t j) {
  const uint32_t smask = sbps >= 32 ? 0xFFFFFFFFu : ((1u << sbps) - 1u);
  const uint64_t hv = ((uint64_t)(2u | (w ? 1u : 0u)) << 56) | (w ? (1ull << (63 - (8 + w - 1))) : 0ull);
  const int64_t wb = 32 * (int64_t)j;
  uint32_t word = j == 0 ? (uint32_t)(hv >> 32) : (j == 1 ? (uint32_t)hv : 0u);
  const int s0 = wb > (int64_t)hdr ? (int)((wb - (int64_t)hdr) / sbps) : 0;
  for (int s = s0; s < n && (int64_t)hdr + (int64_t)s * sbps < wb + 32; s++) {
    const int64_t rel = (int64_t)hdr + (int64_t)s * sbps - wb;
    const int sft = 32 - (int)rel - sbps;
    const uint64_t v = (uint64_t)((uint32_t)smp[sidx(smp, s)] & smask);
    word |= sft >= 0 ? (uint32_t)(v << sft) : (uint32_t)(v >> -sft);
  }
  return word;
}
template <typename SmpT>
__device__ void verbatim_to_slot(uint32_t* slot, const SmpT* smp, int n, uint32_t hdr, int w, int sbps, uint32_t nw,
                                 int t) {
  for (uint32_t j = t; j < nw; j += kThreads) slot[j] = verbatim_word(smp, n, hdr, w, sbps, j);
}
constexpr int kWaves16 = 6;  // waves per SIMD of the 16-bit lag <= 8 instance (register budget 512 / waves)
#ifndef FRA_PREFETCH
// 16-bit full frames: one wave touches, during the Levinson-Durbin phase, the raw rows of the subframe
// FRA_PREFETCH workgroups ahead in dispatch order (a multiple of 8: the same XCD, blocks being dealt
// round-robin over the XCDs; 1024-1536 ~ the workgroups resident at 6 per CU x 256 CUs), one dword per
// 128-byte line, so that workgroup's load phase finds its rows in L2 / the Infinity Cache instead of HBM:
// C4 k_analyze -2.2 %, C3 -2.3 % at 1536 (r03 v11); 1024 another -0.5 % on the step, 768 / 2048 / 3072
// no better (r03 v11, v19).  The 32-bit path does not take it (C5 +1.3 %: 16 KiB of float rows per
// workgroup, r03 v12).  A hint only: nothing depends on it but the speed.  0 = off.
#define FRA_PREFETCH 1024
#endif

// One subframe by one workgroup: frame g, grid row cy (the channel, or for the 32-bit instance of a mid-side
// stream the virtual channel cy + 2); rot rotates the wave roles.  List mode (beside k_analyze_w, the 16-bit lag-8
// instance only): workgroup i takes entry i of the partial-subframe list (frame * 8 + channel), and the L2
// prefetch -- which guesses later workgroups by dispatch order -- is off.  The body is the kernel itself: as a
// device function taking the kernel arguments by reference it compiled to 125 instead of 101 VGPRs (32-bps
// instance) and twice the SGPR spills.
template <bool B32, int MAXLAG>
__global__ void __launch_bounds__(kThreads, B32 ? 5 : (MAXLAG > 8 ? 4 : kWaves16)) k_analyze(JobArgs a, int src) {
  int g_ = a.frame_base + (int)blockIdx.x, c_ = (int)blockIdx.y;
  if (a.part && ((!B32 && MAXLAG == 8) || (B32 && MAXLAG == 12))) {
    const int e = __builtin_amdgcn_readfirstlane(a.part[blockIdx.x]);
    g_ = e >> 3;
    c_ = e & 7;
  }
  const int g = g_, cy = c_, rot = (int)((blockIdx.x + blockIdx.y) & 3);
  const bool pf_allowed = B32 || MAXLAG != 8 || a.part == nullptr;

  __shared__ AnalyzeSmem<B32, MAXLAG> S;
  constexpr int MAXO = MAXLAG > 4 ? MAXLAG : 4;  // predictor taps of the generic residual body
  // wave index (and the wave role below) in SGPRs: a VGPR copy of them was spilled to scratch in the
  // 7-wave 16-bit instance
  const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
  // role of this wave (Levinson-Durbin, model searches, descriptor writes): rotated per workgroup so the
  // single-wave phases do not always land on the same SIMD; data layout (sample ranges, per-wave partials,
  // the encoder's scan) keeps the physical wave index wv
  const int rw = (wv + rot) & 3;
  // the frame's analysis descriptor first: the load phase takes its addresses, block size and stream from it,
  // so the raw loads wait for one scalar load instead of FrameDev -> StreamDev
  const WaveDev wd = a.wave[g];
  // mid-side streams (FRA-1 3.1b): virtual channels 0 L, 1 R, 2 M, 3 S; L and R are analysed by the
  // 16-bit instance, M and S (bps + 1 bits) by the 32-bit one, whose grid rows 0-1 are channels 2-3
  const int c = cy + ((B32 && wd.ms) ? 2 : 0);
  FRA_STAMP(0)
  if (c >= (wd.ms ? (B32 ? 4 : 2) : wd.channels)) return;
  const int n = wd.n;
  const int bps = wd.bps + ((wd.ms && c == 3) ? 1 : 0);
  const int msmode = (wd.ms && c >= 2) ? c - 1 : 0;
  const LevelCfg cfg = level_cfg(a.level);
  SfDesc* d = &a.sf[(size_t)g * a.cmax + c];
#ifdef FRA_DIAG_STOP
  // diagnostic phase-timing build only: a valid VERBATIM descriptor so k_pack stays in bounds
  if (t == 0) {
    d->type = 1; d->order = 0; d->wasted = 0; d->sbps = (uint8_t)bps; d->cval = 0; d->porder = 0;
    d->method = 0; d->precision = 0; d->shift = 0; d->bits = 8u + (uint32_t)n * (uint32_t)bps;
  }
#define FRA_STOP(k) if (FRA_DIAG_STOP == (k)) return;
#else
#define FRA_STOP(k)
#endif

  // ---- 1. load + normalise
  uint32_t pf = 0u;  // prefetch words (FRA_PREFETCH), consumed at the end of the fast path
  bool pf_ok = false;
  if (t < smp_stride<typename AnalyzeSmem<B32, MAXLAG>::SmpT>()) S.smp[t] = 0;  // zero chunk (samples before the block start)
  uint32_t orv = 0;
  int32_t vmin = INT32_MAX, vmax = INT32_MIN;
  {
    const NormParams np = norm_params(wd.norm, a.norm[wd.stream]);
    const int32_t* lut = (a.lut && np.mode) ? a.lut + (int64_t)wd.stream * a.lut_stride : nullptr;
    FRA_LOAD_STAMP(11, (int)np.mn + (int)wd.width + wd.n)
    bool done = false;
    if constexpr (!B32) {
      if (lut && a.vec8 && a.off32 && n == kMaxBlock) {
        done = load_lut_full(src, a.raster, wd, c, lut, S.smp, orv, vmin, vmax);
        pf_ok = done && pf_allowed;  // (the prefetch target is found by dispatch order)
      }
    }
    if (!done) load_channel(src, a.vec8 != 0, a.raster, wd, a.streams + wd.stream, a.frames + g, c, np, lut, S.smp, orv, vmin, vmax, msmode);
  }
  // residual partition sums are accumulated from phase 3 on (FIXED sums overlap wave 0's LPC work)
  for (int i = t; i < kMaxModels * kMaxPart; i += kThreads) (&S.u.psum[0][0])[i] = 0ull;
  if (t < 5) S.ftot_s[t] = 0ull;
  orv = wave_or32(orv);
  const uint32_t kmin = wave_min32((uint32_t)vmin ^ 0x80000000u);   // order-preserving keys
  const uint32_t kmax = ~wave_min32(~((uint32_t)vmax ^ 0x80000000u));
  if (lane == 0) { S.ired[wv][0] = orv; S.ired[wv][1] = kmin; S.ired[wv][2] = kmax; }
  FRA_LOAD_STAMP(14, (int)kmax)
  __syncthreads();
  orv = S.ired[0][0] | S.ired[1][0] | S.ired[2][0] | S.ired[3][0];
  vmin = (int32_t)(min(min(S.ired[0][1], S.ired[1][1]), min(S.ired[2][1], S.ired[3][1])) ^ 0x80000000u);
  vmax = (int32_t)(max(max(S.ired[0][2], S.ired[1][2]), max(S.ired[2][2], S.ired[3][2])) ^ 0x80000000u);
  FRA_STAMP(1)

  FRA_STOP(1)
  // ---- 2. CONSTANT / wasted bits (3.2, 3.3)
  if (vmin == vmax) {
#ifdef FRA_DIAG_STOP
    return;
#endif
    if (t == 0) {
      d->type = 0; d->order = 0; d->wasted = 0; d->sbps = (uint8_t)bps; d->cval = vmin;
      d->bits = 8u + (uint32_t)bps; d->porder = 0; d->method = 0; d->precision = 0; d->shift = 0;
      // blob: 8 header bits (type 0, no wasted bits) + the value in bps bits, MSB first
      uint32_t* slot = a.tmp + ((size_t)g * a.cmax + c) * a.tmp_stride;
      const uint64_t v = (uint64_t)(uint32_t)vmin & (bps >= 32 ? 0xFFFFFFFFull : ((1ull << bps) - 1));
      const uint64_t blob = v << (64 - 8 - bps);  // 8 zero header bits first
      slot[0] = (uint32_t)(blob >> 32);
      slot[1] = (uint32_t)blob;
    }
    return;
  }
  {
  const int w = __builtin_ctz(orv);
  const int sbps = bps - w;
  if (w) {
    for (int i = t; i < n; i += kThreads) S.smp[sidx(S.smp, i)] = S.smp[sidx(S.smp, i)] >> w;
    __syncthreads();
  }
  const uint32_t hdr = 8u + (uint32_t)(w ? w : 0);
  const uint32_t verb = hdr + (uint32_t)n * (uint32_t)sbps;
  const int i0 = t * kChunk;

  // ---- model table: FIXED 0..4 as integer predictors with shift 0
  const int fmax = n - 1 < 4 ? n - 1 : 4;
  if (t < kMaxModels) {
    S.mvalid[t] = (t < 5 && t <= fmax) ? 1 : 0;
    S.mtype[t] = t < 5 ? 2 : 3;
    S.morder[t] = t < 5 ? t : 0;
    S.mshift[t] = 0;
    // [1] [2,-1] [3,-3,1] [4,-6,4,-1]
    const int32_t f1[4] = {1, 0, 0, 0}, f2[4] = {2, -1, 0, 0}, f3[4] = {3, -3, 1, 0}, f4[4] = {4, -6, 4, -1};
#pragma unroll
    for (int j = 0; j < kMaxLpc; j++) {
      int32_t v = 0;
      if (j < 4) v = t == 1 ? f1[j] : t == 2 ? f2[j] : t == 3 ? f3[j] : t == 4 ? f4[j] : 0;
      S.mcoef[t][j] = v;
    }
  }

  // ---- 3a. partition geometry; FIXED residual sums of the fast 16-bit path (3.8), before the LPC
  // analysis: their partition search then runs on waves 1-3 while wave 0 does Levinson-Durbin
  const int P = max_porder(n, 0, cfg.max_porder);
  const int psz = n >> P;
  // x[j] = sample i0 - 12 + j: the last 12 of the previous chunk (the zero chunk for thread 0) and
  // this thread's 16 (samples past n are never counted: their sums/codes are masked by i0 < n / i < n)
  int32_t x[12 + kChunk];
  const bool fastframe = (psz % kChunk) == 0;  // uniform: each thread's 16 samples in one partition
  // FIXED sums by 32-bit finite differences (v_sad_u32): every 16-bit block, and 32-bps blocks whose
  // samples stay within +-2^23 (normalize_to_audio's 24-bit range): |4th difference| < 2^27, so 16 of
  // them fit 32 bits and no residual leaves int32 -- the same integers as the 64-bit sums
  const bool fixfast = fastframe && (!B32 || (vmin > -(1 << 23) && vmax < (1 << 23)));
  const bool head = i0 == 0;                    // this thread holds the warm-up samples (order <= 12 < 16)
  const int pidx0 = i0 < n ? i0 / psz : 0;
  const int nmod = 5 + (MAXLAG > 0 ? a.nwin : 0);
  if (fixfast) {
    read_x28(S.smp, t, x);
    // FIXED 0..4 by finite differences, in place: after step k, x[j] for j >= 8 + k holds the
    // k-th difference; |4th difference| < 2^20, so 16 zig-zags fit 32 bits.  Same integers as the
    // oracle's closed forms; every fixed model is valid here (n >= 16).
    // order k residual at j = the (k-1)-th difference x[j] - x[j-1]; |.| by v_sad_u32 on biased values
    // (x holds the (k-1)-th difference for j >= 7 + k); warm-up samples 0..k-1 belong to thread 0
    // (i0 == 0): those k positions compare a value with itself
    // (r05: kept biased, each difference order by one v_xad_u32 -- xad_bias, as in k_analyze_w)
    uint32_t v[12 + kChunk];
#pragma unroll
    for (int j = 8; j < 12 + kChunk; j++) v[j] = (uint32_t)x[j] ^ kBias;
#pragma unroll
    for (int k = 0; k <= 4; k++) {
      if (k > 1) {
#pragma unroll
        for (int j = 12 + kChunk - 1; j >= 7 + k; j--) v[j] = xad_bias(v[j - 1], v[j]);
      }
      uint32_t s32 = 0;
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) {
        const uint32_t ab = v[12 + jj];
        const uint32_t bb = k == 0 ? kBias : ((jj < k && head) ? ab : v[11 + jj]);
        s32 = sad_acc(ab, bb, s32);
      }
      if (i0 < n && s32) atomicAdd(&S.u.psum[k][pidx0], 2ull * s32);
      // (3.7d) the even quarters' total: a whole wave's 16-sample chunks lie in one quarter (t >> 6 = the wave): one
      // wave sum and one LDS atomic per even wave (64 same-address lanes would serialise)
      if (!(wv & 1)) {
        const uint64_t ws = wave_sum_u64_dpp(i0 < n ? 2ull * s32 : 0ull);
        if (lane == 0 && ws) atomicAdd(&S.ftot_s[k], (unsigned long long)ws);
      }
    }
  }
  FRA_STOP(9)
  FRA_STAMP(2)
  const int lmax = cfg.max_lpc < n - 1 ? cfg.max_lpc : n - 1;
  // FIXED models searched during window 0's Levinson-Durbin (psum complete at its barrier)
  const bool early = fixfast && MAXLAG > 0 && cfg.nsub > 0 && lmax > 0;

  // partial windows are zero outside their segment (host-computed extent [lo, hi)): a wave whose
  // samples + lookahead [1024 wv, 1024 wv + 1024 + MAXLAG) miss it would only sum exact products of
  // zeros, i.e. every chunk partial is +0.0 -- it skips the window and stores those zeros directly
  auto wave_active = [&](const int wi) -> bool {
    const int32_t* r = a.wrange + 2 * ((size_t)wd.win * a.nwin + wi);
    const int lo = __builtin_amdgcn_readfirstlane(r[0]), hi = __builtin_amdgcn_readfirstlane(r[1]);
    const int w0 = wv * 64 * kChunk;
    return lo < w0 + 64 * kChunk + MAXLAG && hi > w0;
  };
  // ---- 3. LPC analysis per apodization window (3.4-3.7)
  const int prec = qlp_precision(bps, n);
  if constexpr (MAXLAG > 0) {
    if (cfg.nsub > 0 && lmax > 0) {
      // 3.1 autocorrelation of every window: windowed samples -> chunk partials -> wave
      // reduce-scatter -> red[wi][wave][lag].  Window 0 is peeled so its prefetched coefficients die
      // at their first use.
      // FRA-1 3.5b: the 16-bit instance's subframes (streams of <= 16 bps) sum integers; the 32-bit instance --
      // 32-bps streams and the mid / side virtual channels of 16-bps stereo -- keeps 3.4's float chunk sums
      constexpr bool irule = !B32;
      auto window_acf = [&](const int wi, const bool act) {
        if (!act) {
          if (lane <= MAXLAG) S.red()[wi][wv][lane] = 0.0;  // = the all-zero partials (+0.0 exactly)
          return;
        }
        // coefficients loaded here, not prefetched before the FIXED sums: a prefetch kept 16 + MAXLAG
        // registers live through them and pushed the 7-wave instance into scratch.  (No plateau skip of the
        // exact-1.0 coefficients here, unlike k_analyze_w: its SGPR pressure cost more than the loads it saved,
        // C5 117.0 -> 115.2 ms without it, profiles/r04_ab_plateau_k_analyze_c5.txt)
        float wcoef[kChunk + MAXLAG];
        load_window<MAXLAG>(a.win + ((size_t)wd.win * a.nwin + wi) * a.blocksize, i0, n, wcoef);
        float wf[kChunk + MAXLAG];
        {
          int32_t y[kChunk + 8];
          read_y24(S.smp, t, y);
          // no bounds select: load_window left the coefficients of samples at or past n at 0.0f, and a
          // finite sample times +-0.0f adds +-0.0 to a chunk partial, which leaves the float sum bit-identical
          // (x + -0.0 == x, +0.0 + -0.0 == +0.0) -- the oracle's skipped terms
#pragma unroll
          for (int j = 0; j < kChunk + MAXLAG; j++) {
            const int i = i0 + j;
            const int32_t v = j < kChunk + 8 ? y[j] : S.smp[sidx(S.smp, min(i, kMaxBlock - 1))];
            wf[j] = (float)v * wcoef[j];
          }
        }

        double acc[MAXLAG + 1];
        if constexpr (irule) {
          // FRA-1 3.5b (the 16-bit instance): the windowed samples rounded to integers (|v| <= 2^15) and their
          // products summed as doubles -- exact (chunk partials < 2^35, totals < 2^43), so the reduction order
          // below does not matter; samples at or past n have 0.0f coefficients: v = 0
          double dv[kChunk + MAXLAG];
#pragma unroll
          for (int j = 0; j < kChunk + MAXLAG; j++) dv[j] = (double)__builtin_rintf(wf[j]);
#pragma unroll
          for (int l = 0; l <= MAXLAG; l++) {
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < kChunk; j++) s = fma(dv[j], dv[j + l], s);
            acc[l] = s;
          }
          autocorr_reduce_wave<MAXLAG + 1>(acc, S.red()[wi][wv], lane);
          return;
        }
        // chunk partials (FRA-1): per lag, the even and the odd samples of the chunk are summed
        // separately in float (fused multiply-add, ascending), then ae + ao in float, widened to double
        // -- one v_pk_fma_f32 per (sample pair, lag).  Samples at or past n are 0.0f, whose products
        // leave a float sum unchanged, so no tail masking is needed (= the oracle's skipped terms).
        f32x2 pacc[MAXLAG + 1];
#pragma unroll
        for (int l = 0; l <= MAXLAG; l++) pacc[l] = f32x2{0.0f, 0.0f};
#pragma unroll
        for (int pp = 0; pp < kChunk / 2; pp++) {
          const f32x2 a2 = {wf[2 * pp], wf[2 * pp + 1]};
#pragma unroll
          for (int l = 0; l <= MAXLAG; l++) {
            const f32x2 b2 = {wf[2 * pp + l], wf[2 * pp + l + 1]};
            pacc[l] = __builtin_elementwise_fma(a2, b2, pacc[l]);
          }
        }
#pragma unroll
        for (int l = 0; l <= MAXLAG; l++) acc[l] = (double)(pacc[l].x + pacc[l].y);
        autocorr_reduce_wave<MAXLAG + 1>(acc, S.red()[wi][wv], lane);
      };
      for (int wi = 0; wi < a.nwin; wi++) window_acf(wi, wave_active(wi));
      __syncthreads();
      FRA_STAMP(3)
      FRA_STOP(8)
      // Levinson-Durbin, order choice and quantisation of 4 windows per wave at once: window wi on wave
      // wi / 4, lanes 16 (wi % 4) .. +15 (the same op sequence per lane: one window's instruction cost for
      // four) -> expected bits of order o on lane 16 (wi % 4) + o -> first minimum per lane group -> qlp
      // quantisation per group.  Levels 3-6 (<= 3 windows) use wave 0, levels 7-8 (<= 6) waves 0-1; the
      // two FIXED candidates are searched meanwhile on the next two waves (psum is complete since the
      // autocorrelation barrier)
      const int nldw = (a.nwin + 3) >> 2;
      if constexpr (!B32) {  // (levels 3-6: wave 3 idles during this phase)
        if (FRA_PREFETCH > 0 && pf_ok && rw == 3)
          pf = (src == ST_U16 || src == ST_I16) ? prefetch_rows<uint16_t, FRA_PREFETCH>(a, lane)
                                                : prefetch_rows<uint8_t, FRA_PREFETCH>(a, lane);
      }
      if (early && (rw == nldw || rw == nldw + 1)) {
        int g1, g2;
        fixed_guess2(S.ftot_s, S.mvalid, lane, g1, g2);
        if (rw == nldw && lane < 5 && lane != g1 && lane != g2) S.mvalid[lane] = 0;
        const int m = rw == nldw ? g1 : g2;
        if (m >= 0) {
          const int pm = max_porder(n, m, cfg.max_porder);
          uint64_t best = 0;
          int bp = pm;
          porder_search(S.u.psum[m], P, pm, n, m, lane, best, bp, S.kbest[m], &S.mtot[m]);
          if (lane == 0) {
            S.mest[m] = (uint32_t)(hdr + (uint64_t)m * sbps + best);
            S.mporder[m] = bp;
          }
        }
        if (rw == nldw) { FRA_ROLE_STAMP(16) } else { FRA_ROLE_STAMP(17) }
      }
      if (rw < nldw) {
        const int gw = lane >> 4, lo = lane & 15;
        const int wi = 4 * rw + gw;
        const bool gon = wi < a.nwin;
        const int ws = gon ? wi : 0;
        double ac[MAXLAG + 1];
#pragma unroll
        for (int l = 0; l <= MAXLAG; l++)
          ac[l] = l <= lmax ? (S.red()[ws][0][l] + S.red()[ws][1][l]) + (S.red()[ws][2][l] + S.red()[ws][3][l]) : 0.0;
        int nord = 0;
        double errv[MAXLAG];
        if (gon && ac[0] != 0.0) nord = levinson_wave<MAXLAG>(ac, lmax, S.lp()[ws], errv, lo == 0);
        double e = errv[0];
#pragma unroll
        for (int j = 1; j < MAXLAG; j++)
          if (lo == j + 1) e = errv[j];
        // first minimum over orders 1..nord: bits >= 0 and finite, so its IEEE pattern orders as an
        // unsigned integer; DPP min inside each 16-lane row (lane 15 of the row), lowest lane among
        // the equal ones
        const bool on = nord > 0 && lo >= 1 && lo <= nord;
        const uint64_t key = on ? (uint64_t)__double_as_longlong(order_bits(e, n, lo, prec + sbps)) : ~0ull;
        uint64_t rk = min(key, dpp64_old<DPP_SHR1, 0xF>(key, ~0ull));
        rk = min(rk, dpp64_old<DPP_SHR2, 0xF>(rk, ~0ull));
        rk = min(rk, dpp64_old<DPP_SHR4, 0xF>(rk, ~0ull));
        rk = min(rk, dpp64_old<DPP_SHR8, 0xF>(rk, ~0ull));
        const uint64_t kmin = __shfl(rk, (lane & 48) | 15, 64);
        const uint64_t bal = __ballot(on && key == kmin);
        const uint32_t rowbits = (uint32_t)(bal >> (16 * gw)) & 0xFFFFu;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // group leaders' lp rows -> all lanes
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        bool ok = false;
        int o = 0, sh = 0;
        int32_t q[MAXLAG];
        if (nord > 0) {
          o = (int)__builtin_ctz(rowbits);
          double lpo[MAXLAG];
#pragma unroll
          for (int j = 0; j < MAXLAG; j++) lpo[j] = j < o ? -S.lp()[ws][lp_row(o - 1) + j] : 0.0;  // lp = -lpc
          ok = quantize<MAXLAG>(lpo, o, prec, q, sh);
        }
        if (gon && lo == 0) {
          const int m = 5 + wi;
          S.mvalid[m] = ok ? 1 : 0;
          S.mtype[m] = 3; S.morder[m] = o; S.mshift[m] = sh;
#pragma unroll
          for (int j = 0; j < MAXLAG; j++) S.mcoef[m][j] = ok ? q[j] : 0;
          if constexpr (MAXLAG > 8) {  // FRA-1 3.7b: the window's score from its chosen order's LD error
            double eo = errv[0];
#pragma unroll
            for (int j = 1; j < MAXLAG; j++) eo = o == j + 1 ? errv[j] : eo;
            S.mscore[m] = ok ? window_score(eo, ac[0], n, o, prec + sbps) : 0.0;
          }
        }
        FRA_ROLE_STAMP(15)
      }
    }
  }

  FRA_STOP(2)
  // ---- 4. residual partition sums at the finest level P for every valid model (3.8)
  uint32_t D[B32 ? 1 : 14];  // 16-bit fast frames: the LDS words of the sample window (read_d14)
  int32_t rkeep[B32 ? 1 : kChunk];  // 16-bit fast frames: residuals of the last LPC model summed (model keep_m)
  int keep_m = -1;
  if constexpr (B32) read_x28(S.smp, t, x);  // (the fast 16-bit path's FIXED sums consumed x)
  else if (fastframe) read_d14(S.smp, t, D);
  else read_x28(S.smp, t, x);
  __syncthreads();  // wave 0's LPC models (mcoef/mshift/mvalid) are visible from here on
  if constexpr (MAXLAG > 8) {
    // FRA-1 3.7b (levels 7-8, r06): only cfg.lpc_keep usable LPC models -- the smallest window scores, the lower
    // window on a tie -- get residual sums and a partition search (oracle analyze_subframe); the others are
    // invalidated here, before any wave reads the table (published by the barrier below)
    if (t == 0 && cfg.lpc_keep > 0) {
      uint32_t keep = 0;
      for (int r = 0; r < cfg.lpc_keep; r++) {
        int bm = -1;
        for (int m = 5; m < nmod; m++)
          if (S.mvalid[m] && !((keep >> m) & 1u) && (bm < 0 || S.mscore[m] < S.mscore[bm])) bm = m;
        if (bm < 0) break;
        keep |= 1u << bm;
      }
      for (int m = 5; m < nmod; m++)
        if (!((keep >> m) & 1u)) S.mvalid[m] = 0;
    }
    if constexpr (!B32) __syncthreads();
  }
  if constexpr (B32) {  // the LPC models' sums held the autocorrelation / LD rows: zero them again
    for (int i = t; i < (kMaxModels - 5) * kMaxPart; i += kThreads) (&S.u.psum[5][0])[i] = 0ull;
    __syncthreads();
  }
  FRA_STAMP(4)
  double xd[B32 ? 12 + kChunk : 1];  // 32-bps fast path: x as exact doubles
  if (fastframe) {
    if constexpr (B32) {
      // 32-bps: FIXED k as the 4-tap predictor [1] [2,-1] [3,-3,1] [4,-6,4,-1], exact in f64
#pragma unroll
      for (int j = 0; j < 12 + kChunk; j++) xd[j] = (double)x[j];
#pragma unroll
      for (int m = 0; m < 5; m++) {
        if (fixfast) break;  // already summed by finite differences (phase 3a)
        constexpr double kF[5][4] = {{0, 0, 0, 0}, {1, 0, 0, 0}, {2, -1, 0, 0}, {3, -3, 1, 0}, {4, -6, 4, -1}};
        const int skip = m > i0 ? m - i0 : 0;
        bool ovf = false;
        const uint64_t acc = lpc_abs2_f64<4>(xd, kF[m], 0, skip, ovf);
        if (i0 < n && acc) atomicAdd(&S.u.psum[m][pidx0], (unsigned long long)acc);
        if (!(wv & 1)) {  // (3.7d, as in the fast FIXED sums above)
          const uint64_t ws = wave_sum_u64_dpp(i0 < n ? acc : 0ull);
          if (lane == 0 && ws) atomicAdd(&S.ftot_s[m], (unsigned long long)ws);
        }
        if (__any(i0 < n && ovf) && lane == 0) S.mvalid[m] = 0;
      }
    }
    // LPC orders: exact-order tap bodies
    for (int m = 5; m < nmod; m++) {
      if (!S.mvalid[m]) continue;  // wave-uniform (LDS)
      const int o = S.morder[m];
      const int sh = __builtin_amdgcn_readfirstlane(S.mshift[m]);
      int32_t q[MAXO];
#pragma unroll
      for (int j = 0; j < MAXO; j++) q[j] = __builtin_amdgcn_readfirstlane(S.mcoef[m][j]);
      double qd[MAXO];  // (32-bps path)
#pragma unroll
      for (int j = 0; j < MAXO; j++) qd[j] = (double)q[j];
      const int skip = o > i0 ? o - i0 : 0;
      bool ovf = false;
      uint64_t acc = 0;
      switch (o) {
#define FRA_CASE(O_) \
  case O_:           \
    if constexpr (O_ <= MAXO) { \
      if constexpr (B32) acc = lpc_abs2_f64<O_>(xd, qd, sh, skip, ovf); \
      else acc = 2ull * lpc_abs16_raw<O_>(D, q, sh, head, rkeep); \
    } \
    break;
        FRA_CASE(1) FRA_CASE(2) FRA_CASE(3) FRA_CASE(4) FRA_CASE(5) FRA_CASE(6)
        FRA_CASE(7) FRA_CASE(8) FRA_CASE(9) FRA_CASE(10) FRA_CASE(11) FRA_CASE(12)
#undef FRA_CASE
      }
      if (i0 < n && acc) atomicAdd(&S.u.psum[m][pidx0], (unsigned long long)acc);
      if constexpr (B32) {
        if (__any(i0 < n && ovf) && lane == 0) S.mvalid[m] = 0;  // benign race: every writer stores 0
      } else {
        keep_m = m;
      }
    }
  } else {
    for (int m = 0; m < nmod; m++) {
      if (!S.mvalid[m]) continue;  // wave-uniform (LDS)
      const int o = S.morder[m];
      const int sh = __builtin_amdgcn_readfirstlane(S.mshift[m]);
      int32_t q[MAXO];
#pragma unroll
      for (int j = 0; j < MAXO; j++) q[j] = __builtin_amdgcn_readfirstlane(S.mcoef[m][j]);
      bool ovf = false;
      uint64_t acc = 0, accs = 0;  // (accs: a FIXED order's even-quarter total, 3.7d)
      if (i0 < n) {
        int pidx = pidx0, pend = (pidx + 1) * psz;
        const int iend = min(i0 + kChunk, n);
        for (int i = max(i0, o); i < iend; i++) {
          if (i >= pend) {
            if (acc) atomicAdd(&S.u.psum[m][pidx], (unsigned long long)acc);
            acc = 0;
            pidx = i / psz;
            pend = (pidx + 1) * psz;
          }
          const int64_t r = gres_lds<B32, MAXO>(S.smp, i, q, sh);
          if constexpr (B32) ovf |= (r > INT32_MAX || r < INT32_MIN);
          acc += abs2_64(r);
          if (m < 5 && !((i >> 10) & 1)) accs += abs2_64(r);
        }
        if (acc) atomicAdd(&S.u.psum[m][pidx], (unsigned long long)acc);
        if (accs) atomicAdd(&S.ftot_s[m], (unsigned long long)accs);
      }
      if constexpr (B32) {
        if (__any(ovf) && lane == 0) S.mvalid[m] = 0;  // benign race: every writer stores 0
      }
    }
  }
  __syncthreads();
  FRA_STAMP(5)

  FRA_STOP(3)
  // ---- 5. every partition order of a model in one pass (one wave per model)
  int fg1 = -1, fg2 = -1;
  if (!early) {  // FIXED candidates (3.7): excluded orders are invalidated before the winner barrier
    fixed_guess2(S.ftot_s, S.mvalid, lane, fg1, fg2);
    if (rw == 0 && lane < 5 && lane != fg1 && lane != fg2) S.mvalid[lane] = 0;
  }
  // the models left to search, dealt to the waves in order (r06: compacted, so that 2 LPC models of 6 windows
  // land on two waves, not both on the wave of their index mod 4)
  for (int m = early ? 5 : 0, slot = 0; m < nmod; m++) {
    if (!S.mvalid[m] || (m < 5 && m != fg1 && m != fg2)) continue;
    if ((slot++ & 3) != rw) continue;
    const int o = S.morder[m];
    const int pm = max_porder(n, o, cfg.max_porder);
    uint64_t best = 0;
    int bp = pm;
    porder_search(S.u.psum[m], P, pm, n, o, lane, best, bp, S.kbest[m], &S.mtot[m]);
    if (lane == 0) {
      S.mest[m] = (uint32_t)(hdr + (uint64_t)o * sbps + (S.mtype[m] == 3 ? 9 + (uint64_t)o * prec : 0) + best);
      S.mporder[m] = bp;
    }
    FRA_ROLE_STAMP(18)
  }
  {  // zero the winner's exact-pass sums (waves 0 and 1 share the 3 x kMaxPart words)
    unsigned long long* ez = &S.nu.e.esum2[0][0];
    const int e1 = min(kMaxPart * 3, (rw + 1) * 2 * kMaxPart);
    for (int i = rw * 2 * kMaxPart + lane; i < e1; i += 64) ez[i] = 0ull;
  }
  __syncthreads();
  FRA_STAMP(6)
  FRA_STOP(5)
  {
    if (fastframe) {
      // ---- 6+7, fast frames: every wave derives the winner and the partition Rice parameters
      // itself (same integers in every wave: no wave-0 section + broadcast barrier), exact sums by LDS
      // atomics, the same refinement in every wave, then the encoder.  4 barriers instead of 7.
      const uint32_t drop = fixed_gate(S.mtot, S.mvalid, nmod);  // FRA-1 3.7c
      uint32_t key = ~0u;
      if (lane < nmod && S.mvalid[lane] && !((drop >> lane) & 1u)) key = (S.mest[lane] << 5) | (uint32_t)lane;
      const int m = (int)(wave_min32(key) & 31u);
      const int type = __builtin_amdgcn_readfirstlane(S.mtype[m]);
      const int o = __builtin_amdgcn_readfirstlane(S.morder[m]);
      const int sh = __builtin_amdgcn_readfirstlane(S.mshift[m]);
      const int ps = __builtin_amdgcn_readfirstlane(S.mporder[m]);
      // estimate k per partition of order ps (3.8): stored by the winner's porder_search
      const int pz = n >> ps;
      const bool live = i0 < n;
      const int pidx = live ? i0 / pz : 0;
      const int k0 = S.kbest[m][pidx];
      // zig-zag residuals of the winner (exact code values), warm-up samples 0
      uint32_t uu[kChunk];
      bool have = false;
      if constexpr (!B32) {
        if (m == keep_m) {  // the winner is the LPC model whose residuals are still in registers
#pragma unroll
          for (int jj = 0; jj < kChunk; jj++) uu[jj] = zz32(rkeep[jj]);
          have = true;
        } else if (type == 3) {
          int32_t q[MAXO];
#pragma unroll
          for (int j = 0; j < MAXO; j++) q[j] = __builtin_amdgcn_readfirstlane(S.mcoef[m][j]);
          fra_short2 Q[(MAXO + 1) / 2];
          q_pairs_rev<(MAXO + 1) / 2>(q, Q);
          read_d14(S.smp, t, D);
#pragma unroll
          for (int jj = 0; jj < kChunk; jj++)
            uu[jj] = zz32(sample_at(D, 12 + jj) - (pred_raw<(MAXO + 1) / 2>(D, 12 + jj, Q) >> sh));
          have = true;
        }
      }
      if (have) {
      } else if (type == 2 && (!B32 || fixfast)) {  // FIXED: finite differences in 32 bits (range checked)
        read_x28(S.smp, t, x);
#pragma unroll
        for (int k = 1; k <= 4; k++) {
          if (k <= o) {
#pragma unroll
            for (int j = 12 + kChunk - 1; j >= 8 + k; j--) x[j] = x[j] - x[j - 1];
          }
        }
#pragma unroll
        for (int jj = 0; jj < kChunk; jj++) uu[jj] = zz32(x[12 + jj]);
      } else {
        read_x28(S.smp, t, x);
        int32_t q[MAXO];
#pragma unroll
        for (int j = 0; j < MAXO; j++) q[j] = __builtin_amdgcn_readfirstlane(S.mcoef[m][j]);
        if constexpr (B32) {  // exact predictor in f64 (|products| < 2^45, sums < 2^50); valid: fits int32
          double qd[MAXO], xd2[12 + kChunk];
#pragma unroll
          for (int j = 0; j < MAXO; j++) qd[j] = (double)q[j];
#pragma unroll
          for (int j = 0; j < 12 + kChunk; j++) xd2[j] = (double)x[j];
          const double scale = ldexp(1.0, -sh);
#pragma unroll
          for (int jj = 0; jj < kChunk; jj++) {
            double sum = 0.0;
#pragma unroll
            for (int j = 0; j < MAXO; j++) sum = fma(qd[j], xd2[11 + jj - j], sum);
            uu[jj] = zz32((int32_t)(xd2[12 + jj] - floor(sum * scale)));
          }
        } else {
          fra_short2 Q[(MAXO + 1) / 2];
          q_pairs<(MAXO + 1) / 2>(q, Q);
#pragma unroll
          for (int jj = 0; jj < kChunk; jj++) uu[jj] = zz32(x[12 + jj] - (pred_dot2<(MAXO + 1) / 2>(x, 12 + jj, Q) >> sh));
        }
      }
      if (head) {
#pragma unroll
        for (int jj = 0; jj < 12; jj++)
          if (jj < o) uu[jj] = 0u;
      }
      if (t < o) S.warm[t] = S.smp[sidx(S.smp, t)];  // smp becomes the bit buffer after the next barrier
      // 16-bit: u < 2^28, so 16 of them fit 32 bits; 32-bps: 64-bit partial sums
      typename std::conditional<B32, uint64_t, uint32_t>::type fs0 = 0, fs1 = 0, fs2 = 0;
      {
        const int km = k0 > 0 ? k0 - 1 : 0;  // fs0 is only used when k0 >= 1
#pragma unroll
        for (int jj = 0; jj < kChunk; jj++) {
          fs0 += uu[jj] >> km;
          fs1 += uu[jj] >> k0;
          fs2 += uu[jj] >> (k0 + 1);
        }
      }
      const int tpp = pz >> 4;  // threads per partition (uniform)
      if ((tpp & (tpp - 1)) == 0) {
        // partitions cover aligned groups of tpp lanes: reduce each group's (<= 64 lanes) sums on the
        // upper-lane tree first, then one LDS atomic per partition and wave from the group's last lane
        // (same-address atomics of up to 64 lanes would serialise).  n is a multiple of pz, so a group
        // is entirely live or entirely past n.
        const int ls = min(6, 31 - __builtin_clz((uint32_t)tpp));
        uint64_t v0 = fs0, v1 = fs1, v2 = fs2;
        if (__all(fs0 <= (0xFFFFFFFFu >> ls))) {
          // 2^ls lanes of at most 2^(32-ls) - 1 (fs0 >= fs1 >= fs2): the group sums fit 32 bits
          uint32_t u0 = fs0, u1 = fs1, u2 = fs2;
#define FRA_UP(S_) \
          if (ls > S_) { u0 = up_add32<S_>(u0); u1 = up_add32<S_>(u1); u2 = up_add32<S_>(u2); }
          FRA_UP(0) FRA_UP(1) FRA_UP(2) FRA_UP(3) FRA_UP(4) FRA_UP(5)
#undef FRA_UP
          v0 = u0; v1 = u1; v2 = u2;
        } else {
#define FRA_UP(S_)                                                                     \
          if (ls > S_) { v0 = up_add64<S_>(v0); v1 = up_add64<S_>(v1); v2 = up_add64<S_>(v2); }
          FRA_UP(0) FRA_UP(1) FRA_UP(2) FRA_UP(3) FRA_UP(4) FRA_UP(5)
#undef FRA_UP
        }
        const int gm = (1 << ls) - 1;
        if (live && (lane & gm) == gm) {
          atomicAdd(&S.nu.e.esum2[pidx][0], (unsigned long long)v0);
          atomicAdd(&S.nu.e.esum2[pidx][1], (unsigned long long)v1);
          atomicAdd(&S.nu.e.esum2[pidx][2], (unsigned long long)v2);
        }
      } else if (live) {
        atomicAdd(&S.nu.e.esum2[pidx][0], (unsigned long long)fs0);
        atomicAdd(&S.nu.e.esum2[pidx][1], (unsigned long long)fs1);
        atomicAdd(&S.nu.e.esum2[pidx][2], (unsigned long long)fs2);
      }
      __syncthreads();
      FRA_STAMP(7)
      FRA_STOP(6)
      // exact Rice bits with k refined over k0-1..k0+1 (3.9), lane j = partition j, in every wave
      const int npp = 1 << ps;
      const int k0j = lane < npp ? (int)S.kbest[m][lane] : 0;
      uint64_t best = 0;
      int bk = 0;
      if (lane < npp) {
        const uint64_t cnt = (uint64_t)(pz - (lane == 0 ? o : 0));
        bool first = true;
        for (int kk = k0j - 1; kk <= k0j + 1; kk++) {
          if (kk < 0 || kk > 30) continue;
          const uint64_t e = cnt * (uint64_t)(kk + 1) + S.nu.e.esum2[lane][kk - k0j + 1];
          if (first || e < best) { best = e; bk = kk; first = false; }
        }
      }
      const bool big = __any(lane < npp && bk > 14);
      const uint64_t rtot = (uint64_t)wave_sum32(lane < npp ? (uint32_t)best : 0u) + (uint64_t)npp * (big ? 5 : 4) + 6;
      const uint64_t exact = hdr + (uint64_t)o * sbps + (type == 3 ? 9 + (uint64_t)o * prec : 0) + rtot;
      const bool verbatim = exact >= verb;
      const int kcur = __shfl(bk, pidx, 64);
      if (rw == 0) {
        if (lane < npp) d->k[lane] = (uint8_t)bk;
        if (lane < kMaxLpc) d->coef[lane] = type == 3 ? S.mcoef[m][lane] : 0;
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
      }
      // encode (RFC 9639 9.2) into the LDS bit buffer (over psum: every wave is past its psum reads)
      const uint32_t fbits = verbatim ? verb : (uint32_t)exact;
      const uint32_t nw = (fbits + 31) >> 5;
      if (verbatim) {  // straight from smp to the slot (the aliased bit buffer is not touched)
        verbatim_to_slot(a.tmp + ((size_t)g * a.cmax + c) * a.tmp_stride, S.smp, n, hdr, w, sbps, nw, t);
        asm volatile("" ::"v"(pf));  // (the prefetch loads stay; they returned long ago)
        return;
      }
      // the bit buffer aliases smp, dead since the barrier above (warm-up samples in S.warm)
      uint32_t* buf = reinterpret_cast<uint32_t*>(S.smp);
      for (uint32_t j = t; j <= nw; j += kThreads) buf[j] = 0u;
      const int pb = big ? 5 : 4;
      const int dk = kcur - k0;
      const bool pstart = live && i0 == pidx * pz;
      const uint32_t cnt = live ? (uint32_t)(kChunk - (head ? o : 0)) : 0u;
      const uint32_t tot = (live && !verbatim)
                               ? (dk < 0 ? fs0 : dk == 0 ? fs1 : fs2) + cnt * (uint32_t)(kcur + 1) + (pstart ? (uint32_t)pb : 0u)
                               : 0u;
      const uint32_t inc = wave_incl_scan32(tot);
      if (lane == 63) S.scan[wv] = inc;
      __syncthreads();
      FRA_STAMP(8)
      FRA_STOP(7)
      const uint32_t smask = sbps >= 32 ? 0xFFFFFFFFu : ((1u << sbps) - 1u);
      if (t == 0) {
        const int tcode = verbatim ? 1 : type == 2 ? 8 + o : 31 + o;
        lds_put(buf, 0, (uint32_t)(tcode << 1) | (w ? 1u : 0u), 8);
        if (w) lds_put(buf, 8 + (uint32_t)(w - 1), 1u, 1);
      }
      {
        if (t < o) lds_put(buf, hdr + (uint32_t)t * sbps, (uint32_t)S.warm[t] & smask, sbps);
        uint32_t pos = hdr + (uint32_t)o * sbps;
        if (type == 3) {
          if (t == 0) {
            lds_put(buf, pos, (uint32_t)(prec - 1), 4);
            lds_put(buf, pos + 4, (uint32_t)sh & 31u, 5);
          }
          if (t < o) lds_put(buf, pos + 9 + (uint32_t)t * prec, (uint32_t)S.mcoef[m][t] & ((1u << prec) - 1u), prec);
          pos += 9 + (uint32_t)o * prec;
        }
        if (t == 0) lds_put(buf, pos, ((uint32_t)(big ? 1 : 0) << 4) | (uint32_t)ps, 6);
        pos += 6;
        uint32_t p = pos + inc - tot;
        for (int ww = 0; ww < wv; ww++) p += S.scan[ww];
        if (pstart) { lds_put(buf, p, (uint32_t)kcur, pb); p += pb; }
        // Rice code (stop bit + kcur low bits) left-aligned: bit 31 = the stop bit
        // (u << (31 - k)) keeps u's low k bits under bit 31 and shifts the higher ones out; bit 31 (u's bit
        // k) is then forced to the stop bit: one v_lshl_or_b32, no mask
        const uint32_t sal = 31u - (uint32_t)kcur;
#pragma unroll
        for (int jj = 0; jj < kChunk; jj++) {
          if (live && !(jj < 12 && head && jj < o)) {
            const uint32_t P = p + (uu[jj] >> kcur);
            lds_put_al(buf, P, (uu[jj] << sal) | 0x80000000u);
            p = P + 1u + (uint32_t)kcur;
          }
        }
      }
      __syncthreads();
      FRA_STAMP(9)
      {
        uint32_t* slot = a.tmp + ((size_t)g * a.cmax + c) * a.tmp_stride;
        for (uint32_t j = t; j < nw; j += kThreads) slot[j] = buf[j];
        asm volatile("" ::"v"(pf));
        FRA_STAMP(10)
        return;
      }
    }
  }
  if (rw == 0) {  // winner = first minimal estimate: argmin over (estimate, model index)
    const uint32_t drop = fixed_gate(S.mtot, S.mvalid, nmod);  // FRA-1 3.7c
    uint32_t key = ~0u;
    if (lane < nmod && S.mvalid[lane] && !((drop >> lane) & 1u)) key = (S.mest[lane] << 5) | (uint32_t)lane;
    key = wave_min32(key);
    if (lane == 0) S.winner = (int)(key & 31u);
  }
  __syncthreads();

  FRA_STOP(4)
  // ---- 6. exact Rice bits for the winner (3.9)
  const int m = S.winner;
  const int type = S.mtype[m], o = S.morder[m], sh = S.mshift[m], ps = S.mporder[m];
  if (rw == 0) {
    uint64_t Sv = lane < (1 << P) ? S.u.psum[m][lane] : 0ull;
    const int smax = P - ps;
    if (smax > 0) Sv = up_add64<0>(Sv);
    if (smax > 1) Sv = up_add64<1>(Sv);
    if (smax > 2) Sv = up_add64<2>(Sv);
    if (smax > 3) Sv = up_add64<3>(Sv);
    if (smax > 4) Sv = up_add64<4>(Sv);
    if (smax > 5) Sv = up_add64<5>(Sv);
    if (lane < (1 << P) && ((lane + 1) & ((1 << smax) - 1)) == 0) {
      const int j = lane >> smax;
      const uint64_t cnt = (uint64_t)((n >> ps) - (j == 0 ? o : 0));
      int k;
      uint64_t bits;
      rice_pick(cnt, Sv, k, bits);
      S.nu.e.kpart[j] = k;
    }
  }
  __syncthreads();
  unsigned long long(*esum)[3] = reinterpret_cast<unsigned long long(*)[3]>(&S.u.psum[0][0]);
  for (int i = t; i < kMaxPart * 3; i += kThreads) (&esum[0][0])[i] = 0ull;
  // zig-zag residuals of the winner for this thread's 16 samples, computed ONCE: used by the exact
  // Rice pass here and by the encoder below.  Slow frames: 0 for warm-up samples and past the block
  // end; fast frames: warm-up samples 0, samples past the block end (threads with i0 >= n) unused.
  uint32_t uu[kChunk];
  uint32_t fs[3] = {0u, 0u, 0u};  // fast frames: this thread's sums of u >> (k0-1), u >> k0, u >> (k0+1)
  if (fastframe) {
    // reload the sample window from LDS (keeps the phase-4 window registers dead across the search)
read_x28(S.smp, t, x);
    if (!B32 && type == 2) {
      // FIXED winner: the o-th finite difference in place (wave-uniform o), as in phase 4
#pragma unroll
      for (int k = 1; k <= 4; k++) {
        if (k <= o) {
#pragma unroll
          for (int j = 12 + kChunk - 1; j >= 8 + k; j--) x[j] = x[j] - x[j - 1];
        }
      }
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) uu[jj] = zz32(x[12 + jj]);
    } else {
      int32_t q[MAXO];
#pragma unroll
      for (int j = 0; j < MAXO; j++) q[j] = __builtin_amdgcn_readfirstlane(S.mcoef[m][j]);
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++)
        if constexpr (B32) uu[jj] = (uint32_t)zz64(gres<B32, MAXO>(x, jj, q, sh));
        else {
          fra_short2 Q[(MAXO + 1) / 2];
          q_pairs<(MAXO + 1) / 2>(q, Q);
          uu[jj] = zz32(x[12 + jj] - (pred_dot2<(MAXO + 1) / 2>(x, 12 + jj, Q) >> sh));
        }
    }
    if (head) {
#pragma unroll
      for (int jj = 0; jj < 12; jj++)
        if (jj < o) uu[jj] = 0u;
    }
  } else {
    int32_t q[MAXO];
#pragma unroll
    for (int j = 0; j < MAXO; j++) q[j] = __builtin_amdgcn_readfirstlane(S.mcoef[m][j]);
#pragma unroll
    for (int jj = 0; jj < kChunk; jj++) {
      const int i = i0 + jj;
      const uint32_t uv = i < n ? (uint32_t)zz64(gres_lds<B32, MAXO>(S.smp, i, q, sh)) : 0u;
      uu[jj] = (i < n && i >= o) ? uv : 0u;
    }
  }
  if (t < o) S.warm[t] = S.smp[sidx(S.smp, t)];  // smp becomes the bit buffer after the decision
  __syncthreads();
  {
    const int pz = n >> ps;
    uint64_t e0 = 0, e1 = 0, e2 = 0;
    if (fastframe) {
      const int pidx = i0 < n ? i0 / pz : 0;
      const int k = S.nu.e.kpart[pidx];
      const int km = k > 0 ? k - 1 : 0;  // e0 is only used when k >= 1
      if constexpr (B32) {
#pragma unroll
        for (int jj = 0; jj < kChunk; jj++) {
          const uint32_t u = uu[jj];
          e0 += u >> km;
          e1 += u >> k;
          e2 += u >> (k + 1);
        }
      } else {  // u < 2^28 on the 16-bit path: 16 of them fit 32 bits
#pragma unroll
        for (int jj = 0; jj < kChunk; jj++) {
          const uint32_t u = uu[jj];
          fs[0] += u >> km;
          fs[1] += u >> k;
          fs[2] += u >> (k + 1);
        }
        e0 = fs[0]; e1 = fs[1]; e2 = fs[2];
      }
      if (i0 < n) {
        atomicAdd(&esum[pidx][0], (unsigned long long)e0);
        atomicAdd(&esum[pidx][1], (unsigned long long)e1);
        atomicAdd(&esum[pidx][2], (unsigned long long)e2);
      }
    } else if (i0 < n) {
      int pidx = i0 / pz, pend = (pidx + 1) * pz;
      int k = S.nu.e.kpart[pidx];
      const int iend = min(i0 + kChunk, n);
      for (int i = max(i0, o); i < iend; i++) {
        if (i >= pend) {
          atomicAdd(&esum[pidx][0], (unsigned long long)e0);
          atomicAdd(&esum[pidx][1], (unsigned long long)e1);
          atomicAdd(&esum[pidx][2], (unsigned long long)e2);
          e0 = e1 = e2 = 0;
          pidx = i / pz;
          pend = (pidx + 1) * pz;
          k = S.nu.e.kpart[pidx];
        }
        uint32_t u = 0;
#pragma unroll
        for (int jj = 0; jj < kChunk; jj++)
          if (i - i0 == jj) u = uu[jj];
        e0 += k > 0 ? (u >> (k - 1)) : 0u;
        e1 += u >> k;
        e2 += u >> (k + 1);
      }
      atomicAdd(&esum[pidx][0], (unsigned long long)e0);
      atomicAdd(&esum[pidx][1], (unsigned long long)e1);
      atomicAdd(&esum[pidx][2], (unsigned long long)e2);
    }
  }
  __syncthreads();
  if (rw == 0) {
    const int npp = 1 << ps;
    uint64_t best = 0;
    int bk = 0;
    if (lane < npp) {
      const uint64_t cnt = (uint64_t)((n >> ps) - (lane == 0 ? o : 0));
      const int k0 = S.nu.e.kpart[lane];
      bool first = true;
      for (int kk = k0 - 1; kk <= k0 + 1; kk++) {
        if (kk < 0 || kk > 30) continue;
        const uint64_t e = cnt * (uint64_t)(kk + 1) + esum[lane][kk - k0 + 1];
        if (first || e < best) { best = e; bk = kk; first = false; }
      }
    }
    const bool big = __any(lane < npp && bk > 14);
    const uint64_t tot = (uint64_t)wave_sum32(lane < npp ? (uint32_t)best : 0u) + (uint64_t)npp * (big ? 5 : 4) + 6;
    const uint64_t exact = hdr + (uint64_t)o * sbps + (type == 3 ? 9 + (uint64_t)o * prec : 0) + tot;
    const bool verbatim = exact >= verb;
    if (lane < npp) { d->k[lane] = (uint8_t)bk; S.nu.e.kfin[lane] = bk; }
    if (lane < kMaxLpc) d->coef[lane] = type == 3 ? S.mcoef[m][lane] : 0;
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
      S.ftype = verbatim ? 1 : type;
      S.fmethod = big ? 1 : 0;
      S.fbits = verbatim ? verb : (uint32_t)exact;
    }
  }
  __syncthreads();

  // ---- 7. encode the subframe (RFC 9639 9.2) into the LDS bit buffer and store it to its slot
  const int ftype = S.ftype;
  const uint32_t fbits = S.fbits;
  const uint32_t nw = (fbits + 31) >> 5;
  const uint32_t smask = sbps >= 32 ? 0xFFFFFFFFu : ((1u << sbps) - 1u);
  if (ftype == 1) {
    // VERBATIM (rare): straight from smp to the slot (the aliased bit buffer is not touched)
    verbatim_to_slot(a.tmp + ((size_t)g * a.cmax + c) * a.tmp_stride, S.smp, n, hdr, w, sbps, nw, t);
    return;
  }
  // every smp read (the winner's residuals, the warm-up copy) precedes the decision barrier
  uint32_t* buf = reinterpret_cast<uint32_t*>(S.smp);
  static_assert(sizeof(S.smp) >= sizeof(uint32_t) * (buf_words<B32>() + 1), "bit buffer inside smp");
  for (uint32_t j = t; j <= nw; j += kThreads) buf[j] = 0u;
  __syncthreads();
  if (t == 0) {
    const int tcode = ftype == 1 ? 1 : ftype == 2 ? 8 + o : 31 + o;
    lds_put(buf, 0, (uint32_t)(tcode << 1) | (w ? 1u : 0u), 8);
    if (w) lds_put(buf, 8 + (uint32_t)(w - 1), 1u, 1);
  }
  {
    const int pb = S.fmethod ? 5 : 4;
    for (int i = t; i < o; i += kThreads) lds_put(buf, hdr + (uint32_t)i * sbps, (uint32_t)S.warm[i] & smask, sbps);
    uint32_t pos = hdr + (uint32_t)o * sbps;
    if (ftype == 3) {
      if (t == 0) {
        lds_put(buf, pos, (uint32_t)(prec - 1), 4);
        lds_put(buf, pos + 4, (uint32_t)sh & 31u, 5);
      }
      if (t < o) lds_put(buf, pos + 9 + (uint32_t)t * prec, (uint32_t)S.mcoef[m][t] & ((1u << prec) - 1u), prec);
      pos += 9 + (uint32_t)o * prec;
    }
    if (t == 0) lds_put(buf, pos, ((uint32_t)S.fmethod << 4) | (uint32_t)ps, 6);
    pos += 6;
    const int pz = n >> ps;
    if (!B32 && fastframe) {
      // one partition per thread: Rice parameter kcur for all 16 codes, code bits from the exact-pass
      // sums (kcur is k0-1, k0 or k0+1), the partition parameter in front of the thread's first code
      const bool live = i0 < n;
      const int pidx = live ? i0 / pz : 0;
      const int kcur = S.nu.e.kfin[pidx];
      const int dk = kcur - S.nu.e.kpart[pidx];
      const bool pstart = live && i0 == pidx * pz;
      const uint32_t cnt = live ? (uint32_t)(kChunk - (head ? o : 0)) : 0u;
      const uint32_t tot = live ? (dk < 0 ? fs[0] : dk == 0 ? fs[1] : fs[2]) + cnt * (uint32_t)(kcur + 1) +
                                      (pstart ? (uint32_t)pb : 0u)
                                : 0u;
      const uint32_t inc = wave_incl_scan32(tot);
      if (lane == 63) S.scan[wv] = inc;
      __syncthreads();
      uint32_t p = pos + inc - tot;
      for (int ww = 0; ww < wv; ww++) p += S.scan[ww];
      if (pstart) { lds_put(buf, p, (uint32_t)kcur, pb); p += pb; }
      // Rice code (stop bit + kcur low bits) left-aligned: bit 31 = the stop bit
      const uint32_t sal = 31u - (uint32_t)kcur;
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) {
        if (live && !(jj < 12 && head && jj < o)) {
          const uint32_t P = p + (uu[jj] >> kcur);
          lds_put_al(buf, P, (uu[jj] << sal) | 0x80000000u);  // (see above: no mask needed)
          p = P + 1u + (uint32_t)kcur;
        }
      }
    } else {
    uint32_t kk[kChunk];  // Rice parameter | partition-start << 8, 0xFFFF = no code
    uint32_t tot = 0;
    int pidx = i0 < n ? i0 / pz : 0, pend = (pidx + 1) * pz;
    int kcur = S.nu.e.kfin[pidx];
#pragma unroll
    for (int jj = 0; jj < kChunk; jj++) {
      const int i = i0 + jj;
      kk[jj] = 0xFFFFu;
      if (i < n && i >= o) {
        if (i >= pend) { pidx++; pend += pz; kcur = S.nu.e.kfin[pidx]; }
        const bool pstart = (pidx == 0) ? (i == o) : (i == pidx * pz);
        kk[jj] = (uint32_t)kcur | (pstart ? 0x100u : 0u);
        tot += (uu[jj] >> kcur) + 1u + (uint32_t)kcur + (pstart ? (uint32_t)pb : 0u);
      }
    }
    const uint32_t inc = wave_incl_scan32(tot);
    if (lane == 63) S.scan[wv] = inc;
    __syncthreads();
    uint32_t p = pos + inc - tot;
    for (int ww = 0; ww < wv; ww++) p += S.scan[ww];
#pragma unroll
    for (int jj = 0; jj < kChunk; jj++) {
      if (kk[jj] != 0xFFFFu) {
        const int k = (int)(kk[jj] & 0xFF);
        if (kk[jj] & 0x100u) { lds_put(buf, p, (uint32_t)k, pb); p += pb; }
        const uint32_t qv = uu[jj] >> k;
        lds_put2(buf, p + qv, (k == 0) ? 1u : ((1u << k) | (uu[jj] & ((1u << k) - 1u))), k + 1);
        p += qv + 1u + (uint32_t)k;
      }
    }
    }
  }
  __syncthreads();
  uint32_t* slot = a.tmp + ((size_t)g * a.cmax + c) * a.tmp_stride;
  for (uint32_t j = t; j < nw; j += kThreads) slot[j] = buf[j];
  }
}


#ifdef FRA_STAMPS
}  // namespace fra
extern "C" __attribute__((visibility("default"))) int fra_diag_stamps(void* host, unsigned long long bytes) {
  if (!host) {
    void* d = nullptr;
    if (hipGetSymbolAddress(&d, HIP_SYMBOL(fra::g_fra_stamps)) != hipSuccess) return -1;
    return hipMemset(d, 0, sizeof(fra::g_fra_stamps)) == hipSuccess ? 0 : -1;
  }
  const size_t nb = bytes < sizeof(fra::g_fra_stamps) ? bytes : sizeof(fra::g_fra_stamps);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(fra::g_fra_stamps), nb, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
namespace fra {
#endif

hipError_t launch_analyze_w(int src, int level, const JobArgs& a, int cw, hipStream_t s);

// wave: 16-bit plans whose full frames k_analyze_w takes (fra_api.hip wave_path): k_analyze_w over the launch's
// frames, k_analyze over `part` (the launch's npart partial subframes, frame * 8 + channel), both complete
// k_analyze over a list of partial subframes (frame * 8 + channel) on stream s (the pipelined execute runs it
// on the norm stream right after the norm stage, a whole execute ahead of the frame scan that needs it)
hipError_t launch_analyze_part(int src, bool b32, const JobArgs& a, const int32_t* part, int npart,
                               int max_part_blocks, hipStream_t s) {
  if (npart <= 0) return hipSuccess;
  JobArgs wa = a;
  wa.part = part;
  wa.npart = npart;
  (void)max_part_blocks;
  if (b32) k_analyze<true, 12><<<(unsigned)npart, kThreads, 0, s>>>(wa, src);  // one workgroup per entry
  else k_analyze<false, 8><<<(unsigned)npart, kThreads, 0, s>>>(wa, src);
  return hipGetLastError();
}

// (side, ev_fork, ev_join: the partial subframes run on the side stream beside k_analyze_w -- a handful of
// workgroups that would otherwise idle the device for their whole latency after it -- joined back before the
// caller's next work on s; null side: after k_analyze_w on s)
hipError_t launch_analyze(int src, bool b32, bool ms, const JobArgs& a, hipStream_t s, bool wave, const int32_t* part,
                          int npart, int max_part_blocks, hipStream_t side, hipEvent_t ev_fork, hipEvent_t ev_join) {
  if (a.frame_count <= 0) return hipSuccess;
  dim3 grid((unsigned)a.frame_count, (unsigned)a.cmax);
  const LevelCfg cfg = level_cfg(a.level);
  const int ml = cfg.nsub == 0 ? 0 : (cfg.max_lpc <= 8 ? 8 : 12);
  if (wave && !b32 && ml == 8) {
    const int cw = ms ? 2 : a.cmax;
    hipError_t e = hipSuccess;
    auto partial = [&](hipStream_t ps) {
      JobArgs wa = a;
      wa.part = part;
      wa.npart = npart;
      k_analyze<false, 8><<<(unsigned)npart, kThreads, 0, ps>>>(wa, src);  // one workgroup per entry
    };
    const bool fork = npart > 0 && side;
    if (fork) {
      if ((e = hipEventRecord(ev_fork, s)) != hipSuccess || (e = hipStreamWaitEvent(side, ev_fork, 0)) != hipSuccess)
        return e;
      partial(side);
      if ((e = hipEventRecord(ev_join, side)) != hipSuccess) return e;
    }
    if ((e = launch_analyze_w(src, a.level, a, cw, s)) != hipSuccess) return e;
    if (fork && (e = hipStreamWaitEvent(s, ev_join, 0)) != hipSuccess) return e;
    if (npart > 0 && !side) partial(s);
    if (ms) {
      grid.y = 2;
      k_analyze<true, 8><<<grid, kThreads, 0, s>>>(a, src);
    }
    return hipGetLastError();
  }
#define FRA_LAUNCH(B, M) k_analyze<B, M><<<grid, kThreads, 0, s>>>(a, src)
  if (ms && !b32) {
    // mid-side 16-bps plan: L, R on the 16-bit instance, then M and S (17-bit samples) on the 32-bit one
    grid.y = 2;
    if (ml == 0) FRA_LAUNCH(false, 0);
    else if (ml == 8) FRA_LAUNCH(false, 8);
    else FRA_LAUNCH(false, 12);
    if (ml == 0) FRA_LAUNCH(true, 0);
    else if (ml == 8) FRA_LAUNCH(true, 8);
    else FRA_LAUNCH(true, 12);
  } else if (b32) {
    if (ml == 0) FRA_LAUNCH(true, 0);
    else if (ml == 8) FRA_LAUNCH(true, 8);
    else FRA_LAUNCH(true, 12);
  } else {
    if (ml == 0) FRA_LAUNCH(false, 0);
    else if (ml == 8) FRA_LAUNCH(false, 8);
    else FRA_LAUNCH(false, 12);
  }
#undef FRA_LAUNCH
  return hipGetLastError();
}

}  // namespace fra
