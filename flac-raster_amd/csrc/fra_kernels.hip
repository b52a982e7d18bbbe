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
//   k_frame_scan per frame group: header + subframe bits + pad + CRC-16 -> bytes -> byte offsets
//   (hipcub exclusive scan of frame bytes -> frame byte offsets)
//   k_pack        per frame: re-read + re-normalise, residual of the chosen model, bit-pack into
//                 an LDS bit buffer, flush to HBM at the frame's byte offset, CRC-8/CRC-16
//
// Numerics: compiled with -ffp-contract=off; every float/double expression on the decision path
// is evaluated in exactly the order the oracle uses (IEEE add/mul/div are correctly rounded on
// gfx950 and on x86-64, so identical op sequences give identical bits).
#include <algorithm>
#include <cstdlib>

#include "fra_device.h"

namespace fra {

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

// Vectorised variant (the plan's hot path): grid x = block of `rows` window rows, y = stream.
// Each lane loads V consecutive elements with one aligned vector load (the host checks that every
// window start, row, band and window width are multiples of V and that the raster pointer is
// aligned); the (row, vector) pairs of a band are spread over the whole block, 8 loads in flight
// per thread.  Per element: a 32-bit ordered key (integers: value / sign-flipped, f32: IEEE order
// key, NaN skipped) -- the same total order as okey() on the float64 value, so the result equals
// k_minmax's.
template <int SRC>
__device__ __forceinline__ uint32_t key32(typename RawType<SRC>::T x, bool& ok) {
  if constexpr (SRC == ST_U8 || SRC == ST_U16 || SRC == ST_U32) {
    ok = true;
    return (uint32_t)x;
  } else if constexpr (SRC == ST_I8 || SRC == ST_I16 || SRC == ST_I32) {
    ok = true;
    return (uint32_t)(int32_t)x ^ 0x80000000u;
  } else {  // ST_F32
    const uint32_t b = __float_as_uint(x);
    ok = x == x;
    return (b >> 31) ? ~b : (b | 0x80000000u);
  }
}
template <int SRC>
__device__ __forceinline__ double unkey32(uint32_t k) {
  if constexpr (SRC == ST_U8 || SRC == ST_U16 || SRC == ST_U32) return (double)k;
  else if constexpr (SRC == ST_I8 || SRC == ST_I16 || SRC == ST_I32) return (double)(int32_t)(k ^ 0x80000000u);
  else return (double)__uint_as_float((k >> 31) ? (k & 0x7FFFFFFFu) : ~k);
}
// streaming (nontemporal) row loads in k_minmax_vec: r05's default (C4 neutral, C3 -0.7 %, C5 quarter -0.6 %), off
// since r06: they fetch 1.105x the raster bytes against 1.007x for plain loads (in-run FETCH_SIZE, C4) and the
// same-box steps are equal (C4 1.440-1.456 / C3 0.927-0.934 ms either way; profiles/r06_ab_minmax_loads_keep17.txt)
#ifndef FRA_MM_NT
#define FRA_MM_NT 0
#endif
typedef unsigned int uint4_v __attribute__((ext_vector_type(4)));
typedef unsigned int uint2_v __attribute__((ext_vector_type(2)));
template <int SRC, int V>
__global__ void __launch_bounds__(256) k_minmax_vec(const void* raster, const StreamDev* streams, NormDev* nd,
                                                    int rows, int nrb, int nitems) {
  using T = typename RawType<SRC>::T;
  using VT = VecT<T, V>;
  // loads in flight per thread: 64 bytes, so that 256 * U vectors divide a band block of rows * nv ~ 2048
  // vectors (the host's block shape): whole rounds only -- with 48 bytes a third of the last round re-read
  // vector E-1 (C4: 3,072 slots for 2,048 vectors per band)
  constexpr int U = sizeof(VT) >= 16 ? 4 : 8;
  __shared__ uint32_t smn[4], smx[4];
  // wave issue priority over co-resident analysis waves (r05: the norm stage of a pipelined execute gates the next
  // analysis; with it and the assembly at priority 2 -- FRA_BG_PRIO, 0 = off -- C3 -3.6 %, the C4 8-way share -5 %,
  // C4 and the C5 quarter neutral, profiles/r05_ab_background.txt 14; the analysis raised instead: C4 +5.5 %)
  if (FRA_BG_PRIO > 0) __builtin_amdgcn_s_setprio(FRA_BG_PRIO);
  const int wv = threadIdx.x >> 6;
  // items (stream, block of `rows` rows) = (item / nrb, item % nrb); a full grid has one item per
  // workgroup (the default, serial and pipelined); a smaller grid (FRA_MM_PER_CU) strides over them
  for (int item = blockIdx.x; item < nitems; item += gridDim.x) {
    const int si = item / nrb;
    const StreamDev st = streams[si];
    const int r0 = (item - si * nrb) * rows;
    if (st.norm == 0 || r0 >= st.height) continue;  // uniform
    const int nr = min(st.height - r0, rows);
    const uint32_t nv = (uint32_t)(st.width / V);
    const uint32_t E = (uint32_t)nr * nv;  // (row, vector) items per band
    // idx / nv by multiply-high: exact while E * nv < 2^32 (checked on the host); nv == 1 (a window one
    // vector wide) would wrap the multiplier to 0, so it divides by 1 directly (uniform branch)
    const uint32_t magic = nv > 1 ? 0xFFFFFFFFu / nv + 1u : 0u;
    uint32_t kmin = ~0u, kmax = 0u;
    for (int b = 0; b < st.channels; b++) {
      // uniform base + 32-bit byte offsets (host: rows * row_stride * itemsize < 2^32): one offset VGPR
      // per load instead of a 64-bit address pair, so the kernel fits the 32 VGPRs a co-resident
      // k_analyze leaves free on each SIMD (cross-execute overlap)
      const char* base =
          (const char*)((const T*)raster + st.base_off + (int64_t)b * st.band_stride + (int64_t)r0 * st.row_stride);
      const uint32_t rsb = (uint32_t)st.row_stride * (uint32_t)sizeof(T);
      for (uint32_t i0 = 0; i0 < E; i0 += 256 * U) {
        VT x[U];
#pragma unroll
        for (int u = 0; u < U; u++) {  // items past E re-read item E-1 (idempotent for min/max)
          const uint32_t idx = min(i0 + (uint32_t)(u * 256) + threadIdx.x, E - 1);
          const uint32_t r = nv > 1 ? __umulhi(idx, magic) : idx, v = idx - r * nv;
          const VT* px = (const VT*)(base + (r * rsb + v * (uint32_t)sizeof(VT)));
#if FRA_MM_NT
          // streaming loads (r05): the rows pass through L2 / the Infinity Cache without displacing what the
          // analysis beside it gathers there (the per-tile tables)
          if constexpr (sizeof(VT) == 16) x[u] = __builtin_bit_cast(VT, __builtin_nontemporal_load((const uint4_v*)px));
          else if constexpr (sizeof(VT) == 8) x[u] = __builtin_bit_cast(VT, __builtin_nontemporal_load((const uint2_v*)px));
          else x[u] = *px;
#else
          x[u] = *px;
#endif
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
#pragma unroll
          for (int e = 0; e < V; e++) {
            bool ok;
            const uint32_t k = key32<SRC>(x[u].v[e], ok);
            kmin = ok ? min(kmin, k) : kmin;
            kmax = ok ? max(kmax, k) : kmax;
          }
        }
      }
    }
    kmin = wave_min32(kmin);
    kmax = ~wave_min32(~kmax);
    if ((threadIdx.x & 63) == 0) { smn[wv] = kmin; smx[wv] = kmax; }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < 4; w++) { kmin = min(kmin, smn[w]); kmax = max(kmax, smx[w]); }
      if (kmin <= kmax) {  // at least one non-NaN value
        atomicMin(&nd[si].mnkey, okey(unkey32<SRC>(kmin)));
        atomicMax(&nd[si].mxkey, okey(unkey32<SRC>(kmax)));
      }
    }
    __syncthreads();  // smn/smx reused by the next item
  }
}

// One frame's header (+ CRC-8) and blob bit bounds -> fmeta, its byte size -> frame_bytes; returns the size.
// FRA-1 3.1b: a mid-side stream keeps the first minimum of L+R, L+S, S+R, M+S (virtual channels 0..3)
__device__ uint64_t frame_bytes_one(const JobArgs& a, int g) {
  const FrameDev fr = a.frames[g];
  const StreamDev st = a.streams[fr.stream];
  int chan_code = st.channels - 1, va = 0, vb = 1;
  if (st.ms) {
    const SfDesc* sd = a.sf + (size_t)g * a.cmax;
    const uint64_t bl = sd[0].bits, br = sd[1].bits, bm = sd[2].bits, bs = sd[3].bits;
    const uint64_t tot[4] = {bl + br, bl + bs, bs + br, bm + bs};
    int best = 0;
    for (int k = 1; k < 4; k++)
      if (tot[k] < tot[best]) best = k;
    chan_code = best == 0 ? 1 : 7 + best;  // 1 independent, 8 left/side, 9 side/right, 10 mid/side
    va = best == 0 ? 0 : (best == 1 ? 0 : (best == 2 ? 3 : 2));
    vb = best == 0 ? 1 : (best == 1 ? 3 : (best == 2 ? 1 : 3));
  }
  uint8_t h[4 * kHdrWords];
  int hl = frame_header(h, st, fr, chan_code);
  uint32_t c8 = 0;  // CRC-8, poly x^8+x^2+x+1, init 0 (RFC 9639 9.1.8)
  for (int i = 0; i < hl; i++) {
    c8 ^= h[i];
    for (int b = 0; b < 8; b++) c8 = (c8 & 0x80u) ? ((c8 << 1) ^ 0x07u) & 0xFF : (c8 << 1);
  }
  h[hl++] = (uint8_t)c8;
  uint32_t* m = a.fmeta + (size_t)g * kMetaWords;
  uint32_t w[kHdrWords] = {};
  for (int b = 0; b < hl; b++) w[b >> 2] |= (uint32_t)h[b] << (24 - 8 * (b & 3));
  // header <= 16 bytes (words 0-3); word kHdrWords - 1 carries the slot of output channels 0 and 1
  w[kHdrWords - 1] = (uint32_t)va | ((uint32_t)vb << 8);
#pragma unroll
  for (int j = 0; j < kHdrWords; j++) m[j] = w[j];
  uint32_t bits = (uint32_t)hl * 8;
  m[kHdrWords] = 0;
  m[kHdrWords + 1] = bits;
#pragma unroll
  for (int c = 0; c < kMaxChannels; c++) {
    const int vc = c == 0 ? va : (c == 1 ? vb : c);
    if (c < st.channels) bits += a.sf[(size_t)g * a.cmax + vc].bits;
    m[kHdrWords + 2 + c] = c < st.channels ? bits : 0xFFFFFFFFu;
  }
  const uint64_t fb = ((uint64_t)(bits + 7) >> 3) + 2;
  a.frame_bytes[g] = fb;
  return fb;
}

// Frame sizes -> byte offsets of a frame group in ONE launch (replaces k_frame_bytes + a library exclusive
// scan + k_group_offsets: two to three fewer dependent launches per execute): every workgroup sizes 256 x ITEMS
// frames, then a single-pass scan with decoupled look-back (Merrill & Garland) over
// workgroups in TICKET order -- a workgroup only ever waits on workgroups that took an earlier ticket, so
// are already running: no assumption on dispatch order or co-residency.  The look-back reads 64
// predecessors per round (one per lane) and stops at the nearest inclusive prefix.  Look-back words:
// [63:62] flag (0 not yet published, 1 aggregate, 2 inclusive prefix), [61:0] bytes; each word carries its
// own payload, so relaxed device-scope atomics suffice (no acquire/release cache maintenance per look-back
// round).  add_base: the group's base offset gbase[grp] is ordered before this launch -> final offsets,
// gbase[grp+1] (+ frame_off[nframes] for the last group, + the host mirror); else group-relative offsets
// (k_group_offsets adds the base once the previous group is done).
//
// The scan state lives on the device, so a launch needs no host-side counter (graph replays and failed
// enqueues cannot desynchronise it): per slot one 64-bit control word, [63:32] epoch, [31:0] next ticket.
// The workgroup that takes the launch's last ticket resets the ticket and advances the epoch (every other
// ticket of the launch is already taken); launch epoch e publishes into half e & 1 of the slot's look-back
// words and zeroes the other half for the next launch (launches on one slot are stream ordered).  A ticket
// past the grid (a desynchronised control word) sets bit 0 of the plan's error word and publishes nothing.
constexpr uint64_t kScanValMask = (1ull << 62) - 1;
constexpr uint64_t kScanAgg = 1ull << 62, kScanInc = 2ull << 62;
template <int ITEMS>  // frames per thread (contiguous): 256 * ITEMS per workgroup
__global__ void __launch_bounds__(256) k_frame_scan(JobArgs a, unsigned long long* gbase, int grp, int last,
                                                    int add_base, unsigned long long* host_mirror,
                                                    unsigned long long* look2, int look_stride,
                                                    unsigned long long* ctl) {
  __shared__ unsigned s_t, s_half;
  __shared__ uint64_t s_w[4];
  __shared__ uint64_t s_excl;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) {
    const unsigned long long old = atomicAdd(ctl, 1ull);
    const unsigned tk = (unsigned)old, ep = (unsigned)(old >> 32);
    if (tk == gridDim.x - 1)
      __hip_atomic_store(ctl, (unsigned long long)(ep + 1u) << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tk >= gridDim.x && a.err) atomicOr(a.err, 1u);
    s_t = tk;
    s_half = ep & 1u;
  }
  __syncthreads();
  if (s_t >= gridDim.x) return;  // (nobody waits on a ticket past the grid)
  const int t = (int)s_t;  // this workgroup's position in the scan
  unsigned long long* const look = look2 + (size_t)s_half * look_stride;
  {
    unsigned long long* const nxt = look2 + (size_t)(s_half ^ 1u) * look_stride;
    for (int i = t * 256 + tid; i < look_stride; i += (int)gridDim.x * 256) nxt[i] = 0ull;
  }
  const int n = a.frame_count;
  const int i0 = (t * 256 + tid) * ITEMS;
  uint64_t fb[ITEMS], loc = 0;
#pragma unroll
  for (int k = 0; k < ITEMS; k++) {
    fb[k] = i0 + k < n ? frame_bytes_one(a, a.frame_base + i0 + k) : 0ull;
    loc += fb[k];
  }
  // workgroup-inclusive scan of the per-thread sums: wave scan by shuffles, then the 4 wave totals
  uint64_t incl = loc;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t v = __shfl_up(incl, d, 64);
    if (lane >= d) incl += v;
  }
  if (lane == 63) s_w[wv] = incl;
  __syncthreads();
  uint64_t wbase = 0, agg = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    wbase += k < wv ? s_w[k] : 0ull;
    agg += s_w[k];
  }
  if (wv == 0) {
    if (lane == 0)
      __hip_atomic_store(&look[t], (t == 0 ? kScanInc : kScanAgg) | (agg & kScanValMask), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint64_t excl = 0;
    for (int j0 = t - 1; j0 >= 0;) {
      // lane l looks at workgroup j0 - l; before workgroup 0: an inclusive prefix of 0
      const int j = j0 - lane;
      const uint64_t w = j >= 0 ? __hip_atomic_load(&look[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kScanInc;
      const uint32_t fl = (uint32_t)(w >> 62);
      const uint64_t incm = __ballot(fl == 2), nrdy = __ballot(fl == 0);
      const int stop = incm ? (int)__builtin_ctzll(incm) : 64;  // the nearest inclusive prefix
      const uint64_t need = stop >= 63 ? ~0ull : ((2ull << stop) - 1);
      if (nrdy & need) {  // a workgroup in the window (an earlier ticket, so running) has not published yet
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      uint64_t v = lane <= stop ? (w & kScanValMask) : 0ull;
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
      excl += v;
      if (stop < 64) break;
      j0 -= 64;
    }
    if (lane == 0) {
      if (t > 0)
        __hip_atomic_store(&look[t], kScanInc | ((excl + agg) & kScanValMask), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      s_excl = excl;
    }
  }
  __syncthreads();
  const uint64_t base = add_base && grp > 0 ? gbase[grp] : 0ull;
  uint64_t off = base + s_excl + wbase + incl - loc;
#pragma unroll
  for (int k = 0; k < ITEMS; k++) {
    const int i = i0 + k;
    if (i < n) {
      a.frame_off[a.frame_base + i] = off;
      off += fb[k];
      if (add_base && i == n - 1) {  // the group's end
        gbase[grp + 1] = off;
        if (last) a.frame_off[a.nframes_total] = off;
        if (host_mirror) {  // page-locked host copy for the host pipeline (no copy-engine command needed)
          host_mirror[grp + 1] = off;
          __threadfence_system();
        }
      }
    }
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

// normalize_to_audio table of a <= 16-bit integer stream, indexed by the raw value itself (lut_index: the
// value's bit pattern as an unsigned 8/16-bit integer, so k_analyze gathers with one 32-bit offset from a
// uniform base): entry of raster value v = the normalised sample of v, for v = mn..mx (the only values the
// tile holds), by the same op sequence as norm_sample.  grid (64, streams), grid-stride over v - mn.
template <int SRC>
__global__ void __launch_bounds__(256) k_norm_lut(const StreamDev* streams, const NormDev* nd, int32_t* lut,
                                                  int64_t stride) {
  const StreamDev st = streams[blockIdx.y];
  if (st.norm == 0 || nd[blockIdx.y].mnkey == ~0ull) return;
  const NormParams np = norm_params(st, nd[blockIdx.y]);
  const int64_t R = (int64_t)np.range;  // integer data: mx - mn, or 1 for a constant stream
  int32_t* out = lut + (int64_t)blockIdx.y * stride;
  for (int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x; d <= R && d < stride; d += (int64_t)gridDim.x * 256) {
    const int v = (int)np.mn + (int)d;
    out[lut_index<SRC>((typename RawType<SRC>::T)v)] = norm_sample<SRC>(np.mn + (double)d, np);
  }
}

hipError_t launch_norm_lut(int src, const JobArgs& a, int nstreams, hipStream_t s) {
  if (!a.lut) return hipSuccess;
  dim3 grid(64, (unsigned)nstreams);
  switch (src) {
    case ST_U8: k_norm_lut<ST_U8><<<grid, 256, 0, s>>>(a.streams, a.norm, (int32_t*)a.lut, a.lut_stride); break;
    case ST_I8: k_norm_lut<ST_I8><<<grid, 256, 0, s>>>(a.streams, a.norm, (int32_t*)a.lut, a.lut_stride); break;
    case ST_U16: k_norm_lut<ST_U16><<<grid, 256, 0, s>>>(a.streams, a.norm, (int32_t*)a.lut, a.lut_stride); break;
    case ST_I16: k_norm_lut<ST_I16><<<grid, 256, 0, s>>>(a.streams, a.norm, (int32_t*)a.lut, a.lut_stride); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_norm_finalize(const JobArgs& a, int nstreams, hipStream_t s) {
  k_norm_finalize<<<(nstreams + 255) / 256, 256, 0, s>>>(a.streams, a.norm, nstreams);
  return hipGetLastError();
}

// vec_bytes = 16 or 8: vector path (host-checked alignment), rows/max_rows its block shape; 0: scalar
hipError_t launch_minmax(int src, const JobArgs& a, int nstreams, int max_segs, int vec_bytes, int rows, int max_rows,
                         hipStream_t s, int max_blocks) {
  k_norm_init<<<(nstreams + 255) / 256, 256, 0, s>>>(a.norm, nstreams);
  if (vec_bytes == 16 || vec_bytes == 8) {
    const int nrb = (max_rows + rows - 1) / rows, nitems = nrb * nstreams;
    const unsigned vgrid = (unsigned)(max_blocks > 0 ? std::min(max_blocks, nitems) : nitems);
#define V(S_, T_)                                                                               \
  case S_:                                                                                      \
    if (vec_bytes == 16) k_minmax_vec<S_, 16 / sizeof(T_)><<<vgrid, 256, 0, s>>>(a.raster, a.streams, a.norm, rows, nrb, nitems); \
    else k_minmax_vec<S_, 8 / sizeof(T_)><<<vgrid, 256, 0, s>>>(a.raster, a.streams, a.norm, rows, nrb, nitems);                  \
    return hipGetLastError();
    switch (src) {
      V(ST_U8, uint8_t) V(ST_I8, int8_t) V(ST_U16, uint16_t) V(ST_I16, int16_t)
      V(ST_U32, uint32_t) V(ST_I32, int32_t) V(ST_F32, float)
      default: break;  // f64: scalar path
    }
#undef V
  }
  dim3 grid((unsigned)max_segs, (unsigned)nstreams);
  switch (src) {
#define M(S_) case S_: k_minmax<S_><<<grid, 256, 0, s>>>(a.raster, a.streams, a.norm); break;
    FRA_SRC_CASES(M)
#undef M
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// frames per thread: one up to 65,536 frames (C4: 0.026 ms serial against 0.053 at four), then 4 / 16 so a
// C5-size group stays at <= 256 workgroups beside the next execute's analysis
// (FRA_SCAN_ITEMS=1/4/16 forces one form for tests; it must be set before the plan is created, which sizes the
// look-back words by it)
static int scan_items(int nframes) {
  if (const char* e = getenv("FRA_SCAN_ITEMS")) {
    const int v = atoi(e);
    if (v == 1 || v == 4 || v == 16) return v;
  }
  return nframes <= 65536 ? 1 : (nframes <= 4 * 65536 ? 4 : 16);
}
int frame_scan_blocks(int nframes) {
  const int per = 256 * scan_items(nframes);
  return (nframes + per - 1) / per;
}
hipError_t launch_frame_scan(const JobArgs& a, unsigned long long* gbase, int grp, int last, int add_base,
                             unsigned long long* host_mirror, unsigned long long* look2, int look_stride,
                             unsigned long long* ctl, hipStream_t s) {
  if (a.frame_count > 0) {
    const int it = scan_items(a.frame_count), nb = frame_scan_blocks(a.frame_count);
    if (nb > look_stride) return hipErrorInvalidValue;
    if (it == 1) k_frame_scan<1><<<nb, 256, 0, s>>>(a, gbase, grp, last, add_base, host_mirror, look2, look_stride, ctl);
    else if (it == 4) k_frame_scan<4><<<nb, 256, 0, s>>>(a, gbase, grp, last, add_base, host_mirror, look2, look_stride, ctl);
    else k_frame_scan<16><<<nb, 256, 0, s>>>(a, gbase, grp, last, add_base, host_mirror, look2, look_stride, ctl);
  }
  return hipGetLastError();
}

// Frame group -> global byte offsets.  frame_off[f0, f0 + n) holds the group's own exclusive scan;
// gbase[grp] (written by the previous group's launch, ordered by an event) is the byte offset of the
// group's first frame.  Adds it, publishes gbase[grp + 1] and, for the last group, frame_off[nframes].
__global__ void k_group_offsets(unsigned long long* frame_off, const unsigned long long* frame_bytes,
                                unsigned long long* gbase, int grp, int f0, int n, int last, int nframes,
                                unsigned long long* host_mirror) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long base = grp == 0 ? 0ull : gbase[grp];
  if (i < n) {
    const unsigned long long loc = frame_off[f0 + i];
    frame_off[f0 + i] = loc + base;
    if (i == n - 1) {
      const unsigned long long end = base + loc + frame_bytes[f0 + i];
      gbase[grp + 1] = end;
      if (last) frame_off[nframes] = end;
      if (host_mirror) {  // page-locked host copy for the host pipeline (no copy-engine command needed)
        host_mirror[grp + 1] = end;
        __threadfence_system();
      }
    }
  } else if (i == 0) {  // empty group
    gbase[grp + 1] = base;
    if (last) frame_off[nframes] = base;
    if (host_mirror) {
      host_mirror[grp + 1] = base;
      __threadfence_system();
    }
  }
}

hipError_t launch_group_offsets(unsigned long long* frame_off, const unsigned long long* frame_bytes,
                                unsigned long long* gbase, int grp, int f0, int n, int last, int nframes,
                                hipStream_t s, unsigned long long* host_mirror) {
  k_group_offsets<<<((n > 1 ? n : 1) + 255) / 256, 256, 0, s>>>(frame_off, frame_bytes, gbase, grp, f0, n, last,
                                                              nframes, host_mirror);
  return hipGetLastError();
}

// ============================================================================ fra_normalize (standalone a3)
// normalize_to_audio of a flat (N, C) array, normalization.py:126-202.  Not on the encode path (the
// encoder fuses this into k_analyze); IEEE division here because user-supplied data_min/data_max
// overrides void the integer-range precondition of div_markstein.
template <int SRC>
__global__ void __launch_bounds__(256) k_minmax_flat(const void* data, uint64_t n, NormDev* nd) {
  unsigned long long kmin = ~0ull, kmax = 0ull;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const double v = load_f64<SRC>(data, (int64_t)i);
    if (v == v) {
      const unsigned long long k = okey(v);
      kmin = k < kmin ? k : kmin;
      kmax = k > kmax ? k : kmax;
    }
  }
  for (int off = 32; off >= 1; off >>= 1) {
    const unsigned long long a = ((unsigned long long)__shfl_xor((uint32_t)(kmin >> 32), off, 64) << 32) |
                                 __shfl_xor((uint32_t)kmin, off, 64);
    const unsigned long long b = ((unsigned long long)__shfl_xor((uint32_t)(kmax >> 32), off, 64) << 32) |
                                 __shfl_xor((uint32_t)kmax, off, 64);
    kmin = a < kmin ? a : kmin;
    kmax = b > kmax ? b : kmax;
  }
  if ((threadIdx.x & 63) == 0 && kmin != ~0ull) {
    atomicMin(&nd->mnkey, kmin);
    atomicMax(&nd->mxkey, kmax);
  }
}

__global__ void k_norm_finalize_flat(NormDev* nd, int has_min, double omin, int has_max, double omax) {
  const double qnan = __longlong_as_double(0x7FF8000000000000ll);
  const bool none = nd->mnkey == ~0ull;
  const double mn = has_min ? omin : (none ? qnan : unkey(nd->mnkey));
  const double mx = has_max ? omax : (none ? qnan : unkey(nd->mxkey));
  nd->mn = mn;
  nd->mx = mx;
  nd->range = (mx <= mn) ? 1.0 : (mx - mn);  // normalization.py:154-159
}

template <int SRC>
__global__ void __launch_bounds__(256) k_normalize_flat(const void* data, uint64_t n, const NormDev* nd, int bps,
                                                        void* out) {
  const double mn = nd->mn, range = nd->range;
  const double scale = bps == 16 ? 32767.0 : (bps == 24 ? 8388607.0 : 2147483647.0);
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    double t = load_f64<SRC>(data, (int64_t)i) - mn;
    t = 2.0 * t;
    t = t / range;
    t = t - 1.0;
    if (t < -1.0) t = -1.0;
    else if (t > 1.0) t = 1.0;
    if (t != t) t = 0.0;
    t = t * scale;
    if (bps == 16) ((int16_t*)out)[i] = (int16_t)(int32_t)t;
    else ((int32_t*)out)[i] = (int32_t)t;
  }
}

hipError_t launch_normalize_flat(int src, const void* data, uint64_t n, int bps, NormDev* nd, int has_min, double omin,
                                 int has_max, double omax, void* out, hipStream_t s) {
  k_norm_init<<<1, 64, 0, s>>>(nd, 1);
  const unsigned grid = (unsigned)std::min<uint64_t>(8192, std::max<uint64_t>(1, (n + 255) / 256));
  if (!(has_min && has_max) && n) {
    switch (src) {
#define M(S_) case S_: k_minmax_flat<S_><<<grid, 256, 0, s>>>(data, n, nd); break;
      FRA_SRC_CASES(M)
#undef M
      default: return hipErrorInvalidValue;
    }
  }
  k_norm_finalize_flat<<<1, 1, 0, s>>>(nd, has_min, omin, has_max, omax);
  if (n) {
    switch (src) {
#define M(S_) case S_: k_normalize_flat<S_><<<grid, 256, 0, s>>>(data, n, nd, bps, out); break;
      FRA_SRC_CASES(M)
#undef M
      default: return hipErrorInvalidValue;
    }
  }
  return hipGetLastError();
}

}  // namespace fra
