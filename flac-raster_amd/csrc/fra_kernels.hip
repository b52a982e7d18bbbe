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

template <bool B32>
__global__ void __launch_bounds__(kThreads) k_pack(JobArgs a, int src) {
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
    {
      uint32_t o_ = 0;
      int32_t a_ = 0, b_ = 0;
      load_channel(src, a.raster, st, fr, c, np, S.smp, o_, a_, b_);
    }
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
      // one generic predictor body for FIXED (integer taps, shift 0) and LPC subframes
      int32_t q[kMaxLpc];
#pragma unroll
      for (int j = 0; j < kMaxLpc; j++) q[j] = d.coef[j];
      if (type == 2) {
        const int32_t f[5][4] = {{0, 0, 0, 0}, {1, 0, 0, 0}, {2, -1, 0, 0}, {3, -3, 1, 0}, {4, -6, 4, -1}};
#pragma unroll
        for (int j = 0; j < kMaxLpc; j++) q[j] = j < 4 ? f[o][j] : 0;
      }
      const int shv = type == 3 ? d.shift : 0;
      uint32_t u[kChunk];
      uint32_t len[kChunk];
      uint32_t tot = 0;
      int pidx = i0 < n ? i0 / pz : 0;
      int pend = (pidx + 1) * pz;
      uint32_t pstartmask = 0;
      uint32_t kk[kChunk];
#pragma unroll
      for (int jj = 0; jj < kChunk; jj++) {
        const int i = i0 + jj;
        u[jj] = 0;
        len[jj] = 0;
        kk[jj] = 0;
        if (i < n && i >= o) {
          if (i >= pend) { pidx++; pend += pz; }
          const int k = d.k[pidx];
          const uint64_t uu = zz64(gres<B32, kMaxLpc>(x, jj, q, shv));
          u[jj] = (uint32_t)uu;
          kk[jj] = (uint32_t)k;
          const bool pstart = (pidx == 0) ? (i == o) : (i == pidx * pz);
          if (pstart) pstartmask |= 1u << jj;
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
        if (len[jj]) {
          const int k = (int)kk[jj];
          uint32_t pp = p;
          if ((pstartmask >> jj) & 1u) { lds_put(S.buf, pp, (uint32_t)k, pb); pp += pb; }
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

hipError_t launch_frame_bytes(const JobArgs& a, hipStream_t s) {
  k_frame_bytes<<<(a.nframes_total + 1 + 255) / 256, 256, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_pack(int src, bool b32, const JobArgs& a, hipStream_t s) {
  dim3 grid((unsigned)a.nframes_total);
  if (b32) k_pack<true><<<grid, kThreads, 0, s>>>(a, src);
  else k_pack<false><<<grid, kThreads, 0, s>>>(a, src);
  return hipGetLastError();
}

}  // namespace fra
