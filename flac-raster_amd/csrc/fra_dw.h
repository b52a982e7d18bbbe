// fra_dw.h -- direct write of encoded subframes, included by fra_analyze.hip.
//
// What k_frame_bytes + scan + k_assemble (fra_kernels.hip, fra_pack.hip) do in three launches and a slot
// round trip through HBM, done at the end of the 16-bit k_analyze instead: the frames libFLAC emits for
// each block (FLAC__stream_encoder_process_interleaved under converter.py:153 / spatial_encoder.py:303)
// are header ++ subframes ++ byte pad ++ CRC-16 (RFC 9639 9.1-9.3); every subframe's final bit offset
// follows from the sizes of all subframes before it in (frame, channel) order.
//
// Launch order = output order: workgroup li of a launch is subframe (frame_base + li / C, li % C).
//  1. publish the look-back word {epoch, aggregate, bits} of this subframe
//  2. CRC-16 residue of the subframe's bit string (slice-by-4 tables in LDS, per-thread runs of m words,
//     each run weighted by x^(32 m (255 - t) - pad) from the x^e table, xor over the workgroup) and its
//     last 8 bits -> residue word
//  3. decoupled look-back (one wave): the 64 predecessors' look-back words (agent-scope, L1-bypassing
//     8-byte loads: each word is its own {data, tag} granule), the nearest inclusive one + the aggregates
//     after it give this subframe's bit offset P (frame ends add the byte pad, the CRC-16 and the next
//     header); publish the inclusive word.  A wait longer than kDwTimeout sets the abort flag and the
//     workgroup leaves: the host redoes the whole launch through the slot path (nothing is lost but time).
//  4. bytes fully inside [P, P + bits) are stored (dwords where whole); the byte shared with the
//     predecessor is merged with its last bits (residue word); the frame's first subframe writes the
//     header, its last one the zero-padded tail byte, the frame CRC-16 (residues combined with x^e
//     weights) and frame_off / frame_bytes.
#pragma once

#include "fra_device.h"

namespace fra {

constexpr uint64_t kLbMask = (1ull << 47) - 1;

// look-back words are hand-off granules: one 8-byte agent-scope store each, polled by agent-scope loads
// (global_ ... sc1, not flat_: the pointers come from DwCtl as generic pointers)
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) int gi32_t;
__device__ __forceinline__ uint64_t lb_load(const unsigned long long* p) {
  return __hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(unsigned long long* p, uint64_t v) {
  __hip_atomic_store((gu64_t*)p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int flag_load(const int* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load((gi32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t wave_xor32(uint32_t v) {  // wave-uniform result
  v ^= dpp32<DPP_SHR1, 0xF>(v);
  v ^= dpp32<DPP_SHR2, 0xF>(v);
  v ^= dpp32<DPP_SHR4, 0xF>(v);
  v ^= dpp32<DPP_SHR8, 0xF>(v);
  v ^= dpp32<DPP_BC15, 0xA>(v);
  v ^= dpp32<DPP_BC31, 0xC>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// T = slice-by-4 CRC-16 tables (T[k][v] = v x^(8k+16) mod P), crc register semantics: CRC(s) = s(x) x^16 mod P
__device__ __forceinline__ uint32_t crc_word(uint32_t crc, uint32_t w, const uint16_t* T) {
  return (uint32_t)T[768 + (((w >> 24) ^ (crc >> 8)) & 0xFFu)] ^ (uint32_t)T[512 + (((w >> 16) ^ crc) & 0xFFu)] ^
         (uint32_t)T[256 + ((w >> 8) & 0xFFu)] ^ (uint32_t)T[w & 0xFFu];
}
// a * b mod P (16-bit operands): carry-less product, its high 15 bits folded by T[1], T[0]
__device__ __forceinline__ uint32_t gf16_mul_t(uint32_t a, uint32_t b, const uint16_t* T) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) p ^= (a << i) & (uint32_t)__builtin_amdgcn_sbfe((int)b, i, 1);
  const uint32_t hi = p >> 16;
  return (p & 0xFFFFu) ^ (uint32_t)T[256 + (hi >> 8)] ^ (uint32_t)T[hi & 0xFFu];
}
__device__ __forceinline__ int xexp(int64_t e) {  // e mod kXOrd in [0, kXOrd)
  int r = (int)(e % kXOrd);
  return r < 0 ? r + kXOrd : r;
}

// Position transform of a run of subframes: A(x): s -> s + x (no frame end inside), C(x, y):
// s -> roundup8(s + x) + y (a frame ends inside: byte pad, then y more bits: CRC-16, next header, ...).
// Closed under composition, so any run of look-back aggregates folds into one (c, x, y).
struct Tf {
  uint32_t c;
  uint64_t x, y;
};
__device__ __forceinline__ Tf tf_then(const Tf& f, const Tf& g) {  // f first, then g
  if (!g.c) return f.c ? Tf{1u, f.x, f.y + g.x} : Tf{0u, f.x + g.x, 0ull};
  return f.c ? Tf{1u, f.x, ((f.y + g.x + 7) & ~7ull) + g.y} : Tf{1u, f.x + g.x, g.y};
}
__device__ __forceinline__ uint64_t tf_apply(const Tf& f, uint64_t s) {
  return f.c ? ((s + f.x + 7) & ~7ull) + f.y : s + f.x;
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}
// composition of the lanes' transforms, lane 63 applied first and lane 0 last (lane l = predecessor l + 1
// back); every lane gets the result (butterfly: the lower, nearer block is applied after the upper one)
__device__ __forceinline__ Tf tf_wave(Tf t, int lane) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    const Tf p{(uint32_t)__shfl_xor((int)t.c, m, 64), shfl_xor64(t.x, m), shfl_xor64(t.y, m)};
    t = (lane & m) ? tf_then(t, p) : tf_then(p, t);
  }
  return t;
}

// LDS scratch of the emit stage (over dead analysis arrays)
struct DwScratch {
  uint16_t T[4 * 256];
  uint32_t red[4];
  unsigned long long P;
  int abort;
};

// the aggregate (bits) of launch subframe li for the successors' look-back: as soon as the size is decided
__device__ __forceinline__ void dw_publish(const JobArgs& a, int li, uint32_t len) {
  const DwCtl* dw = reinterpret_cast<const DwCtl*>(a.tmp);
  const uint64_t epoch = (uint64_t)a.tmp_stride & 0xFFFFu;
  lb_store(&dw->lb[2 * ((int64_t)a.frame_base * a.cmax + li)], (epoch << 48) | (uint64_t)len);
}
// CRC-16 slice-by-4 tables to LDS (2 KiB, 16-byte loads of threads 0..127), over dead analysis arrays
__device__ __forceinline__ void dw_tables(const JobArgs& a, DwScratch& X, int t) {
  if (t < 128) reinterpret_cast<uint4*>(X.T)[t] = reinterpret_cast<const uint4*>(a.crctab)[t];
}

// One subframe at the end of k_analyze: its bit string (big-endian words, MSB first, `len` bits, zero
// after len and one zero word past the end) in the LDS buffer `buf`.  Called by all 256 threads.
// early: dw_publish + dw_tables already done and a barrier passed since (buf complete, tables visible).
__device__ __forceinline__ void dw_emit(const JobArgs& a, const uint32_t* buf, uint32_t len, int li, int C,
                                        uint64_t ts0, DwScratch& X, int t, bool early, bool sync) {
  const DwCtl* dw = reinterpret_cast<const DwCtl*>(a.tmp);
  const uint32_t epoch = (uint32_t)a.tmp_stride & 0xFFFFu;
  const int grp = (int)((a.tmp_stride >> 16) & 0x7FFFFFFF);
  const bool last_grp = ((a.tmp_stride >> 47) & 1) != 0;
  const int lane = t & 63, wv = t >> 6;
  const int g = a.frame_base + li / C, c = li % C;
  const int64_t e0 = (int64_t)a.frame_base * C;  // element index of the launch's first subframe
  const int64_t e = e0 + li;
  unsigned long long* lb = dw->lb;
  const uint64_t tag = (uint64_t)epoch << 48;
  const uint64_t tmo = dw->timeout;
  unsigned long long* tr = dw->trace ? dw->trace + 4 * (size_t)li : nullptr;
  // 1. aggregate (bits) for the successors' look-back, CRC tables
  if (!early) {
    if (t == 0) lb_store(&lb[2 * e], tag | (uint64_t)len);
    dw_tables(a, X, t);
  }
  if (t == 0 && tr) {
    tr[0] = ts0;
    tr[1] = __builtin_amdgcn_s_memrealtime();
  }
  if (sync || !early) __syncthreads();
  const uint32_t nw = (len + 31) >> 5;
  // 2. residue on waves 1-3 (wave 0 does the look-back meanwhile): thread ct = t - 64 folds padded words
  // [ct m, ct m + m) (leading zero words before the blob), weighted by x^(32 m (191 - ct) - pad)
  if (wv > 0) {
    const int ct = t - 64;
    const uint32_t m = ((nw + 191) / 192) | 1u;  // words per thread, odd: conflict-free LDS strides
    const uint32_t padw = 32 * nw - len;
    const uint32_t xw = a.crctab[kXpowOff + xexp((int64_t)32 * m * (uint32_t)(191 - ct) - (int64_t)padw)];
    uint32_t crc = 0;
    int q = (int)(ct * m) - (int)(192 * m - nw);
    for (uint32_t r = 0; r < m; r++, q++)
      if (q >= 0) crc = crc_word(crc, buf[q], X.T);
    crc = crc ? gf16_mul_t(crc, xw, X.T) : 0u;
    crc = wave_xor32(crc);
    if (lane == 0) X.red[wv] = crc;
  }

  // 3. look-back on wave 0: windows of 64 predecessors (lane l = l + 1 back); a window of aggregates
  // without an inclusive word folds into acc and the walk moves 64 further back
  if (wv == 0) {
    // bit offset of the launch's first subframe (the j == -1 lane of whichever window reaches it)
    const uint64_t base = 8 * (grp == 0 ? 0ull : dw->gbase[grp]) + 8 * (uint64_t)dw->hbytes[a.frame_base];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    bool aborted = false;
    uint64_t P = 0, bi = 0, bo = 0;
    Tf acc{0u, 0ull, 0ull};  // windows already folded (nearer than the current one)
    int j = li - 1 - lane;
    uint32_t ynext = (j >= 0 && (j % C) == C - 1) ? 16u + 8u * dw->hbytes[a.frame_base + j / C + 1] : 0u;
    for (;;) {
      const uint64_t v = j >= 0 ? lb_load(&lb[2 * (e0 + j)]) : (j == -1 ? (tag | (1ull << 47) | base) : 0ull);
      const bool ok = j >= -1 && (v >> 48) == epoch;
      const bool inc = ok && ((v >> 47) & 1);
      bi = __ballot(inc);
      bo = __ballot(ok);
      const int k = bi ? (int)__builtin_ctzll(bi) : 64;
      const uint64_t need = k < 64 ? (1ull << k) - 1 : ~0ull;
      if ((bo & need) == need) {
        // lanes 0..k-1 are aggregates: their transforms (identity from lane k on)
        const Tf mine = lane < k ? Tf{ynext ? 1u : 0u, v & kLbMask, (uint64_t)ynext} : Tf{0u, 0ull, 0ull};
        const Tf w = tf_wave(mine, lane);
        if (bi) {
          P = tf_apply(acc, tf_apply(w, readlane64(v, k) & kLbMask));
          break;
        }
        acc = tf_then(w, acc);  // a whole window of aggregates: fold it, go 64 further back
        j -= 64;
        ynext = (j >= 0 && (j % C) == C - 1) ? 16u + 8u * dw->hbytes[a.frame_base + j / C + 1] : 0u;
        continue;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > tmo || flag_load(dw->abort_dev)) {
        aborted = true;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    [[maybe_unused]] const uint64_t dbg_bi = bi, dbg_bo = bo;
    // (defensive: an offset past the output would be a bug upstream -- redo through the slot path)
    if (!aborted && ((P + len + 7) >> 3) + 2 + 16 > a.out_cap) aborted = true;
    if (lane == 0) {
      if (aborted) {
#ifdef FRA_DW_DEBUG
        printf("dw abort: li %d g %d c %d C %d epoch %u bi %llx bo %llx P %llu len %u cap %llu dt %llu\n", li, g, c, C,
               epoch, (unsigned long long)dbg_bi, (unsigned long long)dbg_bo, (unsigned long long)P, len,
               (unsigned long long)a.out_cap, (unsigned long long)(__builtin_amdgcn_s_memrealtime() - t0));
#endif
        if (atomicCAS(&dw->diag[0], 0ull, (unsigned long long)li + 1) == 0ull) {
          dw->diag[1] = dbg_bi;
          dw->diag[2] = dbg_bo;
          dw->diag[3] = __builtin_amdgcn_s_memrealtime() - t0;
          dw->diag[4] = epoch;
          dw->diag[5] = P;
          dw->diag[6] = len;
        }
        atomicAdd(&dw->diag[7], 1ull);
        __hip_atomic_store((gi32_t*)dw->abort_dev, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(dw->abort_host, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        const int y = c == C - 1 ? 16 + 8 * (int)dw->hbytes[g + 1] : 0;
        const uint64_t inc = y ? (((P + len + 7) & ~7ull) + (uint64_t)y) : P + len;
        lb_store(&lb[2 * e], tag | (1ull << 47) | inc);
      }
      X.P = P;
      X.abort = aborted ? 1 : 0;
      if (tr) tr[2] = __builtin_amdgcn_s_memrealtime();
    }
  }
  __syncthreads();
  const uint32_t R = X.red[1] ^ X.red[2] ^ X.red[3];
  if (t == 0) {  // residue word: bits, last 8 bits (len >= 12), CRC-16 residue
    const uint32_t lb8 = len - 8;
    const uint32_t last8 =
        (uint32_t)(((((uint64_t)buf[lb8 >> 5] << 32) | buf[(lb8 >> 5) + 1]) << (lb8 & 31)) >> 56);
    lb_store(&lb[2 * e + 1], tag | ((uint64_t)len << 24) | ((uint64_t)last8 << 16) | R);
  }
  if (X.abort) return;
  const uint64_t P = X.P;
  const uint64_t E = P + len;
  // 4. the bytes fully inside [P, E): dwords where whole, bytes at the two edges
  uint8_t* out = a.out;
  auto bits32 = [&](uint64_t bo) -> uint32_t {  // blob bits [bo, bo + 32), bo >= 0
    const uint32_t wi = (uint32_t)(bo >> 5), sh = (uint32_t)(bo & 31);
    return sh ? __builtin_amdgcn_alignbit(buf[wi], buf[wi + 1], 32 - sh) : buf[wi];
  };
  const uint64_t b0 = (P + 7) >> 3, b1 = E >> 3;  // full bytes
  const uint64_t d0 = (b0 + 3) >> 2, d1 = b1 >> 2;  // full dwords
  uint32_t* out32 = reinterpret_cast<uint32_t*>(out);
  if (d1 > d0) {
    for (uint64_t d = d0 + (uint64_t)t; d < d1; d += kThreads) out32[d] = __builtin_bswap32(bits32(32 * d - P));
  }
  {
    // edge bytes: [b0, min(4 d0, b1)) and [max(4 d1, b0), b1) (all of [b0, b1) when no whole dword)
    const uint64_t h1 = d1 > d0 ? 4 * d0 : b1;
    const uint64_t t0b = d1 > d0 ? 4 * d1 : b1;
    const int nh = (int)(h1 - b0), nt = (int)(b1 - t0b);
    if (t < nh) out[b0 + t] = (uint8_t)(bits32(8 * (b0 + t) - P) >> 24);
    else if (t >= 8 && t < 8 + nt) out[t0b + (t - 8)] = (uint8_t)(bits32(8 * (t0b + (t - 8)) - P) >> 24);
  }
  const uint32_t r = (uint32_t)(P & 7);
  if (t == 16 && r) {  // the byte shared with the predecessor (same frame: c > 0)
    uint64_t v;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    do {
      v = lb_load(&lb[2 * (e - 1) + 1]);
      if ((v >> 48) != epoch) __builtin_amdgcn_s_sleep(1);
    } while ((v >> 48) != epoch && __builtin_amdgcn_s_memrealtime() - t0 < tmo);
    const uint32_t pl = (uint32_t)(v >> 16) & 0xFFu;
    out[P >> 3] = (uint8_t)(((pl & ((1u << r) - 1u)) << (8 - r)) | (buf[0] >> (24 + r)));
  }
  if (c == 0 && t >= 32 && t < 48) {  // frame header (P is byte-aligned: whole header bytes before it)
    const int hb = (int)dw->hbytes[g], i = t - 32;
    if (i < hb) out[(P >> 3) - (uint64_t)hb + i] = (uint8_t)(dw->hdr[4 * (size_t)g + (i >> 2)] >> (24 - 8 * (i & 3)));
  }
  if (c == C - 1 && wv == 1) {
    // frame CRC-16: lanes 0..C-1 the subframes (residue, bits), lane C the header
    const int hb = (int)dw->hbytes[g];
    uint32_t bl = 0, rs = 0;
    if (lane < C - 1) {
      uint64_t v;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      do {
        v = lb_load(&lb[2 * (e - (C - 1) + lane) + 1]);
        if ((v >> 48) != epoch) __builtin_amdgcn_s_sleep(1);
      } while ((v >> 48) != epoch && __builtin_amdgcn_s_memrealtime() - t0 < tmo);
      bl = (uint32_t)(v >> 24) & 0xFFFFFFu;
      rs = (uint32_t)v & 0xFFFFu;
    } else if (lane == C - 1) {
      bl = len;
      rs = R;
    } else if (lane == C) {
      for (int i = 0; i < hb; i++) {
        const uint32_t by = (dw->hdr[4 * (size_t)g + (i >> 2)] >> (24 - 8 * (i & 3))) & 0xFFu;
        rs = ((rs << 8) & 0xFFFFu) ^ (uint32_t)X.T[((rs >> 8) ^ by) & 0xFFu];
      }
    }
    const uint32_t incl = wave_incl_scan32(lane < C ? bl : 0u);
    const uint32_t S = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t pad = (8u - (S & 7u)) & 7u;
    const uint32_t after = lane < C ? S - incl + pad : S + pad;
    const uint32_t term = lane <= C ? gf16_mul_t(rs, a.crctab[kXpowOff + xexp(after)], X.T) : 0u;
    const uint32_t crc16 = wave_xor32(term);
    if (lane == 0) {
      const uint64_t fs = ((P - (S - len)) >> 3) - (uint64_t)hb;  // frame start byte
      const uint64_t eb = (E + 7) >> 3;
      if (E & 7) out[E >> 3] = (uint8_t)(bits32(8 * (E >> 3) - P) >> 24);  // zero-padded tail byte
      out[eb] = (uint8_t)(crc16 >> 8);
      out[eb + 1] = (uint8_t)crc16;
      a.frame_off[g] = fs;
      a.frame_bytes[g] = eb + 2 - fs;
      if (tr) tr[3] = __builtin_amdgcn_s_memrealtime();
      if (li == (int)gridDim.x - 1) {  // the launch's end: next launch's base, host mirror, plan total
        dw->gbase[grp + 1] = eb + 2;
        if (last_grp) a.frame_off[a.nframes_total] = eb + 2;
        if (dw->host_mirror) {
          dw->host_mirror[grp + 1] = eb + 2;
          __threadfence_system();
        }
      }
    }
  }
}

}  // namespace fra
