// fra_assemble.h -- frame assembly + CRC-16 of one frame by one wave (device code) for k_assemble4
// (fra_pack.hip).
//
// Emits what libFLAC's frame writer emits for every 4,096-sample block that
// FLAC__stream_encoder_process_interleaved / _finish produce under the pyflac calls at
// src/flac_raster/converter.py:153-154 and src/flac_raster/spatial_encoder.py:303-304:
// frame header (RFC 9639 9.1, CRC-8) ++ subframes (9.2, encoded by k_analyze into per-subframe
// slots) ++ zero pad to a byte ++ CRC-16.
//
// Gather formulation: every thread builds whole output quads (4 dwords, 16-byte aligned in the
// output).  Global dword G0+k (G0 = (F-A)/4, A = F & 3) holds frame bits [8(4k-A), +32): the header
// and the channel blobs are laid end to end at known bit offsets (k_frame_scan), so a quad that lies
// inside one blob is a funnel shift (one shift for all four) of 5 consecutive slot words: one 16-byte
// load + one dword load + one 16-byte store.  Quads touching the header, a blob boundary or the frame
// ends resolve dword by dword; the first/last dwords (shared with the neighbouring frames) get byte
// stores.
//
// CRC-16 (poly x^16+x^15+x^2+1, init 0) on the same dwords, no extra pass.  Virtual dword v = k + a4
// (a4 = G0 mod 4, so quads in v are the aligned output quads); virtual quad u = v/4 + pad, pad making
// the last quad that holds CRC bytes land on thread 255.  Thread t folds the quads u == t (mod 256) by
// Horner (acc = acc * x^(128*256) ^ crc16(quad), slice-by-16 tables): leading zeros (the pad and the A
// bytes before F read as zero) leave a zero-initialised CRC unchanged; the e < 4 zero dwords after the
// last whole CRC dword are removed by multiplying with x^(-32e).  The 256 accumulators are combined by
// a DPP upper-lane tree (x^(128*2^l)), then the < 4 tail bytes byte-wise.
#pragma once
#include <algorithm>
#include <type_traits>

#include "fra_device.h"

namespace fra {
#ifdef FRA_GUARD
__device__ int g_guard_count;
#define GUARD(cond, ...) do { if (!(cond)) { if (atomicAdd(&g_guard_count, 1) < 40) printf(__VA_ARGS__); } } while (0)
#else
#define GUARD(cond, ...) do {} while (0)
#endif

constexpr int kMLo = 4, kMLevels = 7;  // LDS copy of multiply tables x^(8*2^i), i = 4..10

// multiply a CRC-16 remainder by the constant of table m (512 entries): two byte-table lookups
__device__ __forceinline__ uint32_t crc_mul_tab(const uint16_t* m, uint32_t c) {
  return (uint32_t)m[c & 0xFF] ^ (uint32_t)m[256 + (c >> 8)];
}
// multiply by x^(8*2^i) mod P; M = the tables of levels kMLo.. (LDS copy, or crctab in global memory)
__device__ __forceinline__ uint32_t crc_mul(const uint16_t* M, int i, uint32_t c) {
  return crc_mul_tab(M + (size_t)(i - kMLo) * 512, c);
}

// a * b mod P (bit-serial; one call per frame)
__device__ __forceinline__ uint32_t gf16_mul_dev(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int i = 15; i >= 0; i--) {
    r <<= 1;
    if (r & 0x10000u) r ^= 0x18005u;
    if ((b >> i) & 1u) r ^= a;
  }
  return r & 0xFFFFu;
}

// FRA_ASM_LIGHT (r05 default): only the Horner level's multiply table in LDS (the per-frame tree's six levels read
// from the global table, 6 lookups per frame): 9.3 instead of 15.6 KiB per workgroup, so three workgroups fit the
// 32 KiB a 4-wave k_analyze_w leaves per CU instead of two (with one quad per lane per round, fra_pack.hip)
#ifndef FRA_ASM_LIGHT
#define FRA_ASM_LIGHT 1
#endif
constexpr int kMLds = FRA_ASM_LIGHT ? 1 : kMLevels;  // LDS multiply tables: levels 10 - kMLds + 1 .. 10
struct alignas(16) AssembleSmem {
  uint16_t T[16][256];  // slice-by-16: T[k][v] = CRC of v followed by k zero bytes
  uint16_t M[kMLds][512];  // multiply by x^(8*2^i), i = 4..10 (tree 4..9, Horner 10), or only 10
  uint32_t meta[4][kMetaWords];  // the frame's header words and blob bit bounds (k_frame_scan); [wave]
  uint32_t tailw[4];    // the output window of the last, partial dword (bytes [4*NF - A, L)); [wave]
};

// `take` (1..32) bits at bit b of a big-endian word array, right-aligned
__device__ __forceinline__ uint32_t bits_at(const uint32_t* w, uint32_t b, int take) {
  const uint64_t X = ((uint64_t)w[b >> 5] << 32) | w[(b >> 5) + 1];
  return (uint32_t)((X << (b & 31)) >> (64 - take));
}

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (32 - sh));
}

// CRC tables to LDS (16-byte loads) so no step of the CRC chain waits on a global gather
__device__ __forceinline__ void copy_tables(const JobArgs& a, AssembleSmem& S) {
  const uint4* srcT = reinterpret_cast<const uint4*>(a.crctab + kCrcT16Off);
  const uint4* srcM = reinterpret_cast<const uint4*>(a.crctab + 1024 + (kMLo + kMLevels - kMLds) * 512);
  uint4* dT = reinterpret_cast<uint4*>(&S.T[0][0]);
  uint4* dM = reinterpret_cast<uint4*>(&S.M[0][0]);
  constexpr int NTV = 16 * 256 * 2 / 16, NMV = kMLds * 512 * 2 / 16;  // uint4 counts
  for (int i = (int)threadIdx.x; i < NTV + NMV; i += kThreads) {
    if (i < NTV) dT[i] = srcT[i];
    else dM[i - NTV] = srcM[i - NTV];
  }
}

// one frame by one wave (four frames per workgroup, no workgroup barrier per frame, the CRC tables copied
// to LDS once for the four by the caller), U quads per lane per round.  Header and blob bounds come
// precomputed by k_frame_scan, so every metadata load is issued in the first round
template <int U>
__device__ __forceinline__ void assemble_frame(const JobArgs& a, const int g, AssembleSmem& S) {
  constexpr int NT = 64;  // lanes per frame
  const int lane = (int)threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int t = lane;
  uint32_t* const meta = S.meta[wv];
  uint32_t& tailw = S.tailw[wv];
  // tree levels kMLo..9 (LDS, or the global table: FRA_ASM_LIGHT) and the Horner level x^(128 NT) = x^(8 * 2^10)
  const uint16_t* const M = FRA_ASM_LIGHT ? a.crctab + 1024 + kMLo * 512 : &S.M[0][0];
  const uint16_t* const Mh = &S.M[kMLds - 1][0];
  const uint32_t* gmeta = a.fmeta + (size_t)g * kMetaWords;  // uniform
  auto rfl64 = [](uint64_t v) -> uint64_t {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);  // (readfirstlane is int: no sign extension)
  };
  const uint64_t F = rfl64(a.frame_off[g]);
  const uint64_t L = rfl64(a.frame_bytes[g]) - 2;  // = ceil(TB / 8): bytes covered by the CRC-16
  const int C = __builtin_amdgcn_readfirstlane(a.streams[a.frames[g].stream].channels);
  uint32_t sg[kMaxChannels + 2];  // wave-uniform blob boundaries (bits)
#pragma unroll
  for (int i = 0; i < kMaxChannels + 2; i++) sg[i] = __builtin_amdgcn_readfirstlane(gmeta[kHdrWords + i]);
  const uint32_t* hdrw = meta;
  const uint32_t* seg = meta + kHdrWords;
  uint32_t TB = sg[1];                          // frame bits before the byte pad: sg[C + 1]
#pragma unroll
  for (int i = 2; i < kMaxChannels + 2; i++) TB = (i == C + 1) ? sg[i] : TB;  // (no dynamic index: no scratch)
  const uint32_t A = (uint32_t)(F & 3);
  uint32_t* gw = (uint32_t*)(a.out + (F - A));  // dword k of this frame's span
  const int ND = (int)((F + L - 1) >> 2) - (int)(F >> 2) + 1;  // dwords touching the frame
  const int NF = (int)((F + L) >> 2) - (int)(F >> 2);          // dwords ending inside it
  const int a4 = (int)(((F - A) >> 2) & 3);
  const int NQ = (NF + a4 + 3) >> 2;       // quads holding CRC dwords
  const int NQW = (ND + a4 + 3) >> 2;      // quads holding output dwords (NQ or NQ + 1)
  const int pad = (int)((NT - (NQ % NT)) % NT);
  const int kfull = A == 0 ? 0 : 1;        // first dword written whole
  const uint32_t* slots = a.tmp + (size_t)g * a.cmax * a.tmp_stride;
  // slot of output channels 0 / 1 (k_frame_scan: identity unless a mid-side assignment was chosen)
  const uint32_t smap = C == 2 ? (uint32_t)__builtin_amdgcn_readfirstlane(gmeta[kHdrWords - 1]) : 0u;
  auto vslot = [&](int oc) -> int { return C == 2 ? (int)((smap >> (8 * oc)) & 0xFFu) : oc; };
  {  // a frame whose sizes would leave the output or its slots (only a corrupt descriptor can) is not written
    bool inb = F + L + 2 <= a.out_cap && C >= 1 && C <= kMaxChannels;
#pragma unroll
    for (int i = 0; i < kMaxChannels; i++)
      inb = inb && (i >= C || sg[i + 2] - sg[i + 1] <= 32u * (uint32_t)a.tmp_stride);
    if (!inb) {
      if (t == 0 && a.err) atomicOr(a.err, 2u);
      return;
    }
  }
#ifdef FRA_GUARD
  const uint64_t TOT = a.out_cap;  // frame_off[nframes_total] is final only after the last frame group
  const uint64_t SLOTW = (uint64_t)a.nframes_total * a.cmax * a.tmp_stride;
  {
    const FrameDev frg = a.frames[g];
    const StreamDev stg = a.streams[frg.stream];
    const uint64_t cap = 18 + (uint64_t)C * ((uint64_t)frg.n * stg.bps / 8 + 8);
    if (t == 0) GUARD(L + 2 <= cap, "g %d frame bytes %llu > cap %llu (n %d bps %d C %d) bits %u %u %u %u %u %u %u %u\n", g,
                      (unsigned long long)(L + 2), (unsigned long long)cap, frg.n, stg.bps, C, sg[2] - sg[1], sg[3] - sg[2],
                      sg[4] - sg[3], sg[5] - sg[4], sg[6] - sg[5], sg[7] - sg[6], sg[8] - sg[7], sg[9] - sg[8]);
    const bool ok = (TB + 7) / 8 == L && F + L + 2 <= TOT && F + L + 2 <= a.out_cap && L + 2 <= cap && C >= 1 && C <= kMaxChannels;
    if (t == 0) GUARD(ok, "g %d TB %u L %llu F %llu TOT %llu cap %llu C %d sg %u %u %u %u\n", g, TB, (unsigned long long)L,
                      (unsigned long long)F, (unsigned long long)TOT, (unsigned long long)a.out_cap, C, sg[0], sg[1], sg[2], sg[C + 1]);
    if (!ok) return;
  }
#endif

  // 32 frame bits starting at (possibly negative) bit position bp; bits outside [0, TB) read 0
  auto window = [&](int bp) -> uint32_t {
    uint32_t res = 0;
    int filled = 0;
    if (bp < 0) {
      filled = (int)min<int>(32, -bp);
      bp = 0;
    }
    int s = 0;
    while (filled < 32 && bp < (int)TB) {
      while ((int)seg[s + 1] <= bp) s++;
      const uint32_t take = (uint32_t)min<int>(32 - filled, (int)seg[s + 1] - bp);
      const uint32_t rel = (uint32_t)(bp - seg[s]);
      const uint32_t v =
          s == 0 ? bits_at(hdrw, rel, (int)take) : bits_at(slots + (size_t)vslot(s - 1) * a.tmp_stride, rel, (int)take);
      res |= take == 32 ? v : (v << (32 - filled - (int)take));
      filled += (int)take;
      bp += take;
    }
    return res;
  };

  uint32_t acc = 0;
  int q0 = (int)t - pad;  // quad index in v/4 space
  if (q0 < 0) q0 += NT;
  // slot gather of the U quads of round q0 (fast case: one 16-byte + one dword load, shift later)
  // sh[u] = the funnel shift of a fast quad, kSlow (no single-blob window: the dword-wise path)
  constexpr uint32_t kSlow = 0xFFFFFFFFu;
  auto fetch = [&](const int qr, uint32_t (&w)[U][5], uint32_t (&sh)[U]) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int k = 4 * (qr + (int)u * NT) - a4;  // first dword of the quad
      const int bp = 8 * (4 * k - (int)A);
      sh[u] = kSlow;
#pragma unroll
      for (int i = 0; i < 5; i++) w[u][i] = 0;
      if (qr + (int)u * NT < NQW && k >= 0 && k + 4 <= ND && bp >= (int)sg[1] && bp + 128 <= (int)TB) {
        const uint32_t b = (uint32_t)bp;
        // blob sgi - 1 holds bit b: lo = sg[sgi] <= b < hi = sg[sgi + 1] (b < TB: never past blob C - 1);
        // a select chain, not a dynamically indexed array (which would live in scratch)
        int sgi = 1;
        uint32_t lo = sg[1], hi = sg[2];
#pragma unroll
        for (int i = 2; i <= kMaxChannels; i++) {
          const bool ge = b >= sg[i];
          sgi += ge ? 1 : 0;
          lo = ge ? sg[i] : lo;
          hi = ge ? sg[i + 1] : hi;
        }
        if (b + 128 <= hi) {
          const uint32_t rel = b - lo;
          // uniform base + 32-bit byte offset (saddr addressing: no 64-bit address pair per lane)
          const uint32_t soff = ((uint32_t)vslot(sgi - 1) * (uint32_t)a.tmp_stride + (rel >> 5)) * 4u;
          const uint32_t* src = (const uint32_t*)((const char*)slots + soff);
          GUARD((uint64_t)(src + 4 - a.tmp) < SLOTW && sgi - 1 < C, "g %d slot read sgi %d rel %u\n", g, sgi, rel);
          uint4 v4;
          __builtin_memcpy(&v4, src, 16);
          w[u][0] = v4.x;
          w[u][1] = v4.y;
          w[u][2] = v4.z;
          w[u][3] = v4.w;
          w[u][4] = src[4];
          sh[u] = rel & 31;
        }
      }
    }
  };
  uint32_t wn[U][5], shn[U];
  if (q0 < NQW) fetch(q0, wn, shn);
  // header words to LDS while the first slot loads are in flight
  if (t < kMetaWords) meta[t] = a.fmeta[(size_t)g * kMetaWords + t];
  // this wave's LDS stores -> its own reads
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  for (; q0 < NQW; q0 += NT * U) {
    uint32_t w[U][5], sh[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      sh[u] = shn[u];
#pragma unroll
      for (int i = 0; i < 5; i++) w[u][i] = wn[u][i];
    }
    // next round's loads are in flight while this round is shifted, stored and CRC'd
    if (q0 + NT * U < NQW) fetch(q0 + NT * U, wn, shn);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int q = q0 + (int)u * NT;
      if (q >= NQW) break;
      const int k = 4 * q - a4;
      uint32_t val[4];
      if (sh[u] != kSlow) {
#pragma unroll
        for (int i = 0; i < 4; i++) val[i] = funnel(w[u][i], w[u][i + 1], sh[u]);
      } else {  // (rare) quads at a blob boundary or a frame end: one dword at a time, one copy of window()
#pragma unroll
        for (int i = 0; i < 4; i++) val[i] = 0u;
#pragma nounroll
        for (int i = 0; i < 4; i++) {
          const uint32_t v = (k + i >= 0 && k + i < ND) ? window(8 * (4 * (k + i) - (int)A)) : 0u;
#pragma unroll
          for (int j = 0; j < 4; j++) val[j] = i == j ? v : val[j];
        }
      }
      if (k >= kfull && k + 4 <= NF) {
        uint4 o;
        o.x = __builtin_bswap32(val[0]);
        o.y = __builtin_bswap32(val[1]);
        o.z = __builtin_bswap32(val[2]);
        o.w = __builtin_bswap32(val[3]);
        GUARD(F - A + 4 * k + 16 <= TOT, "g %d quad store k %lld\n", g, (long long)k);
        *reinterpret_cast<uint4*>((char*)gw + 4u * (uint32_t)k) = o;
      } else {
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int kk = k + i;
          if (kk < 0 || kk >= ND) continue;
          if (kk >= kfull && kk < NF) {
            gw[kk] = __builtin_bswap32(val[i]);
          } else {
            for (int b = 0; b < 4; b++) {
              const int fb = 4 * kk - (int)A + b;  // frame byte index
              if (fb >= 0 && fb < (int)L) a.out[F + fb] = (uint8_t)(val[i] >> (24 - 8 * b));
            }
          }
          if (kk == NF) tailw = val[i];
          if (kk >= NF) val[i] = 0;  // trailing zeros in the CRC (removed below)
        }
      }
      if (q < NQ) {
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          c ^= (uint32_t)S.T[15 - 4 * i][val[i] >> 24] ^ (uint32_t)S.T[14 - 4 * i][(val[i] >> 16) & 0xFF] ^
               (uint32_t)S.T[13 - 4 * i][(val[i] >> 8) & 0xFF] ^ (uint32_t)S.T[12 - 4 * i][val[i] & 0xFF];
        }
        acc = crc_mul_tab(Mh, acc) ^ c;  // Horner step: x^(128 NT)
      }
    }
  }
  // combine: lane order == virtual quad order; left groups are multiplied by x^(128*2^l)
  acc ^= crc_mul(M, 4, dpp32<DPP_SHR1, 0xF>(acc));
  acc ^= crc_mul(M, 5, dpp32<DPP_SHR2, 0xF>(acc));
  acc ^= crc_mul(M, 6, dpp32<DPP_SHR4, 0xF>(acc));
  acc ^= crc_mul(M, 7, dpp32<DPP_SHR8, 0xF>(acc));
  acc ^= crc_mul(M, 8, dpp32<DPP_BC15, 0xA>(acc));
  acc ^= crc_mul(M, 9, dpp32<DPP_BC31, 0xC>(acc));
  // the wave's accumulators are the frame's: lane 63 holds the CRC
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // tailw (any lane) -> lane 63
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_wave_barrier();
  uint32_t crc = acc;
  if (lane == 63) {
    // remove the e zero dwords that followed dword NF-1 inside the last CRC quad: * x^(-32e)
    const int e = (int)(4 * NQ - (NF + a4));
    constexpr uint32_t kInvX32[4] = {0x0001u, 0xCAA8u, 0x25DDu, 0x37B1u};  // x^(-32e) mod P
    if (e) crc = gf16_mul_dev(crc, kInvX32[e]);
    // tail: frame bytes [4*NF - A, L) not covered by whole dwords
    const int tb0 = 4 * NF - (int)A;
    if (tb0 < (int)L) {
      const uint32_t val = tailw;
      for (int fb = tb0; fb < (int)L; fb++) {
        const uint32_t by = (val >> (24 - 8 * (int)(fb - tb0))) & 0xFF;
        crc = ((crc << 8) ^ S.T[0][((crc >> 8) ^ by) & 0xFF]) & 0xFFFF;
      }
    }
    a.out[F + L] = (uint8_t)(crc >> 8);
    a.out[F + L + 1] = (uint8_t)crc;
  }
}

}  // namespace fra
