// fra_pack.hip -- k_assemble: frame assembly + CRC-16 (one workgroup per frame).
//
// Emits what libFLAC's frame writer emits for every 4,096-sample block that
// FLAC__stream_encoder_process_interleaved / _finish produce under the pyflac calls at
// src/flac_raster/converter.py:153-154 and src/flac_raster/spatial_encoder.py:303-304:
// frame header (RFC 9639 9.1, CRC-8) ++ subframes (9.2, encoded by k_analyze into per-subframe
// slots) ++ zero pad to a byte ++ CRC-16.
//
// Gather formulation: every thread builds whole output dwords.  Global dword G0+k (G0 = F>>2)
// holds frame bits [8(4k-A), +32) (A = F & 3): the header and the channel blobs are laid end to end
// at known bit offsets, so each 32-bit window is a funnel-shifted read from at most a few segments.
// Dwords entirely inside the frame are written with one aligned store; the first/last dwords
// (shared with the neighbouring frames) get byte stores.
//
// CRC-16 (poly x^16+x^15+x^2+1, init 0) on the same dwords, no extra pass: thread t folds the dwords
// with virtual index v = k + pad == t (mod 256) by Horner (acc = acc * x^(32*256) ^ crc4(dword)); the
// front pad (and the A bytes before F, which read as zero) are leading zeros, which leave a
// zero-initialised CRC unchanged.  The 256 accumulators are combined by a DPP upper-lane tree
// (x^(32*2^l) multipliers, host-precomputed byte tables), then the < 4 tail bytes byte-wise.
#include <algorithm>

#include "fra_device.h"

namespace fra {

// multiply a CRC-16 remainder by x^(8*2^i) mod P: two byte-table lookups (M = the LDS copy of levels
// 2..10 of the host tables, i.e. M + (i - 2) * 512)
__device__ __forceinline__ uint32_t crc_mul(const uint16_t* M, int i, uint32_t c) {
  const uint16_t* m = M + (size_t)(i - 2) * 512;
  return (uint32_t)m[c & 0xFF] ^ (uint32_t)m[256 + (c >> 8)];
}

struct alignas(16) AssembleSmem {
  uint16_t T[4][256];   // slice-by-4: T[k][v] = CRC of v followed by k zero bytes
  uint16_t M[9][512];   // multiply by x^(8*2^i), i = 2..10 (combine steps; i = 10 = x^(32*256): Horner)
  uint32_t meta[kMetaWords];  // this frame's header words and blob bit bounds (k_frame_bytes)
  uint32_t crcw[4];
  uint32_t tailw;       // the output window of the last, partial dword (bytes [4*NF - A, L))
};

// `take` (1..32) bits at bit b of a big-endian word array, right-aligned
__device__ __forceinline__ uint32_t bits_at(const uint32_t* w, uint32_t b, int take) {
  const uint64_t X = ((uint64_t)w[b >> 5] << 32) | w[(b >> 5) + 1];
  return (uint32_t)((X << (b & 31)) >> (64 - take));
}

// one workgroup per frame; the CRC tables (slice-by-4, the combine multipliers) are copied to LDS up
// front (16-byte loads) so no step of the CRC chain waits on a global gather.  Header and blob bounds
// come precomputed from k_frame_bytes, so every metadata load is issued in the first round.
__global__ void __launch_bounds__(kThreads, 8) k_assemble(JobArgs a) {
  __shared__ AssembleSmem S;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int g = blockIdx.x;
  {
    const uint4* srcT = reinterpret_cast<const uint4*>(a.crctab);
    const uint4* srcM = reinterpret_cast<const uint4*>(a.crctab + 1024 + 2 * 512);
    uint4* dT = reinterpret_cast<uint4*>(&S.T[0][0]);
    uint4* dM = reinterpret_cast<uint4*>(&S.M[0][0]);
    constexpr int NT = 1024 * 2 / 16, NM = 9 * 512 * 2 / 16;
    for (int i = t; i < NT + NM; i += kThreads) {
      if (i < NT) dT[i] = srcT[i];
      else dM[i - NT] = srcM[i - NT];
    }
    if (t < kMetaWords) S.meta[t] = a.fmeta[(size_t)g * kMetaWords + t];
  }
  const uint16_t* M = &S.M[0][0];
  const uint32_t* gmeta = a.fmeta + (size_t)g * kMetaWords;  // uniform: scalar loads
  auto rfl64 = [](uint64_t v) -> uint64_t {
    return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
           __builtin_amdgcn_readfirstlane((uint32_t)v);
  };
  const uint64_t F = rfl64(a.frame_off[g]);
  const uint64_t L = rfl64(a.frame_bytes[g]) - 2;  // = ceil(TB / 8): bytes covered by the CRC-16
  const int C = __builtin_amdgcn_readfirstlane(a.streams[a.frames[g].stream].channels);
  __syncthreads();
  const uint32_t* hdrw = S.meta;
  const uint32_t* seg = S.meta + kHdrWords;
  const uint32_t TB = seg[C + 1];               // frame bits before the byte pad
  const uint32_t A = (uint32_t)(F & 3);
  uint32_t* gw = (uint32_t*)(a.out + (F - A));  // dword k of this frame's span
  const int64_t ND = (int64_t)((F + L - 1) >> 2) - (int64_t)(F >> 2) + 1;  // dwords touching the frame
  const int64_t NF = (int64_t)((F + L) >> 2) - (int64_t)(F >> 2);          // dwords ending inside it
  const int pad = (int)((kThreads - (NF % kThreads)) % kThreads);
  const uint32_t* slots = a.tmp + (size_t)g * a.cmax * a.tmp_stride;

  // 32 frame bits starting at (possibly negative) bit position bp; bits outside [0, TB) read 0
  auto window = [&](int64_t bp) -> uint32_t {
    uint32_t res = 0;
    int filled = 0;
    if (bp < 0) {
      filled = (int)min<int64_t>(32, -bp);
      bp = 0;
    }
    int s = 0;
    while (filled < 32 && bp < (int64_t)TB) {
      while ((int64_t)seg[s + 1] <= bp) s++;
      const uint32_t take = (uint32_t)min<int64_t>(32 - filled, (int64_t)seg[s + 1] - bp);
      const uint32_t rel = (uint32_t)(bp - seg[s]);
      const uint32_t v =
          s == 0 ? bits_at(hdrw, rel, (int)take) : bits_at(slots + (size_t)(s - 1) * a.tmp_stride, rel, (int)take);
      res |= take == 32 ? v : (v << (32 - filled - (int)take));
      filled += (int)take;
      bp += take;
    }
    return res;
  };

  // Fast gather: a dword whose 32 bits lie inside ONE channel blob is a funnel shift of two adjacent
  // slot words.  U dwords per thread are resolved and their loads issued together (latency overlap);
  // dwords touching the header, a blob boundary or the frame ends take window() (a few per frame).
  constexpr int U = 4;
  uint32_t sg[kMaxChannels + 2];  // wave-uniform blob boundaries (bits)
#pragma unroll
  for (int i = 0; i < kMaxChannels + 2; i++) sg[i] = __builtin_amdgcn_readfirstlane(gmeta[kHdrWords + i]);
  uint32_t acc = 0;
  int64_t k0 = (int64_t)t - pad;
  if (k0 < 0) k0 += kThreads;
  for (; k0 < ND; k0 += (int64_t)kThreads * U) {
    uint32_t w0[U], w1[U], sh[U];
    bool fast[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t k = k0 + (int64_t)u * kThreads;
      const int64_t bp = 8 * (4 * k - (int64_t)A);
      fast[u] = false;
      w0[u] = w1[u] = sh[u] = 0;
      if (k < ND && bp >= (int64_t)sg[1] && bp + 32 <= (int64_t)TB) {
        const uint32_t b = (uint32_t)bp;
        int sgi = 1;  // blob sgi - 1 holds bit b: sg[sgi] <= b < sg[sgi + 1]
#pragma unroll
        for (int i = 2; i <= kMaxChannels + 1; i++) sgi += (b >= sg[i]) ? 1 : 0;
        if (b + 32 <= sg[sgi + 1]) {
          const uint32_t rel = b - sg[sgi];
          const uint32_t* src = slots + (size_t)(sgi - 1) * a.tmp_stride + (rel >> 5);
          w0[u] = src[0];
          w1[u] = src[1];
          sh[u] = rel & 31;
          fast[u] = true;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t k = k0 + (int64_t)u * kThreads;
      if (k >= ND) break;
      const uint32_t val = fast[u] ? (uint32_t)((((uint64_t)w0[u] << 32) | w1[u]) >> (32 - sh[u]))
                                   : window(8 * (4 * k - (int64_t)A));
      if ((k > 0 || A == 0) && k < NF) {
        gw[k] = __builtin_bswap32(val);
      } else {
        for (int b = 0; b < 4; b++) {
          const int64_t fb = 4 * k - (int64_t)A + b;  // frame byte index
          if (fb >= 0 && fb < (int64_t)L) a.out[F + fb] = (uint8_t)(val >> (24 - 8 * b));
        }
      }
      if (k == NF) S.tailw = val;
      if (k < NF) {
        const uint32_t c4 = (uint32_t)S.T[3][val >> 24] ^ (uint32_t)S.T[2][(val >> 16) & 0xFF] ^
                            (uint32_t)S.T[1][(val >> 8) & 0xFF] ^ (uint32_t)S.T[0][val & 0xFF];
        acc = crc_mul(M, 10, acc) ^ c4;  // Horner step: x^(32*256)
      }
    }
  }
  // combine: lane order == virtual dword order; left groups are multiplied by x^(32*2^l)
  acc ^= crc_mul(M, 2, dpp32<DPP_SHR1, 0xF>(acc));
  acc ^= crc_mul(M, 3, dpp32<DPP_SHR2, 0xF>(acc));
  acc ^= crc_mul(M, 4, dpp32<DPP_SHR4, 0xF>(acc));
  acc ^= crc_mul(M, 5, dpp32<DPP_SHR8, 0xF>(acc));
  acc ^= crc_mul(M, 6, dpp32<DPP_BC15, 0xA>(acc));
  acc ^= crc_mul(M, 7, dpp32<DPP_BC31, 0xC>(acc));
  if (lane == 63) S.crcw[wv] = acc;
  __syncthreads();
  if (t == 0) {
    const uint32_t c01 = crc_mul(M, 8, S.crcw[0]) ^ S.crcw[1];
    const uint32_t c23 = crc_mul(M, 8, S.crcw[2]) ^ S.crcw[3];
    uint32_t crc = crc_mul(M, 9, c01) ^ c23;
    // tail: frame bytes [4*NF - A, L) not covered by whole dwords
    const int64_t tb0 = 4 * NF - (int64_t)A;
    if (tb0 < (int64_t)L) {
      const uint32_t val = S.tailw;
      for (int64_t fb = tb0; fb < (int64_t)L; fb++) {
        const uint32_t by = (val >> (24 - 8 * (int)(fb - tb0))) & 0xFF;
        crc = ((crc << 8) ^ S.T[0][((crc >> 8) ^ by) & 0xFF]) & 0xFFFF;
      }
    }
    a.out[F + L] = (uint8_t)(crc >> 8);
    a.out[F + L + 1] = (uint8_t)crc;
  }
}

hipError_t launch_assemble(const JobArgs& a, hipStream_t s) {
  if (a.nframes_total > 0) k_assemble<<<(unsigned)a.nframes_total, kThreads, 0, s>>>(a);
  return hipGetLastError();
}

}  // namespace fra
