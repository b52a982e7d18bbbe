// fra_decode.cpp -- native FLAC decoder of the read side.
//
// Replaces pyflac.FileDecoder / libFLAC FLAC__stream_decoder_process_until_end_of_stream as used by
// RasterFLACConverter.flac_to_tiff (src/flac_raster/converter.py:179-183) and the tile extract path
// (cli.py:197-330); the PCM_16 / float64 semantics of that path (F8) are applied by the Python host
// (flac_raster/decoder.py), this file returns the exact integer samples.
//
// Host C++, frame-parallel: FLAC frames are self-delimiting only by decoding, so
//   pass 1 (threads over byte ranges): every sync candidate 0xFFF8/0xFFF9 whose header CRC-8 holds
//          is decoded speculatively without output; a candidate is a frame iff its subframes parse
//          and the CRC-16 at the byte after them holds -> (start, end, samples);
//   chain:  from the first audio byte follow start -> end through the candidate table (a false
//          candidate inside a frame is never reached); "fLaC" at a chain break starts the next
//          concatenated stream (spatial files, spatial_encoder.py:196-245) when allowed;
//   pass 2 (threads over chained frames): decode again into the output at the frame's sample
//          position.
// Every channel assignment (independent, L/S, S/R, M/S), wasted bits, CONSTANT, VERBATIM,
// FIXED 0-4, LPC 1-32, RICE/RICE2 with escapes, 4..32 bps.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/flac_raster_amd.h"

extern "C" int fra_internal_set_error(int code, const char* fmt, ...);

namespace {

uint8_t g_crc8[256];
uint16_t g_crc16[256];
struct CrcInit {
  CrcInit() {
    for (int v = 0; v < 256; v++) {
      uint32_t c = (uint32_t)v;
      for (int b = 0; b < 8; b++) c = (c & 0x80u) ? ((c << 1) ^ 0x07u) : (c << 1);
      g_crc8[v] = (uint8_t)c;
      uint32_t d = (uint32_t)v << 8;
      for (int b = 0; b < 8; b++) d = (d & 0x8000u) ? ((d << 1) ^ 0x8005u) : (d << 1);
      g_crc16[v] = (uint16_t)d;
    }
  }
} g_crc_init;

uint32_t crc16(const uint8_t* p, size_t n) {
  uint32_t c = 0;
  for (size_t i = 0; i < n; i++) c = ((c << 8) ^ g_crc16[((c >> 8) ^ p[i]) & 0xFF]) & 0xFFFF;
  return c;
}

// MSB-first bit reader; reads past `end` yield zeros and set `bad`
struct Bits {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t pos = 0;  // bit position from p
  uint64_t nbits;
  bool bad = false;
  Bits(const uint8_t* b, const uint8_t* e) : p(b), end(e), nbits((uint64_t)(e - b) * 8) {}
  inline uint64_t peek64() const {
    const uint64_t byte = pos >> 3;
    uint64_t w = 0;
    const uint64_t avail = (uint64_t)(end - p) - std::min<uint64_t>(byte, (uint64_t)(end - p));
    if (avail >= 8) {
      memcpy(&w, p + byte, 8);
      w = __builtin_bswap64(w);
    } else {
      for (uint64_t i = 0; i < 8; i++) w = (w << 8) | (i < avail ? p[byte + i] : 0u);
    }
    return w << (pos & 7);
  }
  inline uint32_t get(int n) {  // n <= 32
    if (n == 0) return 0;
    const uint32_t v = (uint32_t)(peek64() >> (64 - n));
    pos += (uint64_t)n;
    if (pos > nbits) bad = true;
    return v;
  }
  inline int32_t sget(int n) {
    if (n == 0) return 0;
    const uint32_t v = get(n);
    return n == 32 ? (int32_t)v : (int32_t)(v << (32 - n)) >> (32 - n);
  }
  inline int64_t sget_wide(int n) {  // n <= 33 (side channel of a 32-bps stream)
    if (n <= 32) return sget(n);
    const int64_t hi = sget(n - 32);
    return (int64_t)((uint64_t)hi << 32) | get(32);
  }
  inline uint32_t unary() {  // count of zeros before a one
    uint32_t z = 0;
    for (;;) {
      const uint64_t w = peek64();
      const int avail = 57;  // peek64 keeps at least 57 fresh bits after the shift
      if (w >> (64 - avail)) {
        const int lz = __builtin_clzll(w);
        pos += (uint64_t)lz + 1;
        z += (uint32_t)lz;
        break;
      }
      pos += (uint64_t)avail;
      z += (uint32_t)avail;
      if (pos > nbits) { bad = true; return z; }
    }
    if (pos > nbits) bad = true;
    return z;
  }
  void align() { pos = (pos + 7) & ~7ull; }
};

struct StreamParams {
  int sample_rate = 0, channels = 0, bps = 0, min_bs = 0, max_bs = 0;
  uint64_t total_samples = 0;
};

struct FrameHdr {
  int blocksize = 0, sample_rate = 0, chan_assign = 0, channels = 0, bps = 0;
  uint64_t number = 0;  // frame number (fixed) or first sample (variable)
  bool variable = false;
  int hdr_len = 0;
};

// RFC 9639 9.1; 0 values of sample rate / bps (code 0) take the STREAMINFO ones.
bool parse_header(const uint8_t* p, const uint8_t* end, const StreamParams& sp, FrameHdr& h) {
  if (end - p < 6) return false;
  if (p[0] != 0xFF || (p[1] & 0xFE) != 0xF8) return false;
  h.variable = p[1] & 1;
  const int bsc = p[2] >> 4, src = p[2] & 15, ca = p[3] >> 4, bpc = (p[3] >> 1) & 7;
  if ((p[3] & 1) || bsc == 0 || src == 15 || ca > 10 || bpc == 3) return false;
  const uint8_t* q = p + 4;
  // UTF-8-like coded number
  uint64_t v = *q++;
  int extra = 0;
  if (!(v & 0x80)) extra = 0;
  else if ((v & 0xE0) == 0xC0) { v &= 0x1F; extra = 1; }
  else if ((v & 0xF0) == 0xE0) { v &= 0x0F; extra = 2; }
  else if ((v & 0xF8) == 0xF0) { v &= 0x07; extra = 3; }
  else if ((v & 0xFC) == 0xF8) { v &= 0x03; extra = 4; }
  else if ((v & 0xFE) == 0xFC) { v &= 0x01; extra = 5; }
  else if (v == 0xFE) { v = 0; extra = 6; }
  else return false;
  if (!h.variable && extra > 5) return false;
  if (end - q < extra + 1) return false;
  for (int i = 0; i < extra; i++) {
    if ((*q & 0xC0) != 0x80) return false;
    v = (v << 6) | (*q++ & 0x3F);
  }
  h.number = v;
  if (bsc == 1) h.blocksize = 192;
  else if (bsc <= 5) h.blocksize = 576 << (bsc - 2);
  else if (bsc == 6) { if (end - q < 2) return false; h.blocksize = *q++ + 1; }
  else if (bsc == 7) { if (end - q < 3) return false; h.blocksize = ((q[0] << 8) | q[1]) + 1; q += 2; }
  else h.blocksize = 256 << (bsc - 8);
  static const int kRates[12] = {0, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000};
  if (src == 0) h.sample_rate = sp.sample_rate;
  else if (src < 12) h.sample_rate = kRates[src];
  else if (src == 12) { if (end - q < 2) return false; h.sample_rate = *q++ * 1000; }
  else if (src == 13) { if (end - q < 3) return false; h.sample_rate = (q[0] << 8) | q[1]; q += 2; }
  else { if (end - q < 3) return false; h.sample_rate = ((q[0] << 8) | q[1]) * 10; q += 2; }
  static const int kBps[8] = {0, 8, 12, 0, 16, 20, 24, 32};
  h.bps = bpc == 0 ? sp.bps : kBps[bpc];
  if (h.bps < 4 || h.bps > 32) return false;
  h.chan_assign = ca;
  h.channels = ca < 8 ? ca + 1 : 2;
  if (end - q < 1) return false;
  uint32_t c8 = 0;
  for (const uint8_t* r = p; r < q; r++) c8 = g_crc8[c8 ^ *r];
  if (c8 != *q) return false;
  h.hdr_len = (int)(q - p) + 1;
  return true;
}

// residual (RFC 9639 9.2.7) for a subframe of n samples with `order` warm-up samples
bool read_residual(Bits& br, int n, int order, int32_t* out, bool write) {
  const uint32_t method = br.get(2);
  if (method > 1) return false;
  const int pbits = method == 0 ? 4 : 5, esc = method == 0 ? 15 : 31;
  const int porder = (int)br.get(4);
  const int parts = 1 << porder;
  if ((n % parts) != 0) return false;
  const int psz = n / parts;
  if (psz < order) return false;
  int i = order;
  for (int pi = 0; pi < parts; pi++) {
    const int cnt = pi == 0 ? psz - order : psz;
    const uint32_t k = br.get(pbits);
    if ((int)k == esc) {
      const int w = (int)br.get(5);
      for (int j = 0; j < cnt; j++, i++) {
        const int32_t v = br.sget(w);
        if (write) out[i] = v;
      }
    } else {
      for (int j = 0; j < cnt; j++, i++) {
        const uint32_t q = br.unary();
        if (q > (1u << 28)) return false;
        const uint64_t u = ((uint64_t)q << k) | (k ? br.get((int)k) : 0u);
        const int64_t v = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
        if (v < INT32_MIN || v > INT32_MAX) return false;
        if (write) out[i] = (int32_t)v;
      }
    }
    if (br.bad) return false;
  }
  return true;
}

// decode one subframe into s[0..n) (int64 to hold the side channel of 32-bps streams)
bool read_subframe(Bits& br, int n, int bps, int64_t* s, std::vector<int32_t>& res, bool write) {
  if (br.get(1) != 0) return false;
  const int type = (int)br.get(6);
  int wasted = 0;
  if (br.get(1)) wasted = (int)br.unary() + 1;
  if (wasted >= bps) return false;
  const int eb = bps - wasted;
  // reconstructed samples must fit the subframe's sample width (libFLAC rejects such frames too);
  // keeping every s[] within eb <= 33 bits also bounds the predictor sums below 2^53: no int64 overflow
  const int64_t lo = -((int64_t)1 << (eb - 1)), hi = ((int64_t)1 << (eb - 1)) - 1;
  if (type == 0) {
    const int64_t v = br.sget_wide(eb);
    if (write) for (int i = 0; i < n; i++) s[i] = v;
  } else if (type == 1) {
    for (int i = 0; i < n; i++) {
      const int64_t v = br.sget_wide(eb);
      if (write) s[i] = v;
    }
  } else if (type >= 8 && type <= 12) {
    const int order = type - 8;
    if (order > n) return false;
    for (int i = 0; i < order; i++) {
      const int64_t v = br.sget_wide(eb);
      if (write) s[i] = v;
    }
    if ((int)res.size() < n) res.resize(n);
    if (!read_residual(br, n, order, res.data(), write)) return false;
    if (write) {
      for (int i = order; i < n; i++) {
        int64_t p = 0;
        switch (order) {
          case 1: p = s[i - 1]; break;
          case 2: p = 2 * s[i - 1] - s[i - 2]; break;
          case 3: p = 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3]; break;
          case 4: p = 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4]; break;
        }
        s[i] = p + res[i];
        if (s[i] < lo || s[i] > hi) return false;
      }
    }
  } else if (type >= 32) {
    const int order = type - 31;
    if (order > n) return false;
    for (int i = 0; i < order; i++) {
      const int64_t v = br.sget_wide(eb);
      if (write) s[i] = v;
    }
    const int prec = (int)br.get(4) + 1;
    if (prec == 16) return false;
    const int shift = br.sget(5);
    if (shift < 0) return false;
    int32_t coef[32];
    for (int j = 0; j < order; j++) coef[j] = br.sget(prec);
    if ((int)res.size() < n) res.resize(n);
    if (!read_residual(br, n, order, res.data(), write)) return false;
    if (write) {
      for (int i = order; i < n; i++) {
        int64_t acc = 0;
        for (int j = 0; j < order; j++) acc += (int64_t)coef[j] * s[i - 1 - j];
        s[i] = (acc >> shift) + res[i];
        if (s[i] < lo || s[i] > hi) return false;
      }
    }
  } else {
    return false;
  }
  if (br.bad) return false;
  if (write && wasted)
    for (int i = 0; i < n; i++) s[i] = (int64_t)((uint64_t)s[i] << wasted);
  return true;
}

struct Scratch {
  std::vector<int64_t> ch[8];
  std::vector<int32_t> res;
};

// decode the frame at p; returns its byte length (0 = not a frame).  out: interleaved int32 at the
// frame's first sample (nullptr: validate only).
size_t decode_frame(const uint8_t* p, const uint8_t* end, const StreamParams& sp, const FrameHdr& h, int32_t* out,
                    int out_channels, Scratch& sc) {
  Bits br(p + h.hdr_len, end);
  const int n = h.blocksize;
  const bool write = out != nullptr;
  for (int c = 0; c < h.channels; c++) {
    int bps = h.bps;
    if ((h.chan_assign == 8 && c == 1) || (h.chan_assign == 9 && c == 0) || (h.chan_assign == 10 && c == 1)) bps++;
    if (write && (int)sc.ch[c].size() < n) sc.ch[c].resize(n);
    if (!read_subframe(br, n, bps, write ? sc.ch[c].data() : nullptr, sc.res, write)) return 0;
  }
  br.align();
  const uint64_t body = br.pos >> 3;
  const size_t flen = (size_t)h.hdr_len + body + 2;
  if ((size_t)(end - p) < flen) return 0;
  const uint32_t crc = crc16(p, flen - 2);
  if (crc != (((uint32_t)p[flen - 2] << 8) | p[flen - 1])) return 0;
  (void)sp;
  if (write) {
    int64_t* a = sc.ch[0].data();
    int64_t* b = h.channels > 1 ? sc.ch[1].data() : nullptr;
    if (h.chan_assign == 8) for (int i = 0; i < n; i++) b[i] = a[i] - b[i];            // L/S
    else if (h.chan_assign == 9) for (int i = 0; i < n; i++) a[i] = a[i] + b[i];       // S/R
    else if (h.chan_assign == 10)                                                      // M/S
      for (int i = 0; i < n; i++) {
        const int64_t m = (a[i] * 2) | (b[i] & 1), sd = b[i];
        a[i] = (m + sd) >> 1;
        b[i] = (m - sd) >> 1;
      }
    for (int i = 0; i < n; i++)
      for (int c = 0; c < out_channels; c++) out[(size_t)i * out_channels + c] = (int32_t)sc.ch[c][i];
  }
  return flen;
}

// "fLaC" + metadata blocks; returns the offset of the first audio byte (0 on error)
size_t parse_metadata(const uint8_t* d, size_t len, size_t at, StreamParams& sp) {
  if (at > len || len - at < 8 || memcmp(d + at, "fLaC", 4) != 0) return 0;
  size_t q = at + 4;
  bool have_si = false;
  for (;;) {
    if (len - q < 4) return 0;
    const bool last = d[q] & 0x80;
    const int type = d[q] & 0x7F;
    const size_t bl = ((size_t)d[q + 1] << 16) | ((size_t)d[q + 2] << 8) | d[q + 3];
    q += 4;
    if (len - q < bl) return 0;
    if (type == 0) {
      if (bl < 34) return 0;
      const uint8_t* s = d + q;
      sp.min_bs = (s[0] << 8) | s[1];
      sp.max_bs = (s[2] << 8) | s[3];
      sp.sample_rate = (s[10] << 12) | (s[11] << 4) | (s[12] >> 4);
      sp.channels = ((s[12] >> 1) & 7) + 1;
      sp.bps = (((s[12] & 1) << 4) | (s[13] >> 4)) + 1;
      sp.total_samples = ((uint64_t)(s[13] & 15) << 32) | ((uint64_t)s[14] << 24) | ((uint64_t)s[15] << 16) |
                         ((uint64_t)s[16] << 8) | s[17];
      have_si = true;
    }
    q += bl;
    if (last) break;
  }
  return have_si ? q : 0;
}

struct Cand {
  uint64_t start, len;
  int32_t n;
};

}  // namespace

extern "C" {

FRA_API int fra_decode(const uint8_t* data, uint64_t len, int32_t flags, fra_decoded* info, int32_t** samples_out) {
  if (!data || !info || !samples_out) return fra_internal_set_error(FRA_E_INVALID, "null argument");
  *samples_out = nullptr;
  memset(info, 0, sizeof(*info));
  size_t at = 0;
  if (len >= 10 && memcmp(data, "ID3", 3) == 0) {  // ID3v2 prefix (mutagen may leave one)
    at = 10 + (((size_t)data[6] & 0x7F) << 21 | ((size_t)data[7] & 0x7F) << 14 | ((size_t)data[8] & 0x7F) << 7 |
               ((size_t)data[9] & 0x7F));
    if (at > len) return fra_internal_set_error(FRA_E_INVALID, "ID3v2 tag (%llu bytes) runs past the end of the data",
                                                (unsigned long long)at);
  }
  StreamParams sp;
  size_t audio = parse_metadata(data, len, at, sp);
  if (!audio) return fra_internal_set_error(FRA_E_INVALID, "not a FLAC stream (bad fLaC/STREAMINFO)");
  if (sp.channels < 1 || sp.channels > 8 || sp.bps < 4 || sp.bps > 32)
    return fra_internal_set_error(FRA_E_INVALID, "unsupported STREAMINFO (channels %d, bps %d)", sp.channels, sp.bps);

  // ---- pass 1: speculative validation of every sync candidate
  unsigned nt = std::thread::hardware_concurrency();
  nt = std::max(1u, std::min(nt, 16u));
  const uint64_t span = len - audio;
  if (span < (1u << 20)) nt = 1;
  std::vector<std::vector<Cand>> found(nt);
  auto scan = [&](unsigned t) {
    Scratch sc;
    const uint64_t b0 = audio + span * t / nt, b1 = audio + span * (t + 1) / nt;
    for (uint64_t q = b0; q < b1 && q + 1 < len; q++) {
      if (data[q] != 0xFF || (data[q + 1] & 0xFE) != 0xF8) continue;
      FrameHdr h;
      if (!parse_header(data + q, data + len, sp, h)) continue;
      if (h.channels != sp.channels) continue;
      const size_t fl = decode_frame(data + q, data + len, sp, h, nullptr, sp.channels, sc);
      if (fl) found[t].push_back({q, fl, h.blocksize});
    }
  };
  {
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; t++) th.emplace_back(scan, t);
    scan(0);
    for (auto& x : th) x.join();
  }
  std::vector<Cand> cand;
  for (auto& v : found) cand.insert(cand.end(), v.begin(), v.end());  // already sorted by start

  // ---- chain
  struct Fr { uint64_t start; int32_t n; uint64_t sample0; };
  std::vector<Fr> chain;
  uint64_t pos = audio, nsamp = 0;
  int nstreams = 1;
  while (pos < len) {
    auto it = std::lower_bound(cand.begin(), cand.end(), pos, [](const Cand& c, uint64_t v) { return c.start < v; });
    if (it != cand.end() && it->start == pos) {
      chain.push_back({pos, it->n, nsamp});
      nsamp += (uint64_t)it->n;
      pos += it->len;
      continue;
    }
    if ((flags & FRA_DECODE_CONCAT) && len - pos >= 4 && memcmp(data + pos, "fLaC", 4) == 0) {
      StreamParams sp2;
      const size_t a2 = parse_metadata(data, len, pos, sp2);
      if (!a2 || sp2.channels != sp.channels || sp2.bps != sp.bps)
        return fra_internal_set_error(FRA_E_INVALID, "concatenated stream at byte %llu has a different format",
                                      (unsigned long long)pos);
      pos = a2;
      nstreams++;
      continue;
    }
    return fra_internal_set_error(FRA_E_INVALID, "lost sync / corrupt frame at byte %llu", (unsigned long long)pos);
  }

  // ---- pass 2: decode into place
  const int C = sp.channels;
  int32_t* out = (int32_t*)malloc(std::max<uint64_t>(1, nsamp * (uint64_t)C) * sizeof(int32_t));
  if (!out) return fra_internal_set_error(FRA_E_NOMEM, "out of host memory");
  std::atomic<size_t> next{0};
  std::atomic<bool> fail{false};
  auto work = [&]() {
    Scratch sc;
    for (;;) {
      const size_t i = next.fetch_add(64);
      if (i >= chain.size() || fail.load()) return;
      const size_t e = std::min(chain.size(), i + 64);
      for (size_t k = i; k < e; k++) {
        FrameHdr h;
        const uint8_t* p = data + chain[k].start;
        if (!parse_header(p, data + len, sp, h) ||
            !decode_frame(p, data + len, sp, h, out + chain[k].sample0 * C, C, sc)) {
          fail = true;
          return;
        }
      }
    }
  };
  {
    const unsigned nt2 = chain.size() > 256 ? nt : 1;
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt2; t++) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
  }
  if (fail) {
    free(out);
    return fra_internal_set_error(FRA_E_INVALID, "frame decode failed in pass 2");
  }
  info->sample_rate = sp.sample_rate;
  info->channels = C;
  info->bps = sp.bps;
  info->blocksize = sp.max_bs;
  info->nframes = (int64_t)chain.size();
  info->nsamples = nsamp;
  info->nstreams = nstreams;
  info->audio_offset = audio;
  *samples_out = out;
  return FRA_OK;
}

}  // extern "C"
