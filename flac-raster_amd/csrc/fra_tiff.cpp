// fra_tiff.cpp -- multi-threaded GeoTIFF chunk decoder (host C++): the raster I/O ahead of the encode
// path.  The reference reads rasters with rasterio/GDAL -- whole rasters at
// converter.py:73-79, one window per tile at cli.py:559 and spatial_encoder.py:205-206.  Here the Python
// host (flac_raster/tiff.py) parses the IFD and hands the strips/tiles that overlap a window to
// fra_tiff_decode, which inflates them on a thread pool and writes the overlap straight into a
// band-planar destination -- typically page-locked memory from fra_host_alloc, so the H2D copies of
// fra_plan_encode_host run at full PCIe rate with no staging copy.
//
// Supported (the TIFF 6.0 + Adobe subset GDAL writes for GeoTIFF): Compression 1 (none), 5 (LZW,
// MSB-first codes with the TIFF "early change"), 8 / 32946 (deflate); Predictor 1, 2 (horizontal
// differencing, integer samples, in the file's byte order) and 3 (floating point: byte-plane shuffle +
// byte differencing per row, the Adobe TIFF Technical Note 3 layout libtiff implements); II or MM byte
// order; PlanarConfiguration 1 (chunky) or 2 (planar); 1/2/4/8-byte samples.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/flac_raster_amd.h"

extern "C" int fra_internal_set_error(int code, const char* fmt, ...);

namespace {

// TIFF LZW (compression 5): codes MSB-first, 9..12 bits, 256 = Clear, 257 = EOI, the code width grows
// when the next free entry reaches 2^width - 1 ("early change").  Returns bytes produced, or -1.
int64_t lzw_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap) {
  if (n >= 2 && in[0] == 0 && (in[1] & 1)) return -2;  // pre-5.0 LSB-first "old-style" LZW
  uint16_t prefix[4096];
  uint16_t length[4096];
  uint8_t suffix[4096], first[4096];
  for (int i = 0; i < 256; i++) {
    prefix[i] = 0xFFFF;
    length[i] = 1;
    suffix[i] = first[i] = (uint8_t)i;
  }
  uint64_t acc = 0;
  int nbits = 0;
  size_t ip = 0, o = 0;
  int width = 9, next = 258, prev = -1;
  for (;;) {
    while (nbits < width && ip < n) {
      acc = (acc << 8) | in[ip++];
      nbits += 8;
    }
    if (nbits < width) break;  // ran out of input without EOI: libtiff tolerates it
    const int code = (int)((acc >> (nbits - width)) & ((1u << width) - 1));
    nbits -= width;
    if (code == 257) break;
    if (code == 256) {
      width = 9;
      next = 258;
      prev = -1;
      continue;
    }
    if (prev < 0) {
      if (code > 255) return -1;
      if (o >= cap) return -1;
      out[o++] = (uint8_t)code;
      prev = code;
      continue;
    }
    int L;
    uint8_t f;
    if (code < next) {
      L = length[code];
      if (o + (size_t)L > cap) return -1;
      int c = code;
      for (int j = L - 1; j >= 0; j--) {
        out[o + j] = suffix[c];
        c = prefix[c];
      }
      f = first[code];
    } else if (code == next) {  // KwKwK
      L = length[prev] + 1;
      if (o + (size_t)L > cap) return -1;
      int c = prev;
      for (int j = L - 2; j >= 0; j--) {
        out[o + j] = suffix[c];
        c = prefix[c];
      }
      out[o + L - 1] = first[prev];
      f = first[prev];
    } else {
      return -1;
    }
    if (next < 4096) {
      prefix[next] = (uint16_t)prev;
      suffix[next] = f;
      first[next] = first[prev];
      length[next] = (uint16_t)(length[prev] + 1);
      next++;
      if (next >= (1 << width) - 1 && width < 12) width++;
    }
    o += (size_t)L;
    prev = code;
  }
  return (int64_t)o;
}

int64_t inflate_chunk(const uint8_t* in, size_t n, uint8_t* out, size_t cap) {
  z_stream z;
  memset(&z, 0, sizeof(z));
  if (inflateInit(&z) != Z_OK) return -1;
  z.next_in = const_cast<Bytef*>(in);
  z.avail_in = (uInt)n;
  z.next_out = out;
  z.avail_out = (uInt)cap;
  const int rc = inflate(&z, Z_FINISH);
  const int64_t got = (int64_t)(cap - z.avail_out);
  inflateEnd(&z);
  if (rc != Z_STREAM_END && rc != Z_OK && rc != Z_BUF_ERROR) return -1;
  return got;
}

// TIFF LZW encoder, the inverse of lzw_decode: Clear first, codes MSB-first, 9..12 bits.  The decoder adds
// one entry per code after the first and widens once its next free entry reaches 2^width - 1; the encoder
// adds its entry one code earlier, so it widens when its own next entry reaches 2^width.  Before the table
// could overflow (next entry 4093) a Clear restarts it.  Returns bytes written, or -1 if cap is too small.
int64_t lzw_encode(const uint8_t* in, size_t n, uint8_t* out, size_t cap) {
  constexpr int kHash = 1 << 14;
  std::vector<int32_t> key(kHash);
  std::vector<uint16_t> val(kHash);
  uint64_t acc = 0;
  int nbits = 0;
  size_t o = 0;
  bool ok = true;
  auto emit = [&](int code, int width) {
    acc = (acc << width) | (uint64_t)code;
    nbits += width;
    while (nbits >= 8) {
      if (o >= cap) { ok = false; nbits -= 8; continue; }
      out[o++] = (uint8_t)(acc >> (nbits - 8));
      nbits -= 8;
    }
  };
  auto reset = [&]() { std::fill(key.begin(), key.end(), -1); };
  reset();
  int width = 9, next = 258;
  emit(256, width);
  if (n == 0) {
    emit(257, width);
  } else {
    int w = in[0];
    for (size_t i = 1; i < n; i++) {
      const int c = in[i];
      const int32_t k = (w << 8) | c;
      uint32_t h = ((uint32_t)k * 2654435761u) >> 18;
      int found = -1;
      while (key[h] >= 0) {
        if (key[h] == k) { found = val[h]; break; }
        h = (h + 1) & (kHash - 1);
      }
      if (found >= 0) { w = found; continue; }
      emit(w, width);
      if (next < 4093) {
        key[h] = k;
        val[h] = (uint16_t)next++;
        if (next >= (1 << width) && width < 12) width++;
      } else {
        emit(256, width);
        reset();
        width = 9;
        next = 258;
      }
      w = c;
    }
    emit(w, width);
    // the decoder adds an entry for this code too: keep its width step in step before EOI
    if (next < 4093) {
      next++;
      if (next >= (1 << width) && width < 12) width++;
    }
    emit(257, width);
  }
  if (nbits > 0) {
    if (o >= cap) ok = false;
    else out[o++] = (uint8_t)(acc << (8 - nbits));
  }
  return ok ? (int64_t)o : -1;
}

inline void bswap_inplace(uint8_t* p, size_t nelem, int es) {
  if (es == 2) {
    for (size_t i = 0; i < nelem; i++) std::swap(p[2 * i], p[2 * i + 1]);
  } else if (es == 4) {
    for (size_t i = 0; i < nelem; i++) {
      uint32_t v;
      memcpy(&v, p + 4 * i, 4);
      v = __builtin_bswap32(v);
      memcpy(p + 4 * i, &v, 4);
    }
  } else if (es == 8) {
    for (size_t i = 0; i < nelem; i++) {
      uint64_t v;
      memcpy(&v, p + 8 * i, 8);
      v = __builtin_bswap64(v);
      memcpy(p + 8 * i, &v, 8);
    }
  }
}

// Predictor 2 on native-order samples of one row: x[i] += x[i - spp] (modular arithmetic)
template <typename T>
void hor_acc(uint8_t* row, int64_t nsamp, int spp) {
  T* x = reinterpret_cast<T*>(row);
  for (int64_t i = spp; i < nsamp; i++) x[i] = (T)(x[i] + x[i - spp]);
}

// Predictor 3 on one row of `count` samples of es bytes: undo the byte differencing (stride spp), then
// gather byte planes (most significant plane first) into native little-endian samples.
void fp_acc(uint8_t* row, int64_t count, int es, int spp, std::vector<uint8_t>& tmp) {
  const int64_t nb = count * es;
  for (int64_t i = spp; i < nb; i++) row[i] = (uint8_t)(row[i] + row[i - spp]);
  tmp.assign(row, row + nb);
  for (int64_t k = 0; k < count; k++)
    for (int b = 0; b < es; b++) row[k * es + b] = tmp[(size_t)(es - 1 - b) * count + k];
}

}  // namespace

extern "C" {

FRA_API int fra_tiff_decode(const uint8_t* file, uint64_t file_len, const fra_tiff_layout* L,
                            const fra_tiff_chunk* chunks, int32_t nchunks, void* dst, int32_t threads) {
  if (!file || !L || (!chunks && nchunks) || (!dst && nchunks)) return fra_internal_set_error(FRA_E_INVALID, "null argument");
  const int es = L->bytes_per_sample, spp = L->samples_per_pixel;
  if (es != 1 && es != 2 && es != 4 && es != 8) return fra_internal_set_error(FRA_E_INVALID, "bad sample size %d", es);
  if (spp < 1 || L->bands < 1 || spp > L->bands) return fra_internal_set_error(FRA_E_INVALID, "bad samples per pixel");
  const int comp = L->compression, pred = L->predictor;
  if (comp != 1 && comp != 5 && comp != 8 && comp != 32946)
    return fra_internal_set_error(FRA_E_INVALID, "TIFF compression %d not supported (1, 5 LZW, 8/32946 deflate)", comp);
  if (pred != 1 && pred != 2 && pred != 3)
    return fra_internal_set_error(FRA_E_INVALID, "TIFF predictor %d not supported", pred);
  if (pred == 2 && L->is_float)
    return fra_internal_set_error(FRA_E_INVALID, "TIFF predictor 2 on floating-point samples is invalid");
  if (pred == 3 && !L->is_float)
    return fra_internal_set_error(FRA_E_INVALID, "TIFF predictor 3 needs floating-point samples");
  for (int i = 0; i < nchunks; i++) {
    const fra_tiff_chunk& c = chunks[i];
    if (c.offset > file_len || c.bytes > file_len - c.offset || c.rows < 0 || c.cols < 0 ||
        (spp == 1 && (c.plane < 0 || c.plane >= L->bands)))
      return fra_internal_set_error(FRA_E_INVALID, "TIFF chunk %d out of the file / bad geometry", i);
    // decoded chunk size rows * cols * spp * es from untrusted tags: no 64-bit wrap, and no more than the
    // stored bytes can hold -- uncompressed: their count (checked again per chunk); LZW/deflate: at most
    // 4096 decoded bytes per stored byte (a 12-bit LZW code expands to <= 4096 bytes; deflate <= 1032),
    // so a malformed file is an error, not a huge allocation
    uint64_t need = 0;
    const uint64_t cap = comp == 1 ? c.bytes : c.bytes * 4096ull + 65536ull;
    if (__builtin_mul_overflow((uint64_t)c.cols, (uint64_t)spp * (uint64_t)es, &need) ||
        __builtin_mul_overflow(need, (uint64_t)c.rows, &need) || need > cap)
      return fra_internal_set_error(FRA_E_INVALID, "TIFF chunk %d: %d x %d x %d samples do not fit its %llu stored bytes",
                                    i, c.rows, c.cols, spp, (unsigned long long)c.bytes);
  }
  int nt = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
  nt = std::max(1, std::min({nt, 64, std::max(1, (int)nchunks)}));
  std::atomic<int> next{0};
  std::atomic<int> failed{-1};
  std::atomic<int> why{0};
  auto work_body = [&](std::vector<uint8_t>& buf, std::vector<uint8_t>& tmp, int& cur) {
    for (;;) {
      const int i = next.fetch_add(1);
      cur = i;
      if (i >= nchunks || failed.load() >= 0) return;
      const fra_tiff_chunk& c = chunks[i];
      const size_t row_bytes = (size_t)c.cols * spp * es;
      const size_t need = row_bytes * (size_t)c.rows;
      const uint8_t* raw = file + c.offset;
      const uint8_t* data;
      if (comp == 1) {
        if (c.bytes < need) { failed = i; why = 1; return; }
        if (pred == 1 && !L->big_endian) {
          data = raw;  // no copy: scatter straight from the (mapped) file
        } else {
          buf.assign(raw, raw + need);
          data = buf.data();
        }
      } else {
        buf.resize(need);
        const int64_t got = comp == 5 ? lzw_decode(raw, c.bytes, buf.data(), need) : inflate_chunk(raw, c.bytes, buf.data(), need);
        if (got < 0) { failed = i; why = got == -2 ? 3 : 2; return; }
        if ((size_t)got < need) memset(buf.data() + got, 0, need - got);  // short chunk: libtiff zero-fills
        data = buf.data();
      }
      uint8_t* d8 = const_cast<uint8_t*>(data);
      if (pred == 3) {
        for (int r = 0; r < c.rows; r++) fp_acc(d8 + r * row_bytes, (int64_t)c.cols * spp, es, spp, tmp);
      } else {
        if (L->big_endian && es > 1) bswap_inplace(d8, (size_t)c.cols * spp * c.rows, es);
        if (pred == 2)
          for (int r = 0; r < c.rows; r++) {
            uint8_t* row = d8 + r * row_bytes;
            const int64_t ns = (int64_t)c.cols * spp;
            switch (es) {
              case 1: hor_acc<uint8_t>(row, ns, spp); break;
              case 2: hor_acc<uint16_t>(row, ns, spp); break;
              case 4: hor_acc<uint32_t>(row, ns, spp); break;
              default: hor_acc<uint64_t>(row, ns, spp); break;
            }
          }
      }
      // overlap of the chunk with the destination window
      const int64_t r0 = std::max<int64_t>(c.row0, L->win_row), r1 = std::min<int64_t>((int64_t)c.row0 + c.rows, (int64_t)L->win_row + L->win_h);
      const int64_t c0 = std::max<int64_t>(c.col0, L->win_col), c1 = std::min<int64_t>((int64_t)c.col0 + c.cols, (int64_t)L->win_col + L->win_w);
      if (r0 >= r1 || c0 >= c1) continue;
      uint8_t* o8 = static_cast<uint8_t*>(dst);
      for (int64_t r = r0; r < r1; r++) {
        const uint8_t* srow = data + (size_t)(r - c.row0) * row_bytes + (size_t)(c0 - c.col0) * spp * es;
        const int64_t drow = (r - L->win_row) * L->dst_row_stride + (c0 - L->win_col);
        if (spp == 1) {
          memcpy(o8 + (size_t)(c.plane * L->dst_band_stride + drow) * es, srow, (size_t)(c1 - c0) * es);
        } else {  // chunky: de-interleave the pixels into the band planes
          const int64_t w = c1 - c0;
          for (int b = 0; b < spp; b++) {
            uint8_t* dp = o8 + (size_t)(b * L->dst_band_stride + drow) * es;
            const uint8_t* sp = srow + (size_t)b * es;
            switch (es) {
              case 1: for (int64_t x = 0; x < w; x++) dp[x] = sp[x * spp]; break;
              case 2: for (int64_t x = 0; x < w; x++) memcpy(dp + 2 * x, sp + 2 * x * spp, 2); break;
              case 4: for (int64_t x = 0; x < w; x++) memcpy(dp + 4 * x, sp + 4 * x * spp, 4); break;
              default: for (int64_t x = 0; x < w; x++) memcpy(dp + 8 * x, sp + 8 * x * spp, 8); break;
            }
          }
        }
      }
    }
  };
  // no exception may leave a worker thread (std::terminate) or cross the C ABI: report it as a failure
  auto work = [&]() {
    std::vector<uint8_t> buf, tmp;
    int cur = -1;
    try {
      work_body(buf, tmp, cur);
    } catch (...) {
      int expect = -1;
      failed.compare_exchange_strong(expect, std::max(0, cur));
      why = 4;
    }
  };
  if (nt == 1) {
    work();
  } else {
    std::vector<std::thread> th;
    for (int t = 1; t < nt; t++) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
  }
  if (failed.load() >= 0) {
    const int w = why.load();
    return fra_internal_set_error(FRA_E_INVALID, "TIFF chunk %d: %s", failed.load(),
                                  w == 1 ? "truncated uncompressed chunk"
                                         : (w == 3 ? "old-style (LSB-first) LZW is not supported"
                                                  : (w == 4 ? "out of memory" : "corrupt compressed data")));
  }
  return FRA_OK;
}

}  // extern "C"

extern "C" {

FRA_API uint64_t fra_tiff_compress_bound(int32_t compression, uint64_t chunk_bytes) {
  if (compression == 8 || compression == 32946) return (uint64_t)compressBound((uLong)chunk_bytes) + 64;
  return chunk_bytes + chunk_bytes / 2 + 64;  // LZW: <= 12 bits per input byte + Clear/EOI codes
}

FRA_API int fra_tiff_compress(int32_t compression, int32_t level, const uint8_t* src, uint64_t chunk_bytes,
                              int32_t nchunks, uint8_t* dst, uint64_t dst_stride, uint64_t* sizes, int32_t threads) {
  if ((!src || !dst || !sizes) && nchunks > 0) return fra_internal_set_error(FRA_E_INVALID, "null argument");
  if (compression != 5 && compression != 8 && compression != 32946)
    return fra_internal_set_error(FRA_E_INVALID, "compression %d not supported (5 LZW, 8 deflate)", compression);
  if (dst_stride < fra_tiff_compress_bound(compression, chunk_bytes))
    return fra_internal_set_error(FRA_E_INVALID, "dst_stride below fra_tiff_compress_bound");
  int nt = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
  nt = std::max(1, std::min({nt, 64, std::max(1, (int)nchunks)}));
  std::atomic<int> next{0};
  std::atomic<int> failed{-1};
  auto work = [&]() {
    try {
      for (;;) {
        const int i = next.fetch_add(1);
        if (i >= nchunks || failed.load() >= 0) return;
        const uint8_t* in = src + (size_t)i * chunk_bytes;
        uint8_t* out = dst + (size_t)i * dst_stride;
        if (compression == 5) {
          const int64_t got = lzw_encode(in, chunk_bytes, out, dst_stride);
          if (got < 0) { failed = i; return; }
          sizes[i] = (uint64_t)got;
        } else {
          uLongf got = (uLongf)dst_stride;
          if (compress2(out, &got, in, (uLong)chunk_bytes, level < 0 ? Z_DEFAULT_COMPRESSION : level) != Z_OK) {
            failed = i;
            return;
          }
          sizes[i] = (uint64_t)got;
        }
      }
    } catch (...) {
      int expect = -1;
      failed.compare_exchange_strong(expect, 0);
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; t++) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  if (failed.load() >= 0) return fra_internal_set_error(FRA_E_INVALID, "TIFF chunk %d: compression failed", failed.load());
  return FRA_OK;
}

}  // extern "C"
