// fra_internal.h -- device-side data layout of the MI355X FLAC raster encoder (product code).
//
// The encode path replaces the pyflac/libFLAC call at src/flac_raster/converter.py:139-154 and
// src/flac_raster/spatial_encoder.py:291-304 of the reference.  One "stream" = one FLAC stream =
// one reference encode unit (a streaming/spatial tile, or the whole raster in the standard format).
// One "frame" = blocksize (4096) consecutive samples of every channel of a stream.
// One "subframe" = one channel of one frame (the unit of the analysis kernel).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define FRA_HD __host__ __device__ inline
#else
#define FRA_HD inline
#endif

namespace fra {

enum SrcType : int32_t { ST_U8 = 0, ST_I8, ST_U16, ST_I16, ST_U32, ST_I32, ST_F32, ST_F64 };

constexpr int kMaxBlock = 4096;   // samples per frame handled by one workgroup (reference uses 4096)
constexpr int kThreads = 256;     // 4 waves; each thread owns 16 consecutive samples
constexpr int kChunk = 16;        // samples per thread (also the FRA-1 autocorrelation chunk)
constexpr int kMaxLpc = 12;
constexpr int kMaxChannels = 8;  // FLAC channel limit (RFC 9639)
constexpr int kMaxPart = 64;      // 2^6 partitions (level 6-8 max partition order)
constexpr int kMaxWin = 6;        // subdivide_tukey(3): 1 + 2 + 3 windows
constexpr int kMaxModels = 5 + kMaxWin;  // fixed 0..4, one LPC order per apodization window
// LDS sample array layout of k_analyze: each thread's 16-sample chunk at a stride of 20 words (4 pad
// words), so the per-thread chunk reads (lane stride 20 dwords) are bank-conflict free for
// ds_read_b32..b128; one zeroed chunk in front stands in for the samples before the block start.
// The 32-bit array (32-bps analysis) pads 2 words per chunk instead (8-byte aligned chunks, 2-way conflicts):
// 2 KiB less LDS, so the 32-bps workgroup fits 32 KiB (5 per CU).
constexpr int kSmpStride = kChunk + 4;
constexpr int kSmpWords = (kMaxBlock / kChunk + 1) * kSmpStride;
template <typename T>
FRA_HD constexpr int smp_stride() { return sizeof(T) == 4 ? kChunk + 2 : kChunk + 4; }
template <typename T>
FRA_HD constexpr int smp_words() { return (kMaxBlock / kChunk + 1) * smp_stride<T>(); }
// sample i of the array smp (its element type picks the layout)
template <typename T>
FRA_HD int sidx(const T*, int i) { return smp_stride<T>() + i + (i >> 4) * (smp_stride<T>() - kChunk); }

// FRA-1 3.7b windows kept at levels 7-8 (the oracle's level table must agree).  r06: 2 then 1 -- C5 analysis 88.2 ->
// 72.7 -> 67.7 ms, frame bytes +0.015 % -> +0.026 % against evaluating all 6 windows (profiles/r06_ab_c5_window_pruning.txt)
#ifndef FRA_LPC_KEEP78
#define FRA_LPC_KEEP78 1
#endif
// libFLAC 1.4.3 compression-level table (docs/sonos-pyflac.txt:6926-6934)
struct LevelCfg {
  int32_t max_lpc, max_porder, nsub;
  int32_t ms;        // mid-side stereo column (levels 1, 2, 4-8)
  int32_t lpc_keep;  // FRA-1 3.7b (r06): LPC windows whose residuals are evaluated, by window score (0 = all)
};
FRA_HD LevelCfg level_cfg(int level) {
  switch (level < 0 ? 0 : (level > 8 ? 8 : level)) {
    case 0: return {0, 3, 0, 0, 0};
    case 1: case 2: return {0, 3, 0, 1, 0};
    case 3: return {6, 4, 1, 0, 0};
    case 4: return {8, 4, 1, 1, 0};
    case 5: return {8, 5, 1, 1, 0};
    case 6: return {8, 6, 2, 1, 0};
    case 7: return {12, 6, 2, 1, FRA_LPC_KEEP78};
    default: return {12, 6, 3, 1, FRA_LPC_KEEP78};
  }
}
FRA_HD int num_windows(int nsub) {
  int c = nsub > 0 ? 1 : 0;
  for (int m = 2; m <= nsub; m++) c += m;
  return c;
}
// qlp coefficient precision: libFLAC's automatic rule (qlp_coeff_precision = 0 at every level)
FRA_HD int qlp_precision(int bps, int bs) {
  if (bps < 16) { int p = 2 + bps / 2; return p < 5 ? 5 : p; }
  if (bps == 16) {
    if (bs <= 192) return 7;
    if (bs <= 384) return 8;
    if (bs <= 576) return 9;
    if (bs <= 1152) return 10;
    if (bs <= 2304) return 11;
    if (bs <= 4608) return 12;
    return 13;
  }
  if (bs <= 384) return 13;
  if (bs <= 1152) return 14;
  return 15;
}
FRA_HD int max_porder(int n, int o, int cap) {
  int p = 0;
  while (p < cap && ((n >> (p + 1)) << (p + 1)) == n && (n >> (p + 1)) > o) p++;
  return p;
}

// RFC 9639 frame-header code tables
FRA_HD int bs_code(int bs, int* extra_bits) {
  *extra_bits = 0;
  if (bs == 192) return 1;
  if (bs == 576) return 2;
  if (bs == 1152) return 3;
  if (bs == 2304) return 4;
  if (bs == 4608) return 5;
  for (int c = 8; c <= 15; c++)
    if (bs == (256 << (c - 8))) return c;
  if (bs <= 256) { *extra_bits = 8; return 6; }
  *extra_bits = 16;
  return 7;
}
FRA_HD int sr_code(int sr, int* extra_bits, int* extra_val) {
  *extra_bits = 0;
  *extra_val = 0;
  switch (sr) {
    case 88200: return 1;
    case 176400: return 2;
    case 192000: return 3;
    case 8000: return 4;
    case 16000: return 5;
    case 22050: return 6;
    case 24000: return 7;
    case 32000: return 8;
    case 44100: return 9;
    case 48000: return 10;
    case 96000: return 11;
  }
  if (sr % 1000 == 0 && sr / 1000 <= 255) { *extra_bits = 8; *extra_val = sr / 1000; return 12; }
  if (sr <= 65535) { *extra_bits = 16; *extra_val = sr; return 13; }
  if (sr % 10 == 0 && sr / 10 <= 65535) { *extra_bits = 16; *extra_val = sr / 10; return 14; }
  return 0;
}
FRA_HD int bps_code(int bps) {
  switch (bps) {
    case 8: return 1;
    case 12: return 2;
    case 16: return 4;
    case 20: return 5;
    case 24: return 6;
    case 32: return 7;
  }
  return 0;
}

// ---------------------------------------------------------------- device job description
struct StreamDev {
  int64_t base_off;      // element offset of (band 0, window row 0, window col 0)
  int64_t band_stride;   // elements between bands (channels)
  int64_t row_stride;    // elements between rows
  int64_t col_stride;    // elements between pixels of a row
  int32_t width, height; // window
  int32_t channels;
  int32_t bps;           // FLAC bits per sample: 16 or 32
  int32_t norm;          // 0 = samples are already audio ints; 16 / 24 = normalize_to_audio(bps)
  int32_t sample_rate;
  int32_t first_frame, nframes;
  int64_t nsamples;      // per channel (= width*height)
  uint32_t frame_number0;  // FLAC frame number of the stream's first frame (pyflac shim: blocks already emitted)
  int32_t ms;            // FRA-1 3.1b mid-side: virtual channels 0 L, 1 R, 2 M = (L+R)>>1, 3 S = L-R (bps+1)
};

struct FrameDev {
  int32_t stream;
  int32_t index;   // frame number within its stream
  int32_t n;       // block size of this frame
  int32_t win;     // window-table index (one table set per distinct block size)
  int32_t row0, col0;  // window-relative pixel position of sample 0
};

// per-frame analysis metadata (built at plan creation): everything the load phase of k_analyze_w / k_analyze needs
// in ONE scalar load, instead of FrameDev -> StreamDev (two dependent round trips before the first raw row)
struct WaveDev {
  int64_t off0;         // element offset of band 0, the frame's first row (StreamDev base_off + row0 * row_stride)
  int64_t band_stride;  // elements between channels
  uint32_t row_stride;  // elements between rows
  uint32_t width;       // window width (col_stride 1)
  uint32_t col0;        // window-relative column of sample 0
  int32_t stream;       // stream index (normalisation table row)
  int32_t n;            // block size of the frame
  int32_t win;          // window-table index
  int32_t bps;          // FLAC bits per sample
  int32_t nch;          // channels the wave kernel analyses (mid-side: L and R)
  int32_t channels;     // StreamDev::channels
  int32_t ms;           // StreamDev::ms
  int32_t norm;         // StreamDev::norm
};

struct NormDev {       // per stream, filled on device
  unsigned long long mnkey, mxkey;  // ordered-key min/max (NaN excluded)
  double mn, mx, range;             // normalize_to_audio parameters (normalization.py:148-159)
};

// One analysed subframe (FRA-1 decision), written by k_analyze, read by k_frame_scan / k_assemble.
struct SfDesc {
  uint32_t bits;      // exact subframe size in bits
  uint8_t type;       // 0 CONSTANT, 1 VERBATIM, 2 FIXED, 3 LPC
  uint8_t order;
  uint8_t wasted;
  uint8_t sbps;       // sample bits after wasted-bit shift (CONSTANT: stream bps)
  uint8_t porder;
  uint8_t method;     // 0 RICE (4-bit params), 1 RICE2 (5-bit)
  uint8_t precision;
  int8_t shift;
  int32_t cval;       // CONSTANT value
  int32_t coef[kMaxLpc];
  uint8_t k[kMaxPart];
};

// per-frame metadata written by k_frame_scan for k_assemble: words [0, kHdrWords) = frame header and
// its CRC-8 as big-endian words (zero padded), words [kHdrWords, +kMaxChannels+2) = bit bounds:
// 0, header bits, end of channel 0, ..., end of channel C-1 (unused entries = 0xFFFFFFFF)
// CRC-16 table layout (fra_api.hip crc16_tables): [0, 1024) slice-by-4 byte tables, [1024, +24*512)
// multiply-by-x^(8*2^i) tables, [kCrcT16Off, +16*256) slice-by-16 byte tables
constexpr int kCrcT16Off = 1024 + 24 * 512;
constexpr int kHdrWords = 6;
constexpr int kMetaWords = 16;
// wave issue priority (s_setprio) of the background kernels of a pipelined execute -- k_minmax_vec and k_assemble4 --
// over the co-resident k_analyze_w waves (r05; 0 = off)
#ifndef FRA_BG_PRIO
#define FRA_BG_PRIO 2
#endif
static_assert(kHdrWords + kMaxChannels + 2 <= kMetaWords, "frame metadata layout");

struct JobArgs {
  const void* raster;
  const StreamDev* streams;
  const FrameDev* frames;
  NormDev* norm;
  const float* win;        // [ntables][nwin][blocksize]
  const int32_t* wrange;   // [ntables][nwin][2]: nonzero extent [lo, hi) of each window
  const int32_t* wplat;    // [ntables][nwin][2]: the longest run [lo, hi) of coefficients exactly 1.0f
  SfDesc* sf;              // [nframes_total][cmax]
  unsigned long long* frame_bytes;  // [nframes_total + 1] (last = 0)
  unsigned long long* frame_off;  // [nframes_total + 1] exclusive scan of frame_bytes
  uint8_t* out;            // concatenated frames
  uint64_t out_cap;        // bytes allocated at out
  const uint16_t* crctab;  // CRC-16 slice-by-4 tables [4][256] + multiply-by-x^(8*2^i) tables [24][2][256]
  uint32_t* fmeta;         // [nframes_total][kMetaWords]: header (+CRC-8) as big-endian words, blob bit bounds
  uint32_t* tmp;           // encoded subframes: slot (frame*cmax + channel) of tmp_stride words
  const int32_t* lut;      // normalize_to_audio table per stream (<= 16-bit integer dtypes), or null
  int64_t lut_stride;      // entries per stream: 256 (8-bit) or 65536 (16-bit), indexed by the raw value (lut_index)
  int64_t tmp_stride;
  int32_t nframes_total;
  int32_t cmax;
  int32_t blocksize;
  int32_t level;
  int32_t nwin;
  int32_t vec8;            // k_analyze may load 8-byte sample vectors (host-checked alignment)
  int32_t off32;           // every frame's samples of one channel lie within 2^31 bytes of its first row
                           // (k_analyze fast load path: 32-bit lane offsets from a uniform base)
  int32_t frame_base;      // frame group of this launch (k_analyze / k_frame_scan / k_assemble):
  int32_t frame_count;     //   frames [frame_base, frame_base + frame_count)
  const int32_t* part;     // k_analyze list mode (beside k_analyze_w): (frame * 8 + channel) of the partial
  int32_t npart;           //   subframes of the launch's frames, npart entries (null: the normal grid)
  uint32_t* cnt17;         // k_analyze_w: += 1 per wave whose kept residuals needed bit 16 (null: not counted)
  int32_t k17;             // k_analyze_w instance: kept residuals up to 17 bits (1) or 16 (0)
  uint32_t* err;           // plan error word (checked at every sync): bit 0 frame-scan ticket desync, bit 1 a
                           //   frame outside its output / slot bounds (not written)
  const WaveDev* wave;     // [nframes_total]
};

}  // namespace fra
