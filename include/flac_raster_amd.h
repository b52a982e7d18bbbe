/*
 * flac_raster_amd.h -- C ABI of the MI355X (gfx950) FLAC raster encoder.
 *
 * This library replaces the encode half of the reference's pyflac/libFLAC boundary:
 *
 *   reference call site                                   what replaces it here
 *   ---------------------------------------------------   -------------------------------------
 *   pyflac.StreamEncoder(write_callback, sample_rate,     fra_encode() / fra_plan_*() with
 *     compression_level, blocksize=4096)                  fra_job.norm = 0 (samples are already
 *   encoder.process(audio); encoder.finish()              int16/int32 audio, pyflac semantics F3:
 *     src/flac_raster/converter.py:139-154                bps = itemsize*8)
 *     src/flac_raster/spatial_encoder.py:291-304
 *     (pyflac 3.0.0 _Encoder.process/finish,
 *      docs/sonos-pyflac.txt:1968-2014; libFLAC C ABI
 *      FLAC__stream_encoder_new, set_..., init_stream,
 *      process_interleaved/finish, :3205-3262)
 *
 *   normalize_to_audio(interleave(raster)) + the above,   fra_job.norm = 16 or 24: raw raster in,
 *     once per encode unit (whole raster / tile)          per-window nanmin/nanmax + the float64
 *     normalization.py:126-202, converter.py:93-154,      normalisation fused on the GPU
 *     spatial_encoder.py:196-245, cli.py:553-622
 *
 * Output of an encode = the FLAC *frames* of every window's stream, concatenated in window order,
 * plus per-stream info.  The 86-byte stream header (fLaC + STREAMINFO + VORBIS_COMMENT, F4 of
 * SURVEY.md) is produced by fra_stream_header(); the Python host layer assembles headers, tags
 * (mutagen-equivalent) and containers.
 *
 * Conventions: every function returns 0 on success or a negative fra_status; the message of the
 * last failure on the calling thread is fra_last_error().  No C++ exception crosses this ABI.
 * Library-allocated buffers are released with fra_free().  A context is bound to one HIP device
 * and owns one HIP stream; plans are not thread-safe, distinct plans may run on distinct threads.
 */
#ifndef FLAC_RASTER_AMD_H
#define FLAC_RASTER_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FRA_ABI_VERSION 3

#if defined(__GNUC__) || defined(__clang__)
#define FRA_API __attribute__((visibility("default")))
#else
#define FRA_API
#endif

typedef enum {
  FRA_OK = 0,
  FRA_E_INVALID = -1,   /* bad argument */
  FRA_E_HIP = -2,       /* HIP runtime error (message in fra_last_error) */
  FRA_E_NODEVICE = -3,  /* no usable gfx950 device */
  FRA_E_NOMEM = -4,
  FRA_E_STATE = -5,     /* call out of order (e.g. result before execute) */
  FRA_E_SPACE = -6      /* caller's output buffer too small (the required size is reported) */
} fra_status;

/* dtype codes of the source samples (numpy names) */
typedef enum {
  FRA_U8 = 0, FRA_I8 = 1, FRA_U16 = 2, FRA_I16 = 3, FRA_U32 = 4, FRA_I32 = 5, FRA_F32 = 6, FRA_F64 = 7
} fra_dtype;

/* one encode unit: a rasterio Window (cli.py:553-559 / spatial_encoder.py:110-121) */
typedef struct {
  int32_t row_off, col_off, height, width;
} fra_window;

typedef struct {
  const void *raster;       /* element (band 0, row 0, col 0) */
  int32_t raster_on_device; /* 1: device pointer on the context's GPU; 0: host memory (copied) */
  int32_t dtype;            /* fra_dtype */
  int32_t channels;         /* bands -> FLAC channels (1..8) */
  int64_t band_stride;      /* elements between bands */
  int64_t row_stride;       /* elements between rows */
  int64_t col_stride;       /* elements between pixels of a row (1 planar, C interleaved) */
  const fra_window *windows;
  int32_t nwindows;
  int32_t level;            /* FLAC compression level 0..8 (cli.py:60-62, default 5) */
  int32_t blocksize;        /* samples per frame, 16..4096 (reference passes 4096) */
  int32_t norm;             /* 0: samples already audio ints (pyflac path); 16 / 24: normalize_to_audio */
  int32_t sample_rate;      /* 0: calculate_audio_params rule from window H*W (normalization.py:108-120) */
  int32_t first_frame;      /* FLAC frame number of every stream's first frame (0; the pyflac shim
                               continues a stream across process() calls, sonos-pyflac.txt:1968-2001) */
} fra_job;

typedef struct {
  uint64_t offset;          /* byte offset of this stream's frames in the concatenated output */
  uint64_t frame_bytes;     /* bytes of frames (header excluded) */
  double data_min, data_max;/* normalize_to_audio params (NaN if all-NaN); 0/0 when norm == 0 */
  int32_t sample_rate, bps, channels, nframes;
} fra_stream_info;

typedef struct fra_ctx fra_ctx;
typedef struct fra_plan fra_plan;

FRA_API const char *fra_last_error(void);
FRA_API int fra_abi_version(void);
FRA_API int fra_device_count(int *count);
FRA_API void fra_free(void *p);

FRA_API int fra_ctx_create(int device, fra_ctx **out);
FRA_API void fra_ctx_destroy(fra_ctx *ctx);

/* Plan = all device workspace for one job shape; execute enqueues only (no allocation/sync). */
FRA_API int fra_plan_create(fra_ctx *ctx, const fra_job *job, fra_plan **out);
/* The same plan over FRAME RANGES of the windows (r05, multi-GPU work items of equal size):
 * frame_ranges[2 w] = first frame, frame_ranges[2 w + 1] = frame count (-1: to the stream's end) of window
 * w.  The normalisation (data_min/max, sample rate) still spans the whole window and the frames keep their
 * frame numbers, so the concatenated frames of all ranges of one window, in order, are exactly the stream
 * fra_plan_create would encode (the reference encodes a window as one stream, cli.py:553-597).
 * fra_stream_info.nframes / frame_bytes describe the range.  A count past the stream's end is clipped to it; a
 * first frame < 0 or past the stream's frame count, or a count < -1, is FRA_E_INVALID. */
FRA_API int fra_plan_create_ranged(fra_ctx *ctx, const fra_job *job, const int32_t *frame_ranges, fra_plan **out);
FRA_API int fra_plan_set_raster(fra_plan *plan, const void *raster, int32_t raster_on_device);
FRA_API int fra_plan_execute(fra_plan *plan);
FRA_API int fra_plan_sync(fra_plan *plan);
/* after sync: per-window info (array of plan's nwindows) and total output bytes */
FRA_API int fra_plan_result(fra_plan *plan, fra_stream_info *infos, uint64_t *total_bytes);
/* after sync: copy the concatenated frames (total_bytes) to host memory */
FRA_API int fra_plan_download(fra_plan *plan, uint8_t *host_out, uint64_t capacity);
/* device pointer of the concatenated frames (valid until the next execute / destroy) */
FRA_API int fra_plan_device_output(fra_plan *plan, const uint8_t **dev_ptr, uint64_t *capacity);
/* after sync: byte offset of every frame of the concatenated output, frames of all windows in
 * window order; offsets[nframes] = total bytes.  n must be sum(infos[].nframes) + 1.  This is what
 * the pyflac-compatible shim needs to replay libFLAC's one-write-callback-per-frame sequence
 * (docs/sonos-pyflac.txt:2311-2332). */
FRA_API int fra_plan_frame_offsets(fra_plan *plan, uint64_t *offsets, uint64_t n);
/* per-kernel timing with HIP events on the plan's stream: 0 minmax, 1 analyze, 2 frame-bytes+scan, 3 pack */
FRA_API int fra_plan_enable_timing(fra_plan *plan, int32_t on);
FRA_API int fra_plan_timing(fra_plan *plan, float *ms_sum4, int32_t *executes);
FRA_API void fra_plan_destroy(fra_plan *plan);

/* Host-resident raster -> host-resident frames in one pipelined pass (the PCIe-inclusive path that
 * replaces rasterio read -> pyflac encode -> file write per tile, cli.py:553-602 / converter.py:73-154).
 * The windows are grouped into row bands; the raster rows of band b are copied H2D on a copy stream
 * while the kernels of band b-1 run on the plan's stream, and band b's frames are copied D2H on a
 * second copy stream as soon as they are assembled (PCIe is full duplex).  host_raster has the job's
 * dtype and strides; host_raster and host_out should be page-locked (fra_host_alloc/fra_host_register)
 * for full link rate.  Frames land at the offsets fra_plan_result reports; *total_bytes = their sum.
 * If capacity < total, FRA_E_SPACE is returned (frames beyond capacity are not copied; the complete
 * output stays on the device for fra_plan_download).  Synchronous: returns when the frames are in
 * host_out.  A plan's capacity bound: fra_plan_capacity. */
FRA_API int fra_plan_encode_host(fra_plan *plan, const void *host_raster, uint8_t *host_out, uint64_t capacity,
                                 uint64_t *total_bytes);
/* The same pipelined pass over a raster that is still being produced (file-to-container path: a decoder
 * thread fills host_raster top to bottom, cli.py:553-559 reads each tile's window before its encode):
 * before the H2D copy of a row band is enqueued, the call waits until *rows_ready >= the band's last row
 * + 1 (the producer publishes rows with a release store; -1 = the producer failed: FRA_E_STATE).  Rows
 * are image rows of the job's raster (row_stride units).  Contract: the producer MUST eventually publish
 * either every row or -1 (also when it fails or is cancelled); the call waits without a time limit. */
FRA_API int fra_plan_encode_host_progress(fra_plan *plan, const void *host_raster, uint8_t *host_out, uint64_t capacity,
                                          uint64_t *total_bytes, const volatile int64_t *rows_ready);
/* The same pass with BOUNDED host memory for the raster (r05): the producer decodes into a ring of
 * ring_rows rows per channel instead of the whole raster -- image row r of channel c lives at ring row
 * r % ring_rows, the ring laid out (channels, ring_rows, row_stride) in the job's dtype (row_stride and
 * col_stride as in the job; channel c at c * ring_rows * row_stride elements; pixel-interleaved jobs use
 * one run).  *rows_ready as above; the call publishes in *rows_done (release store) the rows whose H2D copy
 * has completed: the producer may write image row r once r < *rows_done + ring_rows.  ring_rows must hold
 * the tallest host band (fra_plan_host_band_rows) plus the producer's own step, else FRA_E_INVALID.
 * Replaces the reference's per-tile window read (cli.py:553-559), which also never holds the raster. */
FRA_API int fra_plan_encode_ring(fra_plan *plan, const void *ring, int64_t ring_rows, uint8_t *host_out,
                                 uint64_t capacity, uint64_t *total_bytes, const volatile int64_t *rows_ready,
                                 volatile int64_t *rows_done);
/* rows of the tallest host band of a plan (the ring of fra_plan_encode_ring must hold it) */
FRA_API int fra_plan_host_band_rows(fra_plan *plan, int64_t *max_rows);
/* frame number of every stream's first frame for the next execute (the job's first_frame until set) */
FRA_API int fra_plan_set_first_frame(fra_plan *plan, int32_t first_frame);
/* upper bound of a plan's output bytes (every subframe VERBATIM + headers) and its number of host bands */
FRA_API int fra_plan_capacity(fra_plan *plan, uint64_t *capacity, int32_t *host_bands);
/* how the plan encodes (FRA_PLAN_*): PIPELINED = executes overlap (two or three sets of subframe slots, the
 * next execute's normalisation stage and this one's assembly run beside k_analyze); WAVE = full frames are
 * analysed one subframe per wave (k_analyze_w), the partial ones by k_analyze
 * beside it; otherwise every subframe goes to the k_analyze workgroup kernel.  FRA_PLAN_DIRECT_WRITE is never
 * set (the direct-write path was measured slower than slots + k_assemble and removed in r03).  KEEP17 (with
 * WAVE) = the next execute's k_analyze_w keeps residuals up to 17 bits (else 16): a pipelined plan picks the
 * instance from how many waves of an earlier execute needed bit 16 (FRA_KEEP17=0/1 in the environment forces it);
 * both produce the same bytes. */
#define FRA_PLAN_DIRECT_WRITE 1
#define FRA_PLAN_PIPELINED 2
#define FRA_PLAN_WAVE 4
#define FRA_PLAN_KEEP17 8
FRA_API int fra_plan_flags(fra_plan *plan, int32_t *flags);

/* page-locked host memory (hipHostMalloc / hipHostRegister, portable across devices) */
FRA_API int fra_host_alloc(uint64_t bytes, void **host_ptr);
FRA_API int fra_host_free(void *host_ptr);
FRA_API int fra_host_register(void *host_ptr, uint64_t bytes);
FRA_API int fra_host_unregister(void *host_ptr);

/* One-shot convenience: plan, execute, download.  *out (malloc'ed, fra_free) receives the
 * concatenated frames; infos must hold job->nwindows entries. */
FRA_API int fra_encode(int device, const fra_job *job, uint8_t **out, uint64_t *out_len, fra_stream_info *infos);

/* fLaC + STREAMINFO(min=max blocksize, sizes 0, total samples 0, MD5 0) + VORBIS_COMMENT(vendor,
 * 0 comments, last) -- the 86-byte libFLAC 1.4.3 stream header layout. */
FRA_API int fra_stream_header(uint8_t *out86, int32_t channels, int32_t bps, int32_t sample_rate, int32_t blocksize);

/* normalize_to_audio (normalization.py:126-202) on the GPU for n elements of any dtype:
 * mn = nanmin, mx = nanmax unless overridden (data_min / data_max non-NULL), R = mx - mn or 1.0 if
 * mx <= mn, y = ((2.0*(x-mn))/R) - 1.0, clip[-1,1], NaN -> 0, then *32767 -> int16 (bps 16),
 * *8388607 -> int32 (bps 24), *2147483647 -> int32 (any other bps), truncating.
 * data: host or device (on_device) pointer; out_host: host buffer of n int16/int32.
 * mn_out/mx_out receive the (possibly NaN) min/max actually used. */
FRA_API int fra_normalize(fra_ctx *ctx, const void *data, int32_t on_device, int32_t dtype, uint64_t n, int32_t bps,
                          const double *data_min, const double *data_max, void *out_host, double *mn_out,
                          double *mx_out);

/* Native FLAC decoder (read side; replaces pyflac.FileDecoder at
 * converter.py:179-183): frame-parallel host decode of a complete stream (ID3v2 prefix allowed).
 * *samples (malloc'ed, fra_free) receives nsamples x channels interleaved int32.  With
 * FRA_DECODE_CONCAT, streams concatenated after the first one (the --spatial file layout,
 * spatial_encoder.py:196-245) are appended if their format matches. Every CRC-8/CRC-16 is
 * verified; a corrupt or truncated frame fails with FRA_E_INVALID. */
#define FRA_DECODE_CONCAT 1
typedef struct {
  int32_t sample_rate, channels, bps, blocksize; /* STREAMINFO (blocksize = max blocksize) */
  int64_t nframes;
  uint64_t nsamples;                             /* per channel */
  int32_t nstreams;
  uint64_t audio_offset;                         /* first frame byte of the first stream */
} fra_decoded;
FRA_API int fra_decode(const uint8_t *data, uint64_t len, int32_t flags, fra_decoded *info, int32_t **samples);

/* Synthetic rasters, generated on the device with integer-exact hashes so a
 * host numpy mirror reproduces any window bit for bit.  kind: 3 = C3 DEM int16, 4 = C4 S2-like
 * uint16 (4 bands), 5 = C5 reflectance float32.  dev_out: device buffer (bands, height, width). */
FRA_API int fra_synth_raster(fra_ctx *ctx, int32_t kind, uint64_t seed, int32_t bands, int32_t height, int32_t width,
                     void *dev_out);

/* GeoTIFF chunk decoder (host, multi-threaded; raster I/O ahead of the path, SURVEY.md 8(f) f3,
 * replacing rasterio's window reads at cli.py:559 / converter.py:73-79 / spatial_encoder.py:205-206).
 * The caller parses the IFD and lists the strips/tiles overlapping the window; each is decompressed
 * (none, LZW, deflate), un-predicted (1, 2 horizontal, 3 floating point) and its overlap with the
 * window written band-planar into dst (element (b, r, c) of the window at
 * b*dst_band_stride + r*dst_row_stride + c, native byte order).  threads <= 0: hardware concurrency. */
typedef struct {
  uint64_t offset, bytes;   /* compressed chunk within the file buffer */
  int32_t row0, col0;       /* image position of the chunk's first pixel */
  int32_t rows, cols;       /* chunk extent as stored (full tile, or strip rows x image width) */
  int32_t plane;            /* band of a planar (PlanarConfiguration 2) chunk; ignored when chunky */
  int32_t pad;
} fra_tiff_chunk;
typedef struct {
  int32_t compression;        /* 1, 5 (LZW), 8 or 32946 (deflate) */
  int32_t predictor;          /* 1, 2, 3 */
  int32_t bytes_per_sample;   /* 1, 2, 4, 8 */
  int32_t samples_per_pixel;  /* per chunk: SamplesPerPixel when chunky, 1 when planar */
  int32_t is_float;           /* SampleFormat 3 */
  int32_t big_endian;         /* MM file */
  int32_t bands;              /* bands of the destination */
  int32_t win_row, win_col, win_h, win_w;  /* destination window in image pixels */
  int32_t pad;
  int64_t dst_band_stride, dst_row_stride; /* elements */
} fra_tiff_layout;
FRA_API int fra_tiff_decode(const uint8_t *file, uint64_t file_len, const fra_tiff_layout *layout,
                            const fra_tiff_chunk *chunks, int32_t nchunks, void *dst, int32_t threads);

/* GeoTIFF chunk encoder (host, multi-threaded; the write side of the raster I/O, replacing rasterio's
 * tile GeoTIFF writes at cli.py:577-591 / converter.py flac_to_tiff): nchunks raw chunks of chunk_bytes
 * each, contiguous in src (already in file layout, predictor applied by the caller), are compressed with
 * compression 5 (TIFF LZW, MSB-first, early change -- what fra_tiff_decode and libtiff read) or 8 (zlib
 * deflate at `level`); chunk i goes to dst + i * dst_stride (dst_stride >= fra_tiff_compress_bound) and its
 * size to sizes[i]. */
FRA_API uint64_t fra_tiff_compress_bound(int32_t compression, uint64_t chunk_bytes);
FRA_API int fra_tiff_compress(int32_t compression, int32_t level, const uint8_t *src, uint64_t chunk_bytes,
                              int32_t nchunks, uint8_t *dst, uint64_t dst_stride, uint64_t *sizes, int32_t threads);

/* device memory helpers for hosts without a GPU array library */
FRA_API int fra_device_alloc(fra_ctx *ctx, uint64_t bytes, void **dev_ptr);
FRA_API int fra_device_free(fra_ctx *ctx, void *dev_ptr);
FRA_API int fra_memcpy_d2h(fra_ctx *ctx, void *dst, const void *src, uint64_t bytes);
FRA_API int fra_memcpy_h2d(fra_ctx *ctx, void *dst, const void *src, uint64_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* FLAC_RASTER_AMD_H */
