// fra_api.hip -- host orchestration + C ABI (include/flac_raster_amd.h) of the MI355X encoder.
//
// A plan owns every device buffer a job needs (raster copy if host-resident, stream/frame tables,
// window tables, subframe descriptors, frame sizes/offsets, output, scan workspace), so that
// fra_plan_execute() only enqueues kernels and events: no allocation, no host sync; the frame scan's
// ticket / epoch state lives on the device, not in launch arguments.  Per-job launch sequence (fra_kernels.hip):
//   k_norm_init, k_minmax, k_norm_finalize  (skipped when norm == 0)
//   k_analyze  [frames x channels]
//   k_frame_scan (frame sizes + decoupled look-back scan; k_group_offsets after a previous group)
//   k_assemble [frames]
// Large plans run as FRA_GROUPS frame groups on their own streams (fra_plan_execute).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <ctime>
#include <deque>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/flac_raster_amd.h"
#include "fra_internal.h"

namespace fra {
hipError_t launch_minmax(int src, const JobArgs& a, int nstreams, int max_segs, int vec_bytes, int rows, int max_rows,
                         hipStream_t s, int max_blocks);
hipError_t launch_norm_finalize(const JobArgs& a, int nstreams, hipStream_t s);
hipError_t launch_norm_lut(int src, const JobArgs& a, int nstreams, hipStream_t s);
hipError_t launch_analyze(int src, bool b32, bool ms, const JobArgs& a, hipStream_t s, bool wave, const int32_t* part,
                          int npart, int max_part_blocks, hipStream_t side, hipEvent_t ev_fork, hipEvent_t ev_join);
hipError_t launch_analyze_part(int src, bool b32, const JobArgs& a, const int32_t* part, int npart, int max_part_blocks,
                               hipStream_t s);
int frame_scan_blocks(int nframes);
hipError_t launch_frame_scan(const JobArgs& a, unsigned long long* gbase, int grp, int last, int add_base,
                             unsigned long long* host_mirror, unsigned long long* look2, int look_stride,
                             unsigned long long* ctl, hipStream_t s);
hipError_t launch_assemble(const JobArgs& a, hipStream_t s);
hipError_t launch_group_offsets(unsigned long long* frame_off, const unsigned long long* frame_bytes,
                                unsigned long long* gbase, int grp, int f0, int n, int last, int nframes,
                                hipStream_t s, unsigned long long* host_mirror = nullptr);
hipError_t launch_synth(int kind, uint64_t seed, int bands, int H, int W, void* out, hipStream_t s);
hipError_t launch_normalize_flat(int src, const void* data, uint64_t n, int bps, NormDev* nd, int has_min, double omin,
                                 int has_max, double omax, void* out, hipStream_t s);
}  // namespace fra

using namespace fra;

static thread_local std::string g_err;
static int set_err(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
#define HIPCHK(x)                                                                                \
  do {                                                                                           \
    hipError_t _e = (x);                                                                         \
    if (_e != hipSuccess) return set_err(FRA_E_HIP, "%s: %s (%s:%d)", #x, hipGetErrorString(_e), \
                                         __FILE__, __LINE__);                                    \
  } while (0)

struct fra_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // encode_host's D2H workers for pageable outputs: page-locked staging (stage_n pieces of 64 MiB) and one stream
  // per worker, kept across plans (the file path builds a plan per call); one encode at a time holds them
  std::mutex stage_mu;
  uint8_t* stage = nullptr;
  int stage_n = 0;
  std::vector<hipStream_t> stage_st;
};

// Pipelined execute: does the norm stage of execute k wait for the assembly of execute k-2 (one background kernel
// at a time beside the analysis)?  16-bit plans: no -- the norm stage then runs beside that assembly and the
// analysis of execute k-1 (C4 step 1.526 -> 1.497-1.504 ms, its 8-way shares -4 %, C3 -0.8 %); 32-bps plans:
// yes (C5 quarter +0.4 % without) -- profiles/r05_ab_bg_serial.txt.  FRA_BG_SERIAL=0/1 overrides (A/B)
static bool bg_serial(bool b32) {
  static const int v = getenv("FRA_BG_SERIAL") ? atoi(getenv("FRA_BG_SERIAL")) : -1;
  return v < 0 ? b32 : v == 1;
}

struct fra_plan {
  fra_ctx* ctx = nullptr;
  fra_job job{};
  std::vector<fra_window> windows;
  std::vector<int32_t> franges;  // fra_plan_create_ranged: [2 w] first frame, [2 w + 1] count (-1: to the end)
  std::vector<StreamDev> streams;
  std::vector<FrameDev> frames;
  int src = 0;
  bool b32 = false;
  int nwin = 0;
  int max_segs = 0;
  int mm_vec = 0, mm_rows = 1, mm_max_rows = 0;  // vectorised k_minmax shape (0 = scalar path)
  bool ld_vec8 = false;  // k_analyze 8-byte sample vectors possible (pointer alignment checked at execute)
  bool ld_off32 = false;  // k_analyze 32-bit lane offsets (JobArgs::off32)
  int cmax = 1;
  int ncu = 256;  // compute units of the device (background grids)
  size_t raster_bytes = 0;
  // device buffers
  void* d_raster_owned = nullptr;
  const void* d_raster = nullptr;
  StreamDev* d_streams = nullptr;
  FrameDev* d_frames = nullptr;
  NormDev* d_norm = nullptr;
  float* d_win = nullptr;
  int32_t* d_wrange = nullptr;
  int32_t* d_wplat = nullptr;
  // wave-path plans: the partial subframes k_analyze takes beside k_analyze_w (frame * 8 + channel, ascending;
  // a launch over frames [f0, f1) passes the entries in [8 f0, 8 f1))
  std::vector<int32_t> h_part;
  int32_t* d_part = nullptr;
  WaveDev* d_wave = nullptr;  // per-frame analysis descriptors (JobArgs::wave)
  bool wave_ok = false;
  hipStream_t pside = nullptr;  // the partial subframes' stream (beside k_analyze_w) and its fork / join
  hipEvent_t ev_pfork = nullptr, ev_pjoin = nullptr;
  // k_analyze_w instance (r05): kept residuals up to 17 bits or 16 (JobArgs::k17), picked per execute from how many
  // waves of an earlier execute needed bit 16.  Pipelined plans count into d_cnt17[j] (ring slot j of kCnt, never
  // reset: an execute's count is its snapshot minus the slot's previous one) and copy the counter into page-locked
  // h_cnt17[j] after the analysis; the host reads a snapshot once its event has completed (no sync)
  static constexpr int kCnt = 4;
  uint32_t* d_cnt17 = nullptr;
  uint32_t* h_cnt17 = nullptr;
  uint32_t cnt_base[kCnt] = {};
  hipEvent_t ev_cnt[kCnt] = {};
  bool cnt_pending[kCnt] = {};
  uint64_t cnt_seq[kCnt] = {};
  uint32_t cnt_sub[kCnt] = {};
  uint64_t cnt_next = 0, cnt_newest = 0;
  int cnt_cur = -1;  // the counter slot the last run_group launch counted into (-1: none)
  int k17 = 1;  // start with 17 bits: never slower than the sample path by more than its VGPR cost
  hipEvent_t ev_part[3] = {};  // pipelined: the partial subframes of buffer set b done (on the norm stream)
  SfDesc* d_sf = nullptr;
  unsigned long long* d_fbytes = nullptr;
  unsigned long long* d_foff = nullptr;
  uint8_t* d_out = nullptr;
  size_t out_cap = 0;
  // k_frame_scan look-back words and tickets per scan slot (frame group g: slot g; host bands and the
  // timing pass: slot 0) and, on the host, each slot's ticket base and launch tag (launches on one slot
  // are stream-ordered)
  unsigned long long* d_look = nullptr;
  uint32_t* d_err = nullptr;  // JobArgs::err (plan_sync_all)
  unsigned long long* d_ticket = nullptr;  // per scan slot: [63:32] epoch, [31:0] next ticket (k_frame_scan)
  int look_stride = 0;
  uint16_t* d_crctab = nullptr;
  uint32_t* d_tmp = nullptr;
  uint32_t* d_fmeta = nullptr;
  int32_t* d_lut = nullptr;
  int64_t tmp_stride = 0;
  JobArgs args{};
  // frame groups: contiguous window runs [w0, w1) with frames [f0, f1).  Group g > 0 runs on aux[g - 1]
  // (group 0 on the context stream) so one group's minmax/assemble overlaps another's k_analyze.
  struct Group { int w0, w1, f0, f1; };
  std::vector<Group> groups;            // pipelined execution (size 1 = serial)
  Group all{0, 0, 0, 0};                // the whole plan as one group (timing mode)
  std::vector<hipStream_t> aux;
  std::vector<hipEvent_t> gev;          // [0] start, then per group: offsets-published, done
  unsigned long long* d_gbase = nullptr;  // [max(groups, host bands) + 1] byte offset of each group's first frame
  // host pipeline (fra_plan_encode_host): row bands of windows; band b copies raster rows [r0, r1)
  // before its kernels run (rows already copied by earlier bands are not copied again)
  struct HBand { Group g; int64_t r0, r1; };
  std::vector<HBand> hbands;
  hipStream_t h2d = nullptr, d2h = nullptr;
  std::vector<hipEvent_t> hev;          // per band: rows copied, frames assembled (+ end offset mirrored)
  hipEvent_t hev_start = nullptr;
  unsigned long long* h_gbase = nullptr;  // page-locked mirror of d_gbase[1..bands]
  unsigned long long* d_gbase_mirror = nullptr;  // its device address
  // cross-execute pipelining (FRA_PIPE, default on when a second buffer set fits in a third of the free
  // device memory, single frame group): execute k analyses into slot set k % nslot on an analysis stream
  // while the frame-size chain + assembly of earlier executes (reading the other sets) run on the pack stream
  bool pipe = false;
  int cur = 0;  // buffer set of the last execute
  // slot sets (descriptors, encoded-subframe slots, frame sizes / offsets): nslot = 3 (execute k's analysis waits for
  // the assembly of execute k-3), or 2 when memory is short or FRA_SLOT_SETS=2; the analysis streams alternate by execute
  static constexpr int kSlotSets = 3;
  int nslot = 2;
  unsigned exec_n = 0;
  SfDesc* sf2[kSlotSets] = {};
  uint32_t* tmp2[kSlotSets] = {};
  uint32_t* fmeta2[kSlotSets] = {};
  unsigned long long* fbytes2[kSlotSets] = {};
  unsigned long long* foff2[kSlotSets] = {};
  hipStream_t pack = nullptr;
  // execute k's analysis runs on astream[k % 2] (highest priority): execute k+1's is queued on the other stream
  // than execute k's, so its first waves fill the CUs that execute k's tail leaves idle instead of waiting for
  // that kernel to end
  hipStream_t astream[2] = {};
  hipEvent_t ev_scan[kSlotSets] = {}, ev_pack[kSlotSets] = {};
  bool pack_pending[kSlotSets] = {};
  // ... and the normalisation stage (k_minmax -> k_norm_finalize -> k_norm_lut) of execute k+1 runs on
  // the norm stream under k_analyze of execute k.  k_analyze_w (4 waves of 8 KiB and 97 VGPRs per SIMD) leaves
  // 32 KiB of LDS and 96 VGPRs per SIMD beside it for the norm stage and the assembly; the 32-bps k_analyze (5
  // workgroups of 31.6 KiB) leaves none, so there they run in the gaps between analysis waves
  // norm sets (NormDev + table) cycle over kNormSets executes, the slot sets above over nslot (r05): execute k+1's norm
  // stage waits for execute k-2's analysis, not k-1's, so the norm stream runs up to a whole execute ahead and
  // execute k+1's table is ready before execute k's analysis drains (its waves fill that grid's last, partly empty
  // generation instead of waiting behind a k_minmax_vec that runs ~1.1 ms beside the analysis)
  static constexpr int kNormSets = 3;
  NormDev* norm2[kNormSets] = {};
  int32_t* lut2[kNormSets] = {};
  int curn = 0;  // norm set of the last pipelined execute
  hipEvent_t ev_nfree[kNormSets] = {};  // the last analysis (+ partial list) reading norm set n is done
  bool nfree_pending[kNormSets] = {};
  hipStream_t nstream = nullptr;
  hipEvent_t ev_norm[kSlotSets] = {}, ev_ana[kSlotSets] = {}, ev_raster = nullptr;
  bool ana_pending[kSlotSets] = {};
  bool raster_dirty = false;  // a host raster copy on the plan's stream the norm stream must wait for
  bool resync = false;        // serial work was queued on the plan's stream since the last pipelined execute
  // timing
  bool timing = false;
  hipEvent_t ev[5] = {};
  float ms[4] = {0, 0, 0, 0};
  int nexec = 0;
  bool pending_times = false;
  bool executed = false;
};

// ----------------------------------------------------------------------------- host helpers
static int elem_size(int dt) {
  switch (dt) {
    case FRA_U8: case FRA_I8: return 1;
    case FRA_U16: case FRA_I16: return 2;
    case FRA_U32: case FRA_I32: case FRA_F32: return 4;
    case FRA_F64: return 8;
  }
  return 0;
}
// normalization.py:108-120 (calculate_audio_params, total_pixels = H*W of the encode unit)
static int sample_rate_for_pixels(int64_t px) {
  if (px < 1000000) return 44100;
  if (px < 10000000) return 48000;
  if (px < 100000000) return 96000;
  return 192000;
}
// tukey(p) window as defined in DESIGN.md 3.4 (same formula as the oracle, computed on the host)
static void tukey(float* w, int N, double p) {
  for (int i = 0; i < N; i++) w[i] = 1.0f;
  int Np = (int)(p / 2.0 * (double)N) - 1;
  if (Np > 0) {
    for (int n = 0; n <= Np; n++) {
      w[n] = (float)(0.5 - 0.5 * cos(M_PI * (double)n / (double)Np));
      w[N - Np - 1 + n] = (float)(0.5 - 0.5 * cos(M_PI * (double)(n + Np) / (double)Np));
    }
  }
}
static void window_set(float* w, int N, int stride, int nsub) {
  if (nsub <= 0) return;
  tukey(w, N, 0.5);
  int idx = 1;
  for (int m = 2; m <= nsub; m++)
    for (int j = 0; j < m; j++, idx++) {
      float* o = w + (size_t)idx * stride;
      const int a = (int)((int64_t)j * N / m), b = (int)((int64_t)(j + 1) * N / m);
      for (int i = 0; i < N; i++) o[i] = 0.0f;
      if (b - a > 0) tukey(o + a, b - a, 0.5);
    }
}

// CRC-16 (poly x^16+x^15+x^2+1) tables for k_crc16: slice-by-4 byte tables T[k][v] = CRC of v
// followed by k zero bytes, and M[i][0|1][b] = b * x^(8*2^i) (resp. b*x^8*x^(8*2^i)) mod P.
static uint32_t gf16_mul(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int i = 15; i >= 0; i--) {
    r <<= 1;
    if (r & 0x10000u) r ^= 0x18005u;
    if ((b >> i) & 1u) r ^= a;
  }
  return r & 0xFFFFu;
}
static std::vector<uint16_t> crc16_tables() {
  std::vector<uint16_t> tab(kCrcT16Off + 16 * 256);
  for (int v = 0; v < 256; v++) {
    uint32_t d = (uint32_t)v << 8;
    for (int b = 0; b < 8; b++) d = (d & 0x8000u) ? ((d << 1) ^ 0x8005u) : (d << 1);
    tab[v] = (uint16_t)d;
  }
  for (int k = 1; k < 4; k++)
    for (int v = 0; v < 256; v++) {
      const uint32_t p = tab[(k - 1) * 256 + v];
      tab[k * 256 + v] = (uint16_t)(((p << 8) & 0xFFFFu) ^ tab[p >> 8]);
    }
  for (int k = 0; k < 16; k++)  // slice-by-16 (k_assemble): T16[k] = T[k] for k < 4
    for (int v = 0; v < 256; v++) {
      if (k == 0) { tab[kCrcT16Off + v] = tab[v]; continue; }
      const uint32_t p = tab[kCrcT16Off + (k - 1) * 256 + v];
      tab[kCrcT16Off + k * 256 + v] = (uint16_t)(((p << 8) & 0xFFFFu) ^ tab[p >> 8]);
    }
  uint32_t X = 0x100;  // x^8
  for (int i = 0; i < 24; i++) {
    for (int b = 0; b < 256; b++) {
      tab[1024 + i * 512 + b] = (uint16_t)gf16_mul((uint32_t)b, X);
      tab[1024 + i * 512 + 256 + b] = (uint16_t)gf16_mul(gf16_mul((uint32_t)b, 0x100), X);
    }
    X = gf16_mul(X, X);
  }
  return tab;
}

static const char kVendor[] = "flac-raster-amd 0.1.0 gfx950 HIP";  // 32 bytes, as libFLAC's vendor string

extern "C" {

int fra_internal_set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

const char* fra_last_error(void) { return g_err.c_str(); }
int fra_abi_version(void) { return FRA_ABI_VERSION; }
void fra_free(void* p) { free(p); }

int fra_device_count(int* count) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *count = n;
  return FRA_OK;
}

int fra_ctx_create(int device, fra_ctx** out) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return set_err(FRA_E_NODEVICE, "no HIP device visible");
  if (device < 0 || device >= n) return set_err(FRA_E_INVALID, "device %d out of range (%d devices)", device, n);
  HIPCHK(hipSetDevice(device));
  fra_ctx* c = new (std::nothrow) fra_ctx();
  if (!c) return set_err(FRA_E_NOMEM, "out of host memory");
  c->device = device;
  // the highest stream priority: background kernels of pipelined plans (low-priority streams) fill the
  // CU resources k_analyze leaves free rather than competing for them
  int lo = 0, hi = 0;
  if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
  hipError_t e = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi);
  if (e != hipSuccess) { delete c; return set_err(FRA_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e)); }
  *out = c;
  return FRA_OK;
}

void fra_ctx_destroy(fra_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  for (auto st : c->stage_st) (void)hipStreamDestroy(st);
  if (c->stage) (void)hipHostFree(c->stage);
  delete c;
}

void fra_plan_destroy(fra_plan* p) {
  if (!p) return;
  (void)hipSetDevice(p->ctx->device);
  (void)hipFree(p->d_raster_owned);
  (void)hipFree(p->d_streams);
  (void)hipFree(p->d_frames);
  if (!p->pipe) (void)hipFree(p->d_norm);
  (void)hipFree(p->d_win);
  (void)hipFree(p->d_wrange);
  (void)hipFree(p->d_wplat);
  (void)hipFree(p->d_part);
  (void)hipFree(p->d_wave);
  if (p->pside) (void)hipStreamDestroy(p->pside);
  if (p->ev_pfork) (void)hipEventDestroy(p->ev_pfork);
  if (p->ev_pjoin) (void)hipEventDestroy(p->ev_pjoin);
  for (auto e : p->ev_part)
    if (e) (void)hipEventDestroy(e);
  if (p->pipe) {  // d_* alias set 0 or 1: free both sets through the arrays
    for (int b = 0; b < fra_plan::kSlotSets; b++) {
      (void)hipFree(p->sf2[b]);
      (void)hipFree(p->fbytes2[b]);
      (void)hipFree(p->foff2[b]);
      (void)hipFree(p->tmp2[b]);
      (void)hipFree(p->fmeta2[b]);
    }
    for (int n = 0; n < fra_plan::kNormSets; n++) {
      (void)hipFree(p->norm2[n]);
      (void)hipFree(p->lut2[n]);
      if (p->ev_nfree[n]) (void)hipEventDestroy(p->ev_nfree[n]);
    }
    p->d_sf = nullptr; p->d_fbytes = nullptr; p->d_foff = nullptr; p->d_tmp = nullptr; p->d_fmeta = nullptr;
    p->d_norm = nullptr; p->d_lut = nullptr;
  }
  if (p->pack) (void)hipStreamDestroy(p->pack);
  if (p->nstream) (void)hipStreamDestroy(p->nstream);
  for (auto& st : p->astream)
    if (st) (void)hipStreamDestroy(st);
  for (int b = 0; b < fra_plan::kSlotSets; b++) {
    if (p->ev_scan[b]) (void)hipEventDestroy(p->ev_scan[b]);
    if (p->ev_pack[b]) (void)hipEventDestroy(p->ev_pack[b]);
    if (p->ev_norm[b]) (void)hipEventDestroy(p->ev_norm[b]);
    if (p->ev_ana[b]) (void)hipEventDestroy(p->ev_ana[b]);
  }
  if (p->ev_raster) (void)hipEventDestroy(p->ev_raster);
  (void)hipFree(p->d_sf);
  (void)hipFree(p->d_fbytes);
  (void)hipFree(p->d_foff);
  (void)hipFree(p->d_out);
  (void)hipFree(p->d_look);
  (void)hipFree(p->d_ticket);
  (void)hipFree(p->d_err);
  (void)hipFree(p->d_crctab);
  (void)hipFree(p->d_tmp);
  (void)hipFree(p->d_fmeta);
  if (!p->pipe) (void)hipFree(p->d_lut);
  (void)hipFree(p->d_gbase);
  for (auto& st : p->aux)
    if (st) (void)hipStreamDestroy(st);
  if (p->h2d) (void)hipStreamDestroy(p->h2d);
  if (p->d2h) (void)hipStreamDestroy(p->d2h);
  for (auto& e : p->hev)
    if (e) (void)hipEventDestroy(e);
  if (p->hev_start) (void)hipEventDestroy(p->hev_start);
  if (p->h_gbase) (void)hipHostFree(p->h_gbase);
  if (p->h_cnt17) (void)hipHostFree(p->h_cnt17);
  (void)hipFree(p->d_cnt17);
  for (auto e : p->ev_cnt)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : p->gev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : p->ev)
    if (e) (void)hipEventDestroy(e);
  delete p;
}

// Row bands for the host pipeline: runs of windows sharing a row offset (a row of tiles), merged until a
// band holds >= 1/16 of the frames (one band for small plans, where launch latency dominates).  Band b
// copies the raster rows its windows cover that no earlier band copied; if the windows' row ranges are
// not monotone the plan falls back to one band covering every row.
static void build_host_bands(fra_plan* p, int nfr) {
  p->hbands.clear();
  const int ns = (int)p->streams.size();
  if (ns == 0) return;
  const int64_t min_frames = nfr < 2048 ? (int64_t)nfr + 1 : std::max<int64_t>(1, nfr / 16);
  std::vector<fra_plan::Group> bands;
  int w = 0, f = 0;
  while (w < ns) {
    fra_plan::Group g{w, w, f, f};
    while (w < ns && (g.f1 - g.f0 < min_frames || g.w1 == g.w0)) {
      const int r = p->windows[w].row_off;
      while (w < ns && p->windows[w].row_off == r) {  // a whole row of windows
        f += p->streams[w].nframes;
        w++;
      }
      g.w1 = w;
      g.f1 = f;
    }
    bands.push_back(g);
  }
  if (bands.size() > 1 && bands.back().f1 - bands.back().f0 < min_frames / 2) {  // fold a small tail band
    bands[bands.size() - 2].w1 = bands.back().w1;
    bands[bands.size() - 2].f1 = bands.back().f1;
    bands.pop_back();
  }
  int64_t lo_all = INT64_MAX, hi_all = 0, prev_lo = -1, hi = 0;
  bool mono = true;
  for (const auto& g : bands) {
    int64_t lo = INT64_MAX, hb = 0;
    for (int k = g.w0; k < g.w1; k++)
      if (p->streams[k].nsamples > 0) {
        lo = std::min<int64_t>(lo, p->windows[k].row_off);
        hb = std::max<int64_t>(hb, (int64_t)p->windows[k].row_off + p->windows[k].height);
      }
    if (lo == INT64_MAX) { lo = hi; hb = hi; }
    if (lo < prev_lo) mono = false;
    prev_lo = lo;
    lo_all = std::min(lo_all, lo);
    hi_all = std::max(hi_all, hb);
    p->hbands.push_back({g, std::max(lo, hi), std::max(std::max(lo, hi), hb)});
    hi = std::max(hi, hb);
  }
  if (!mono) {
    p->hbands.clear();
    p->hbands.push_back({p->all, lo_all == INT64_MAX ? 0 : lo_all, hi_all});
  }
}

static int plan_build(fra_plan* p) {
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, p->ctx->device) == hipSuccess && ncu > 0)
      p->ncu = ncu;
  }
  const fra_job& j = p->job;
  p->src = j.dtype;
  const int nsub = level_cfg(j.level).nsub;
  p->nwin = num_windows(nsub);
  int bps;
  if (j.norm == 16) bps = 16;
  else if (j.norm == 24) bps = 32;  // int32 audio -> 32-bps FLAC
  else bps = (j.dtype == FRA_I16 || j.dtype == FRA_U8 || j.dtype == FRA_I8) ? 16 : 32;
  p->b32 = bps == 32;
  // FRA-1 3.1b mid-side for 2-channel 16-bps streams at the levels whose libFLAC preset enables it:
  // four virtual channels (L, R, M, S) are analysed per frame, k_frame_scan keeps the cheapest pair
  const bool ms = j.channels == 2 && bps == 16 && level_cfg(j.level).ms;
  p->cmax = ms ? 4 : j.channels;
  const int sbps_max = ms ? bps + 1 : bps;  // side samples carry one more bit
  p->streams.clear();
  p->frames.clear();
  std::map<int, int> win_index;  // block size -> window table index
  std::vector<int> win_sizes;
  int64_t nf_total = 0;
  int64_t max_extent = 0;
  size_t out_cap = 0;
  for (int w = 0; w < j.nwindows; w++) {
    const fra_window& wd = p->windows[w];
    StreamDev st{};
    st.base_off = (int64_t)wd.row_off * j.row_stride + (int64_t)wd.col_off * j.col_stride;
    st.band_stride = j.band_stride;
    st.row_stride = j.row_stride;
    st.col_stride = j.col_stride;
    st.width = wd.width;
    st.height = wd.height;
    st.channels = j.channels;
    st.bps = bps;
    st.norm = j.norm;
    st.nsamples = (int64_t)wd.width * wd.height;
    st.sample_rate = j.sample_rate > 0 ? j.sample_rate : sample_rate_for_pixels(st.nsamples);
    st.first_frame = (int32_t)nf_total;
    st.frame_number0 = (uint32_t)j.first_frame;
    st.ms = ms ? 1 : 0;
    const int64_t nfr_all = (st.nsamples + j.blocksize - 1) / j.blocksize;
    // frame range of this window (fra_plan_create_ranged): frames [fa, fa + nfr) of its stream; the
    // normalisation still spans the whole window, frame numbers stay those of the whole stream
    int64_t fa = 0, nfr = nfr_all;
    if (!p->franges.empty()) {
      fa = std::min<int64_t>(p->franges[2 * w], nfr_all);
      nfr = p->franges[2 * w + 1] < 0 ? nfr_all - fa : std::min<int64_t>(p->franges[2 * w + 1], nfr_all - fa);
    }
    st.nframes = (int32_t)nfr;
    if (st.nsamples > 0) {
      int64_t ext = st.base_off + (int64_t)(j.channels - 1) * j.band_stride + (int64_t)(wd.height - 1) * j.row_stride +
                    (int64_t)(wd.width - 1) * j.col_stride + 1;
      max_extent = std::max(max_extent, ext);
      const int segs = (wd.width + 4095) / 4096;
      p->max_segs = (int)std::max<int64_t>(p->max_segs, (int64_t)segs * wd.height);
    }
    for (int64_t f = fa; f < fa + nfr; f++) {
      FrameDev fr{};
      fr.stream = w;
      fr.index = (int32_t)f;
      const int64_t first = f * j.blocksize;
      fr.n = (int32_t)std::min<int64_t>(j.blocksize, st.nsamples - first);
      fr.row0 = (int32_t)(first / wd.width);
      fr.col0 = (int32_t)(first % wd.width);
      auto it = win_index.find(fr.n);
      if (it == win_index.end()) {
        int idx = (int)win_sizes.size();
        win_index[fr.n] = idx;
        win_sizes.push_back(fr.n);
        fr.win = idx;
      } else fr.win = it->second;
      p->frames.push_back(fr);
      out_cap += 16 + 2 + (size_t)j.channels * ((size_t)fr.n * sbps_max / 8 + 8);
    }
    nf_total += nfr;
    p->streams.push_back(st);
  }
  // vectorised min/max: every window start, row, band and width a multiple of V = vec/itemsize
  p->mm_vec = 0;
  if (j.norm != 0 && j.col_stride == 1 && elem_size(j.dtype) <= 4) {
    for (int vb : {16, 8}) {
      const int64_t V = vb / elem_size(j.dtype);
      bool ok = V >= 2 && j.row_stride % V == 0 && (j.channels == 1 || j.band_stride % V == 0);
      int64_t max_nv = 1;
      for (int w = 0; ok && w < j.nwindows; w++) {
        const StreamDev& st = p->streams[w];
        if (st.nsamples == 0) continue;
        ok = st.base_off % V == 0 && st.width % V == 0 && st.width / V <= 65535;
        max_nv = std::max<int64_t>(max_nv, st.width / V);
      }
      if (!ok) continue;
      const int64_t rows = std::max<int64_t>(1, std::min<int64_t>(64, 2048 / max_nv));
      if (rows * max_nv * max_nv >= (int64_t(1) << 32)) continue;
      if (rows * j.row_stride * elem_size(j.dtype) >= (int64_t(1) << 32)) continue;  // 32-bit byte offsets
      p->mm_vec = vb;
      p->mm_rows = (int)rows;
      p->mm_max_rows = 0;
      for (const StreamDev& st : p->streams) p->mm_max_rows = std::max(p->mm_max_rows, (int)st.height);
      break;
    }
  }
  // k_analyze 8-byte sample vectors: V = 8/itemsize samples never straddle a row and stay aligned
  {
    const int64_t V = 8 / std::max(1, elem_size(j.dtype));
    bool ok = elem_size(j.dtype) <= 4 && j.col_stride == 1 && j.blocksize % V == 0 && j.row_stride % V == 0 &&
              (j.channels == 1 || j.band_stride % V == 0);
    for (int w = 0; ok && w < j.nwindows; w++) {
      const StreamDev& st = p->streams[w];
      if (st.nsamples) ok = st.base_off % V == 0 && st.width % V == 0;
    }
    p->ld_vec8 = ok;
    // 32-bit lane offsets of the fast load path: a frame's rows of one channel span < 2^31 bytes
    bool o32 = j.row_stride >= 0;
    for (int w = 0; o32 && w < j.nwindows; w++) {
      const StreamDev& st = p->streams[w];
      if (!st.nsamples) continue;
      const int64_t rows = (j.blocksize + st.width - 1) / st.width + 1;
      o32 = (rows * j.row_stride + st.width) * elem_size(j.dtype) < (int64_t(1) << 31);
    }
    p->ld_off32 = o32;
  }
  if (nf_total > INT32_MAX / 2) return set_err(FRA_E_INVALID, "too many frames (%lld)", (long long)nf_total);
  p->raster_bytes = (size_t)max_extent * elem_size(j.dtype);
  p->out_cap = out_cap + 64;
  const int nfr = (int)nf_total;
  (void)hipSetDevice(p->ctx->device);
  HIPCHK(hipMalloc(&p->d_streams, sizeof(StreamDev) * std::max<size_t>(1, p->streams.size())));
  HIPCHK(hipMalloc(&p->d_frames, sizeof(FrameDev) * std::max(1, nfr)));
  HIPCHK(hipMalloc(&p->d_norm, sizeof(NormDev) * std::max<size_t>(1, p->streams.size())));
  HIPCHK(hipMalloc(&p->d_sf, sizeof(SfDesc) * (size_t)std::max(1, nfr) * p->cmax));
  HIPCHK(hipMalloc(&p->d_fbytes, sizeof(unsigned long long) * (nfr + 1)));
  HIPCHK(hipMalloc(&p->d_foff, sizeof(unsigned long long) * (nfr + 1)));
  HIPCHK(hipMalloc(&p->d_out, p->out_cap));
  const size_t wn = (size_t)std::max<size_t>(1, win_sizes.size()) * std::max(1, p->nwin) * j.blocksize;
  // exact size: k_analyze reads entries [0, n) of the table of block size n only (load_window)
  // + slack: k_analyze_w reads a whole chunk's look-ahead of coefficients without a bound (its samples past n
  // are zero), which may run 16 + MAXLAG entries past the last row
  std::vector<float> wt(wn + 64, 0.0f);
  for (size_t t = 0; t < win_sizes.size(); t++)
    window_set(wt.data() + t * std::max(1, p->nwin) * j.blocksize, win_sizes[t], j.blocksize, nsub);
  HIPCHK(hipMalloc(&p->d_win, sizeof(float) * wt.size()));
  HIPCHK(hipMemcpy(p->d_win, wt.data(), sizeof(float) * wt.size(), hipMemcpyHostToDevice));
  {  // nonzero extent [lo, hi) of every window (k_analyze: waves outside it skip the autocorrelation)
    const int nw = std::max(1, p->nwin), nt = (int)std::max<size_t>(1, win_sizes.size());
    std::vector<int32_t> wr(2 * (size_t)nt * nw, 0);
    for (int t = 0; t < nt; t++)
      for (int w = 0; w < nw; w++) {
        const float* o = wt.data() + ((size_t)t * nw + w) * j.blocksize;
        int lo = j.blocksize, hi = 0;
        for (int i = 0; i < j.blocksize; i++)
          if (o[i] != 0.0f) { lo = std::min(lo, i); hi = i + 1; }
        wr[2 * ((size_t)t * nw + w)] = lo < hi ? lo : 0;
        wr[2 * ((size_t)t * nw + w) + 1] = lo < hi ? hi : 0;
      }
    HIPCHK(hipMalloc(&p->d_wrange, sizeof(int32_t) * wr.size()));
    HIPCHK(hipMemcpy(p->d_wrange, wr.data(), sizeof(int32_t) * wr.size(), hipMemcpyHostToDevice));
    // longest run of coefficients exactly 1.0f (the tukey plateau): its products are the samples themselves
    std::vector<int32_t> wp(2 * (size_t)nt * nw, 0);
    for (int t = 0; t < nt; t++)
      for (int w = 0; w < nw; w++) {
        const float* o = wt.data() + ((size_t)t * nw + w) * j.blocksize;
        int best = 0, blo = 0, run = 0;
        for (int i = 0; i < j.blocksize; i++) {
          run = o[i] == 1.0f ? run + 1 : 0;
          if (run > best) { best = run; blo = i + 1 - run; }
        }
        wp[2 * ((size_t)t * nw + w)] = blo;
        wp[2 * ((size_t)t * nw + w) + 1] = blo + best;
      }
    HIPCHK(hipMalloc(&p->d_wplat, sizeof(int32_t) * wp.size()));
    HIPCHK(hipMemcpy(p->d_wplat, wp.data(), sizeof(int32_t) * wp.size(), hipMemcpyHostToDevice));
  }
  if (!p->streams.empty())
    HIPCHK(hipMemcpy(p->d_streams, p->streams.data(), sizeof(StreamDev) * p->streams.size(), hipMemcpyHostToDevice));
  if (nfr) HIPCHK(hipMemcpy(p->d_frames, p->frames.data(), sizeof(FrameDev) * nfr, hipMemcpyHostToDevice));
  {  // per-frame analysis descriptors (WaveDev: the load phase's metadata in one scalar load)
    std::vector<WaveDev> wv(std::max(1, nfr));
    for (int g = 0; g < nfr; g++) {
      const FrameDev& fr = p->frames[g];
      const StreamDev& st = p->streams[fr.stream];
      WaveDev& w = wv[g];
      w.off0 = st.base_off + (int64_t)fr.row0 * st.row_stride;
      w.band_stride = st.band_stride;
      w.row_stride = (uint32_t)st.row_stride;
      w.width = (uint32_t)st.width;
      w.col0 = (uint32_t)fr.col0;
      w.stream = fr.stream;
      w.n = fr.n;
      w.win = fr.win;
      w.bps = st.bps;
      w.nch = st.ms ? 2 : st.channels;
      w.channels = st.channels;
      w.ms = st.ms;
      w.norm = st.norm;
    }
    HIPCHK(hipMalloc(&p->d_wave, sizeof(WaveDev) * wv.size()));
    HIPCHK(hipMemcpy(p->d_wave, wv.data(), sizeof(WaveDev) * wv.size(), hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemset(p->d_norm, 0, sizeof(NormDev) * std::max<size_t>(1, p->streams.size())));
  // frame groups: FRA_GROUPS (default 1: measured no gain on C4) contiguous window runs of about equal frame count;
  // one group for small plans, where launch latency dominates
  {
    int G = 1;
    if (const char* ev = getenv("FRA_GROUPS")) G = std::max(1, std::min(8, atoi(ev)));
    if (nfr < 4096) G = 1;
    p->all = {0, (int)p->streams.size(), 0, nfr};
    p->groups.clear();
    int w = 0, f = 0;
    for (int g = 0; g < G && w < (int)p->streams.size(); g++) {
      const int64_t target = (int64_t)nfr * (g + 1) / G;
      fra_plan::Group gr{w, w, f, f};
      while (w < (int)p->streams.size() && (g == G - 1 || f < target || gr.f1 == gr.f0)) {
        f += p->streams[w].nframes;
        w++;
        gr.w1 = w;
        gr.f1 = f;
      }
      p->groups.push_back(gr);
    }
    if (p->groups.empty()) p->groups.push_back(p->all);
    p->groups.back().w1 = (int)p->streams.size();
    p->groups.back().f1 = nfr;
    build_host_bands(p, nfr);
    // look-back words (zero: no tag yet) and tickets of every scan slot, sized for the whole plan
    const int nslot = (int)p->groups.size();
    // any group of <= nfr frames needs <= 256 words by default, or nfr's count (one frame per thread when forced)
    p->look_stride = std::max({256, frame_scan_blocks(nfr), (nfr + 255) / 256});
    HIPCHK(hipMalloc(&p->d_look, sizeof(unsigned long long) * (size_t)p->look_stride * 2 * nslot));
    HIPCHK(hipMemset(p->d_look, 0, sizeof(unsigned long long) * (size_t)p->look_stride * 2 * nslot));
    HIPCHK(hipMalloc(&p->d_ticket, sizeof(unsigned long long) * nslot));
    HIPCHK(hipMemset(p->d_ticket, 0, sizeof(unsigned long long) * nslot));
    HIPCHK(hipMalloc(&p->d_err, sizeof(uint32_t)));
    HIPCHK(hipMemset(p->d_err, 0, sizeof(uint32_t)));
    p->args.err = p->d_err;
    HIPCHK(hipMalloc(&p->d_gbase, sizeof(unsigned long long) * (std::max(p->groups.size(), p->hbands.size()) + 1)));
    for (size_t g = 1; g < p->groups.size(); g++) {
      hipStream_t st = nullptr;
      HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      p->aux.push_back(st);
    }
    if (j.blocksize == kMaxBlock && ((!p->b32 && j.level >= 3 && j.level <= 6 && j.norm != 0 &&
                                      elem_size(j.dtype) <= 2 && j.dtype != FRA_F64) ||
                                     (p->b32 && j.level >= 7 && j.norm == 24 && j.dtype == FRA_F32 &&
                                      j.channels == p->cmax))) {  // plans k_analyze_w may take (wave_path)
      // the partial subframes (frame * 8 + channel, ascending): k_analyze's share of a wave-path launch
      p->h_part.clear();
      for (int g = 0; g < nfr; g++) {
        const FrameDev& fr = p->frames[g];
        if (fr.n == j.blocksize) continue;
        const StreamDev& st = p->streams[fr.stream];
        for (int c = 0; c < (st.ms ? 2 : st.channels); c++) p->h_part.push_back(g * 8 + c);
      }
      HIPCHK(hipMalloc(&p->d_part, sizeof(int32_t) * std::max<size_t>(1, p->h_part.size())));
      if (!p->h_part.empty())
        HIPCHK(hipMemcpy(p->d_part, p->h_part.data(), sizeof(int32_t) * p->h_part.size(), hipMemcpyHostToDevice));
      p->wave_ok = true;
      if (!p->h_part.empty()) {
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&p->pside, hipStreamNonBlocking, hi));
        HIPCHK(hipEventCreateWithFlags(&p->ev_pfork, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&p->ev_pjoin, hipEventDisableTiming));
      }
    }
    p->gev.assign(1 + 2 * p->groups.size(), nullptr);
    for (auto& e : p->gev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  // per-subframe slots for the encoded subframes (k_analyze -> k_assemble)
  p->tmp_stride = ((int64_t)j.blocksize * sbps_max + 64 + 31) / 32 + 4;
  HIPCHK(hipMalloc(&p->d_tmp, sizeof(uint32_t) * (size_t)p->tmp_stride * std::max(1, nfr) * p->cmax));
  HIPCHK(hipMalloc(&p->d_fmeta, sizeof(uint32_t) * kMetaWords * std::max(1, nfr)));
  {
    const std::vector<uint16_t> ct = crc16_tables();
    HIPCHK(hipMalloc(&p->d_crctab, sizeof(uint16_t) * ct.size()));
    HIPCHK(hipMemcpy(p->d_crctab, ct.data(), sizeof(uint16_t) * ct.size(), hipMemcpyHostToDevice));
  }
  // normalisation tables for <= 16-bit integer rasters (k_norm_lut -> gathered by k_analyze)
  int64_t lut_stride = 0;
  if (j.norm != 0 && (j.dtype == FRA_U8 || j.dtype == FRA_I8 || j.dtype == FRA_U16 || j.dtype == FRA_I16) &&
      !p->streams.empty()) {
    lut_stride = elem_size(j.dtype) == 1 ? 256 : 65536;
    HIPCHK(hipMalloc(&p->d_lut, sizeof(int32_t) * (size_t)lut_stride * p->streams.size()));
  }
  JobArgs& a = p->args;
  a.streams = p->d_streams;
  a.frames = p->d_frames;
  a.wave = p->d_wave;
  a.norm = p->d_norm;
  a.win = p->d_win;
  a.wrange = p->d_wrange;
  a.wplat = p->d_wplat;
  a.sf = p->d_sf;
  a.frame_bytes = p->d_fbytes;
  a.frame_off = p->d_foff;
  a.out = p->d_out;
  a.crctab = p->d_crctab;
  a.tmp = p->d_tmp;
  a.fmeta = p->d_fmeta;
  a.err = p->d_err;
  a.out_cap = p->out_cap;
  a.tmp_stride = p->tmp_stride;
  a.lut = p->d_lut;
  a.lut_stride = lut_stride;
  a.nframes_total = nfr;
  a.cmax = p->cmax;
  a.blocksize = j.blocksize;
  a.level = j.level;
  a.nwin = std::max(1, p->nwin);
  a.off32 = p->ld_off32 ? 1 : 0;
  for (auto& e : p->ev) HIPCHK(hipEventCreate(&e));
  {  // second buffer set for cross-execute pipelining
    const char* ev = getenv("FRA_PIPE");
    // large plans only (>= 1024 frames: a C4 scene split 8 ways, ~3.7k frames per rank, stays
    // pipelined); small ones (the pyflac shim, single tiles) execute once per plan
    static const int min_frames = getenv("FRA_PIPE_MIN_FRAMES") ? atoi(getenv("FRA_PIPE_MIN_FRAMES")) : 1024;
    const bool want = !(ev && atoi(ev) == 0) && p->groups.size() == 1 && nfr >= min_frames;
    const size_t nsf = (size_t)nfr * p->cmax;
    const size_t nst = std::max<size_t>(1, p->streams.size());
    const size_t extra = sizeof(SfDesc) * nsf + sizeof(uint32_t) * (size_t)p->tmp_stride * nsf +
                         sizeof(uint32_t) * kMetaWords * nfr + 2 * sizeof(unsigned long long) * (nfr + 1) +
                         (fra_plan::kNormSets - 1) * (sizeof(NormDev) * nst + (p->d_lut ? sizeof(int32_t) * (size_t)lut_stride * nst : 0));
    size_t freeb = 0, totalb = 0;
    if (want && hipMemGetInfo(&freeb, &totalb) == hipSuccess && extra <= freeb / 3) {
      p->sf2[0] = p->d_sf; p->tmp2[0] = p->d_tmp; p->fmeta2[0] = p->d_fmeta;
      p->fbytes2[0] = p->d_fbytes; p->foff2[0] = p->d_foff;
      p->norm2[0] = p->d_norm; p->lut2[0] = p->d_lut;
      p->pipe = true;  // from here on destroy frees through the arrays
      for (int n = 1; n < fra_plan::kNormSets; n++) {
        HIPCHK(hipMalloc(&p->norm2[n], sizeof(NormDev) * nst));
        HIPCHK(hipMemset(p->norm2[n], 0, sizeof(NormDev) * nst));
        if (p->d_lut) HIPCHK(hipMalloc(&p->lut2[n], sizeof(int32_t) * (size_t)lut_stride * nst));
      }
      for (auto& e : p->ev_nfree) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      {  // background streams at the lowest priority (the plan's stream is created at the highest)
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&p->nstream, hipStreamNonBlocking, lo));
      }
      HIPCHK(hipEventCreateWithFlags(&p->ev_raster, hipEventDisableTiming));
      {
        // three slot sets by default (r05: with the 16-bit k_analyze_w instance C4 neutral, its 8-way share -4.6 %, C3
        // -2.3 %, C5 quarter -0.7 %, profiles/r05_ab_background.txt) when twice the extra set fits a third of the free
        // memory; FRA_SLOT_SETS=2 (A/B) keeps two
        static const int want3 = getenv("FRA_SLOT_SETS") ? atoi(getenv("FRA_SLOT_SETS")) : 3;
        size_t f2 = 0, t2 = 0;
        p->nslot = (want3 == 3 && hipMemGetInfo(&f2, &t2) == hipSuccess && 2 * extra <= f2 / 3) ? 3 : 2;
      }
      for (int b = 1; b < p->nslot; b++) {
        HIPCHK(hipMalloc(&p->sf2[b], sizeof(SfDesc) * std::max<size_t>(1, nsf)));
        HIPCHK(hipMalloc(&p->tmp2[b], sizeof(uint32_t) * (size_t)p->tmp_stride * std::max<size_t>(1, nsf)));
        HIPCHK(hipMalloc(&p->fmeta2[b], sizeof(uint32_t) * kMetaWords * nfr));
        HIPCHK(hipMalloc(&p->fbytes2[b], sizeof(unsigned long long) * (nfr + 1)));
        HIPCHK(hipMalloc(&p->foff2[b], sizeof(unsigned long long) * (nfr + 1)));
      }
      {
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&p->pack, hipStreamNonBlocking, lo));
        // 16-bit plans: C4 -1.2 %, C3 -2.4 % (r03 v14); 32-bps plans too since the background assembly that the
        // early start displaced is gone (r03: C5 +5 % with it; r04: C5 106.50 -> 106.24 ms,
        // profiles/r04_ab_dual_streams_32bps.txt)
        for (int b = 0; b < 2; b++) HIPCHK(hipStreamCreateWithPriority(&p->astream[b], hipStreamNonBlocking, hi));
        if (p->wave_ok) {  // the k_analyze_w instance counters (fra_plan::kCnt ring)
          HIPCHK(hipMalloc(&p->d_cnt17, sizeof(uint32_t) * fra_plan::kCnt));
          HIPCHK(hipMemset(p->d_cnt17, 0, sizeof(uint32_t) * fra_plan::kCnt));
          HIPCHK(hipHostMalloc((void**)&p->h_cnt17, sizeof(uint32_t) * fra_plan::kCnt, hipHostMallocPortable));
          for (auto& e : p->ev_cnt) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
      }
      for (int b = 0; b < fra_plan::kSlotSets; b++) {
        HIPCHK(hipEventCreateWithFlags(&p->ev_scan[b], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&p->ev_pack[b], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&p->ev_norm[b], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&p->ev_ana[b], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&p->ev_part[b], hipEventDisableTiming));
      }
    }
  }
  return FRA_OK;
}

// point the plan (and its kernel arguments) at buffer set b
static void use_buffers(fra_plan* p, int b, int nb) {
  if (!p->pipe) return;
  p->d_sf = p->sf2[b]; p->d_tmp = p->tmp2[b]; p->d_fmeta = p->fmeta2[b];
  p->d_fbytes = p->fbytes2[b]; p->d_foff = p->foff2[b];
  p->d_norm = p->norm2[nb]; p->d_lut = p->lut2[nb];
  p->args.sf = p->d_sf; p->args.tmp = p->d_tmp; p->args.fmeta = p->d_fmeta; p->args.err = p->d_err;
  p->args.frame_bytes = p->d_fbytes; p->args.frame_off = p->d_foff;
  p->args.norm = p->d_norm; p->args.lut = p->d_lut;
  p->cur = b;
  p->curn = nb;
}
// make the plan's stream wait for every k_assemble still running on the pack stream, then use set 0
static int drain_pipeline(fra_plan* p) {
  if (!p->pipe) return FRA_OK;
  for (int b = 0; b < fra_plan::kSlotSets; b++) {
    if (p->pack_pending[b]) {
      HIPCHK(hipStreamWaitEvent(p->ctx->stream, p->ev_pack[b], 0));
      p->pack_pending[b] = false;
    }
    // (an analysis on astream[b] is followed by its chain + assembly on the pack stream: covered above;
    // the wait below also orders a pipelined execute's analysis before the serial work that follows)
    if (p->ana_pending[b] && p->astream[0]) HIPCHK(hipStreamWaitEvent(p->ctx->stream, p->ev_ana[b], 0));
    p->ana_pending[b] = false;  // (covered by the resync below)
  }
  for (int n = 0; n < fra_plan::kNormSets; n++) {  // (norm stream: its partial-subframe lists)
    if (p->nfree_pending[n]) HIPCHK(hipStreamWaitEvent(p->ctx->stream, p->ev_nfree[n], 0));
    p->nfree_pending[n] = false;
  }
  // serial executes and host raster copies now go onto the plan's stream; when pipelining resumes, the
  // first background norm stage waits for ALL of it (an event recorded on the plan's stream at that
  // point): a pipelined analysis still reading a norm set or a raster copy queued before this drain
  // cannot be overtaken
  p->resync = true;
  p->raster_dirty = false;
  use_buffers(p, 0, 0);
  return FRA_OK;
}
// device-detected inconsistencies (JobArgs::err): bit 0 a frame-scan ticket past its grid, bit 1 a frame the
// assembly did not write because its sizes left the output or its slots -- the stream is not handed back.  The
// word is sticky: once set, every later sync / result / host encode of the plan reports it (call after the work
// that may set it has completed)
static int check_dev_err(fra_plan* p) {
  if (p->d_err) {
    uint32_t e = 0;
    HIPCHK(hipMemcpy(&e, p->d_err, sizeof(e), hipMemcpyDeviceToHost));
    if (e) return set_err(FRA_E_STATE, "device error word 0x%x (%s%s)", e, (e & 1u) ? "frame-scan ticket desync " : "",
                          (e & 2u) ? "frame outside its output/slot bounds" : "");
  }
  return FRA_OK;
}
static int plan_sync_all(fra_plan* p) {
  for (auto& st : p->astream)
    if (st) HIPCHK(hipStreamSynchronize(st));
  if (p->nstream) HIPCHK(hipStreamSynchronize(p->nstream));
  if (p->pack) HIPCHK(hipStreamSynchronize(p->pack));
  HIPCHK(hipStreamSynchronize(p->ctx->stream));
  return check_dev_err(p);
}

int fra_plan_set_raster(fra_plan* p, const void* raster, int32_t on_device) {
  if (!p) return set_err(FRA_E_INVALID, "null plan");
  (void)hipSetDevice(p->ctx->device);
  if (on_device) {
    p->d_raster = raster;
  } else {
    if (!p->d_raster_owned && p->raster_bytes) HIPCHK(hipMalloc(&p->d_raster_owned, p->raster_bytes));
    // the copy must not overtake a pipelined analysis (its own stream) still reading the old rows
    for (int b = 0; b < fra_plan::kSlotSets; b++)
      if (p->ana_pending[b] && p->astream[0]) HIPCHK(hipStreamWaitEvent(p->ctx->stream, p->ev_ana[b], 0));
    if (p->raster_bytes) {
      HIPCHK(hipMemcpyAsync(p->d_raster_owned, raster, p->raster_bytes, hipMemcpyHostToDevice, p->ctx->stream));
      if (p->pipe) {  // the next pipelined norm stage (norm stream) reads the new raster after this copy
        HIPCHK(hipEventRecord(p->ev_raster, p->ctx->stream));
        p->raster_dirty = true;
      }
    }
    p->d_raster = p->d_raster_owned;
  }
  p->args.raster = p->d_raster;
  p->job.raster = raster;
  p->job.raster_on_device = on_device;
  return FRA_OK;
}

static int plan_create(fra_ctx* ctx, const fra_job* job, const int32_t* franges, fra_plan** out);
int fra_plan_create(fra_ctx* ctx, const fra_job* job, fra_plan** out) {
  return plan_create(ctx, job, nullptr, out);
}
int fra_plan_create_ranged(fra_ctx* ctx, const fra_job* job, const int32_t* frame_ranges, fra_plan** out) {
  if (!frame_ranges) return set_err(FRA_E_INVALID, "null frame_ranges");
  return plan_create(ctx, job, frame_ranges, out);
}
static int plan_create(fra_ctx* ctx, const fra_job* job, const int32_t* franges, fra_plan** out) {
  if (!ctx || !job || !out) return set_err(FRA_E_INVALID, "null argument");
  if (job->channels < 1 || job->channels > 8) return set_err(FRA_E_INVALID, "channels must be 1..8 (got %d)", job->channels);
  if (job->blocksize < 16 || job->blocksize > kMaxBlock)
    return set_err(FRA_E_INVALID, "blocksize must be 16..%d (got %d)", kMaxBlock, job->blocksize);
  if (job->level < 0 || job->level > 8) return set_err(FRA_E_INVALID, "level must be 0..8 (got %d)", job->level);
  if (job->dtype < FRA_U8 || job->dtype > FRA_F64) return set_err(FRA_E_INVALID, "bad dtype %d", job->dtype);
  if (job->norm != 0 && job->norm != 16 && job->norm != 24) return set_err(FRA_E_INVALID, "norm must be 0, 16 or 24");
  if (job->norm == 0 && job->dtype != FRA_I16 && job->dtype != FRA_I32)
    return set_err(FRA_E_INVALID, "norm == 0 (pre-normalised audio) needs int16 or int32 samples");
  if (job->nwindows < 0 || (job->nwindows > 0 && !job->windows)) return set_err(FRA_E_INVALID, "bad windows");
  if (job->first_frame < 0) return set_err(FRA_E_INVALID, "first_frame must be >= 0");
  // (the analysis descriptors hold the row stride in 32 bits: WaveDev)
  if (job->band_stride < 0 || job->row_stride < 0 || job->col_stride < 1 || job->row_stride > (int64_t)UINT32_MAX)
    return set_err(FRA_E_INVALID, "strides must be >= 0 (col_stride >= 1) with row_stride < 2^32 elements");
  for (int w = 0; w < job->nwindows; w++) {
    const fra_window& wd = job->windows[w];
    if (wd.height < 0 || wd.width < 0 || wd.row_off < 0 || wd.col_off < 0 || (wd.height > 0) != (wd.width > 0))
      return set_err(FRA_E_INVALID, "window %d invalid (%d,%d,%d,%d)", w, wd.row_off, wd.col_off, wd.height, wd.width);
  }
  fra_plan* p = new (std::nothrow) fra_plan();
  if (!p) return set_err(FRA_E_NOMEM, "out of host memory");
  p->ctx = ctx;
  p->job = *job;
  p->windows.assign(job->windows, job->windows + job->nwindows);
  p->job.windows = p->windows.data();
  if (franges) {
    // a range must start inside its window's stream (a count past the end is clipped to it): a first frame past
    // the end or a negative count other than -1 (to the end) is a malformed work item of a multi-GPU split
    // 
    for (int w = 0; w < job->nwindows; w++) {
      const fra_window& wd = job->windows[w];
      const int64_t nfr_all = ((int64_t)wd.width * wd.height + job->blocksize - 1) / job->blocksize;
      const int32_t f0 = franges[2 * w], n = franges[2 * w + 1];
      if (f0 < 0 || f0 > nfr_all || n < -1) {
        delete p;
        return set_err(FRA_E_INVALID, "window %d: frame range (%d, %d) outside its %lld frames", w, f0, n,
                       (long long)nfr_all);
      }
    }
    p->franges.assign(franges, franges + 2 * (size_t)job->nwindows);
  }
  int rc = plan_build(p);
  if (rc == FRA_OK && job->raster) rc = fra_plan_set_raster(p, job->raster, job->raster_on_device);
  if (rc != FRA_OK) {
    std::string keep = g_err;
    fra_plan_destroy(p);
    g_err = keep;
    return rc;
  }
  *out = p;
  return FRA_OK;
}

static void collect_times(fra_plan* p) {
  if (!p->pending_times) return;
  (void)hipEventSynchronize(p->ev[4]);
  for (int k = 0; k < 4; k++) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, p->ev[k], p->ev[k + 1]) == hipSuccess) p->ms[k] += ms;
  }
  p->nexec++;
  p->pending_times = false;
}

// k_analyze_w (one subframe per wave, fra_analyze_w.hip) takes the full frames of 16-bit plans normalised
// through the per-tile table with 8-byte sample vectors at levels 3-6 (the partial frames' subframes go to
// k_analyze as a list); FRA_ANALYZE_WG=1 keeps every frame on the workgroup kernel (tests compare both)
static bool wave_path(const fra_plan* p) {
  const bool wg = getenv("FRA_ANALYZE_WG") && atoi(getenv("FRA_ANALYZE_WG")) == 1;
  if (wg || !p->wave_ok || !p->args.vec8 || !p->args.off32 || p->job.blocksize != kMaxBlock) return false;
  // (32-bps plans stay on k_analyze: a one-subframe-per-wave 32-bps kernel, r05's k_analyze_w32, was measured
  // slower -- C5 quarter 28.5 against 22.8 ms of analysis, profiles/r05_ab_w32_c5q.txt -- and removed in r06)
  if (p->b32) return false;
  return p->args.lut && p->job.level >= 3 && p->job.level <= 6;  // k_analyze_w
}
// one frame group on stream st: minmax/LUT of its windows, analysis, frame sizes, the group's own scan,
// global offsets after the previous group's (event ordered), assembly.  ev_* null = serial.
static int run_group(fra_plan* p, const fra_plan::Group& gr, int gi, int ng, hipStream_t st, hipEvent_t ev_prev,
                     hipEvent_t ev_pub, hipEvent_t t_norm, hipEvent_t t_ana, hipEvent_t t_scan, int slot = -1,
                     unsigned long long* host_mirror = nullptr, hipStream_t pack_st = nullptr,
                     hipEvent_t ev_scan = nullptr, hipStream_t norm_st = nullptr, hipEvent_t ev_norm = nullptr,
                     hipEvent_t ev_ana = nullptr) {
  const JobArgs& a = p->args;
  const hipStream_t nst_s = norm_st ? norm_st : st;  // the normalisation stage's stream
  const int nst = gr.w1 - gr.w0, nf = gr.f1 - gr.f0;
  // the minmax family indexes streams by blockIdx.y: launched per chunk of <= kMaxGridY windows, with the
  // stream/norm/LUT pointers offset to the chunk (grid Y is limited to 65535 on the device)
  constexpr int kMaxGridY = 65535;
  for (int c0 = 0; p->job.norm != 0 && p->max_segs > 0 && c0 < nst; c0 += kMaxGridY) {
    const int nc = std::min(kMaxGridY, nst - c0);
    JobArgs ma = a;
    ma.streams += gr.w0 + c0;
    ma.norm += gr.w0 + c0;
    if (ma.lut) ma.lut += (int64_t)(gr.w0 + c0) * a.lut_stride;
    const int vec = (p->mm_vec && (uintptr_t)p->d_raster % p->mm_vec == 0) ? p->mm_vec : 0;  // pointer alignment
    // the norm stage of a pipelined execute: the full grid, one workgroup per row block, as in serial plans --
    // measured against one workgroup per CU striding over the blocks (FRA_MM_PER_CU=n: n per CU): C4 step
    // 1.666 -> 1.626 ms, 8-way share 0.292 -> 0.274 ms, 4-way 0.505 -> 0.488 ms, C5 neutral, C3 1.089 -> 1.101
    // (profiles/r04_ab_assemble_fpw_minmax_grid.txt, r04_ab_minmax_grid_shards.txt)
    static const int mm_per_cu = getenv("FRA_MM_PER_CU") ? atoi(getenv("FRA_MM_PER_CU")) : 0;
    HIPCHK(launch_minmax(p->src, ma, nc, p->max_segs, vec, p->mm_rows, p->mm_max_rows, nst_s,
                         norm_st ? mm_per_cu * p->ncu : 0));
    HIPCHK(launch_norm_finalize(ma, nc, nst_s));
    HIPCHK(launch_norm_lut(p->src, ma, nc, nst_s));
  }
  JobArgs ga = a;
  ga.frame_base = gr.f0;
  ga.frame_count = nf;
  // wave path: k_analyze_w for the full frames, k_analyze for this group's partial subframes -- pipelined, on
  // the norm stream right after the norm stage (a whole execute before the frame scan that waits for them),
  // else beside k_analyze_w on the side stream
  const bool wave = wave_path(p);
  // (tests: FRA_REQUIRE_WAVE=1 makes a plan that would not take the wave path fail instead)
  const bool require_wave = getenv("FRA_REQUIRE_WAVE") && atoi(getenv("FRA_REQUIRE_WAVE")) == 1;
  if (require_wave && !wave && nf > 0) return set_err(FRA_E_STATE, "FRA_REQUIRE_WAVE: the plan does not take k_analyze_w");
  const auto plo = std::lower_bound(p->h_part.begin(), p->h_part.end(), gr.f0 * 8);
  const auto phi = std::lower_bound(p->h_part.begin(), p->h_part.end(), gr.f1 * 8);
  const int npart = wave ? (int)(phi - plo) : 0;
  const int32_t* part = wave ? p->d_part + (plo - p->h_part.begin()) : nullptr;
  const hipEvent_t ev_part = (norm_st && npart > 0) ? p->ev_part[p->cur] : nullptr;
  if (norm_st) {
    HIPCHK(hipEventRecord(ev_norm, norm_st));
    HIPCHK(hipStreamWaitEvent(st, ev_norm, 0));
    if (ev_part) {
      // (these slots: execute k-2's assembly read them -- the norm stream waited for it, or, FRA_BG_SERIAL=0,
      // this stream does just before the launch)
      if (!bg_serial(p->b32) && p->pack_pending[p->cur]) HIPCHK(hipStreamWaitEvent(norm_st, p->ev_pack[p->cur], 0));
      HIPCHK(launch_analyze_part(p->src, p->b32, ga, part, npart, 8 * p->ncu, norm_st));
      HIPCHK(hipEventRecord(ev_part, norm_st));
    }
  }
  if (t_norm) HIPCHK(hipEventRecord(t_norm, st));
  int cj = -1;  // the counter slot of this launch (-1: not counted)
  if (wave) {
    // the snapshots that have arrived (newest wins): 17 bits when more than 1/32 of its waves needed bit 16 -- a wave
    // that does on the 16-bit instance re-derives its residuals from the samples (the sample path)
    for (int j = 0; j < fra_plan::kCnt; j++) {
      if (!p->cnt_pending[j] || hipEventQuery(p->ev_cnt[j]) != hipSuccess) continue;
      p->cnt_pending[j] = false;
      const uint32_t n17 = p->h_cnt17[j] - p->cnt_base[j];
      p->cnt_base[j] = p->h_cnt17[j];
      if (p->cnt_seq[j] >= p->cnt_newest) {
        p->cnt_newest = p->cnt_seq[j];
        p->k17 = n17 > p->cnt_sub[j] / 32 ? 1 : 0;
      }
    }
    const char* ek = getenv("FRA_KEEP17");  // tests / A/B: 0 or 1 forces the instance
    ga.k17 = (ek && ek[0] == '0') ? 0 : (ek && ek[0] == '1') ? 1 : p->k17;
    const int j = (int)(p->cnt_next % fra_plan::kCnt);
    if (p->d_cnt17 && !p->cnt_pending[j] && nf > 0 && ng == 1) {
      cj = j;
      ga.cnt17 = p->d_cnt17 + j;
    }
  }
  p->cnt_cur = cj;  // (fra_plan_execute copies the count out after everything the execute timed or waits on)
  {
    HIPCHK(launch_analyze(p->src, p->b32, p->cmax == 4 && p->job.channels == 2, ga, st, wave,
                          ev_part ? nullptr : part, ev_part ? 0 : npart, 8 * p->ncu, p->pside, p->ev_pfork,
                          p->ev_pjoin));
  }
  if (t_ana) HIPCHK(hipEventRecord(t_ana, st));
  if (cj >= 0) p->cnt_sub[cj] = (uint32_t)nf * (uint32_t)p->cmax;
  if (ev_ana) HIPCHK(hipEventRecord(ev_ana, st));  // the norm set is free for execute k+2's norm stage
  // pipelined execute: the frame-size chain (k_frame_scan) only feeds this
  // execute's assembly, so it goes onto the pack stream with it and the plan's stream proceeds straight to
  // the next execute's analysis
  if (pack_st && !ev_prev && !ev_pub && !host_mirror) {
    HIPCHK(hipEventRecord(ev_scan, st));
    HIPCHK(hipStreamWaitEvent(pack_st, ev_scan, 0));
    st = pack_st;
    pack_st = nullptr;
  }
  if (ev_part) HIPCHK(hipStreamWaitEvent(st, ev_part, 0));  // the partial subframes (norm stream) are done
  // frame sizes and offsets: one k_frame_scan; with the group's base already ordered (first / only group,
  // host bands on one stream) it writes the final offsets itself, else k_group_offsets adds the base once
  // the previous group has published it
  if (nf > 0) {
    const int sl = slot < 0 ? gi : slot;
    HIPCHK(launch_frame_scan(ga, p->d_gbase, gi, gi == ng - 1, ev_prev ? 0 : 1, host_mirror,
                             p->d_look + (size_t)sl * 2 * p->look_stride, p->look_stride, p->d_ticket + sl, st));
  }
  if (ev_prev) HIPCHK(hipStreamWaitEvent(st, ev_prev, 0));
  if (nf == 0 || ev_prev)
    HIPCHK(launch_group_offsets(p->d_foff, p->d_fbytes, p->d_gbase, gi, gr.f0, nf, gi == ng - 1,
                                a.nframes_total, st, host_mirror));
  if (ev_pub) HIPCHK(hipEventRecord(ev_pub, st));
  if (t_scan) HIPCHK(hipEventRecord(t_scan, st));
  if (pack_st) {  // assembly on the pack stream once this group's offsets exist
    HIPCHK(hipEventRecord(ev_scan, st));
    HIPCHK(hipStreamWaitEvent(pack_st, ev_scan, 0));
    HIPCHK(launch_assemble(ga, pack_st));
  } else {
    HIPCHK(launch_assemble(ga, st));
  }
  return FRA_OK;
}

// after an execute: copy its k_analyze_w count (fra_plan::d_cnt17 slot) to page-locked memory on the analysis
// stream s, behind everything the execute's frame scan, assembly and timing events wait for
static int count_out(fra_plan* p, hipStream_t s) {
  const int cj = p->cnt_cur;
  if (cj < 0) return FRA_OK;
  p->cnt_cur = -1;
  HIPCHK(hipMemcpyAsync(p->h_cnt17 + cj, p->d_cnt17 + cj, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipEventRecord(p->ev_cnt[cj], s));
  p->cnt_pending[cj] = true;
  p->cnt_seq[cj] = p->cnt_next++;
  return FRA_OK;
}

int fra_plan_execute(fra_plan* p) {
  if (!p) return set_err(FRA_E_INVALID, "null plan");
  if (!p->d_raster && !p->streams.empty()) return set_err(FRA_E_STATE, "plan has no raster");
  (void)hipSetDevice(p->ctx->device);
  hipStream_t s = p->ctx->stream;
  if (p->timing) collect_times(p);
  p->args.vec8 = (p->ld_vec8 && (uintptr_t)p->d_raster % 8 == 0) ? 1 : 0;
  int rc = FRA_OK;
  if (p->pipe && !p->timing) {
    // cross-execute pipelining: this execute's analysis overlaps the previous execute's k_assemble
    const int b = (p->cur + 1) % p->nslot;
    const int ai = (int)(p->exec_n++ & 1u);
    const hipStream_t as = p->astream[ai] ? p->astream[ai] : s;  // this execute's analysis stream
    if (p->pack_pending[b]) HIPCHK(hipStreamWaitEvent(as, p->ev_pack[b], 0));  // execute k-nslot is done with set b
    // one background kernel at a time beside k_analyze: this norm stage after k_assemble of execute k-2
    // (which runs under the analysis of execute k-1) -- 32-bps plans; 16-bit plans: only the partial-subframe list launch
    // after the norm stage waits for that assembly (it rewrites the slots; the norm stage writes only this set's
    // NormDev / table, which execute k-2's analysis and partial list -- both earlier on this stream or waited
    // for below -- read)
    if (p->pack_pending[b] && bg_serial(p->b32)) HIPCHK(hipStreamWaitEvent(p->nstream, p->ev_pack[b], 0));
    // norm set: the next of kNormSets (FRA_NORM_SETS=2: the slot set's, as before r05 -- A/B)
    static const int nsets = getenv("FRA_NORM_SETS") && atoi(getenv("FRA_NORM_SETS")) == 2 ? 2 : fra_plan::kNormSets;
    const int nb = nsets == 2 ? b : (p->curn + 1) % fra_plan::kNormSets;
    use_buffers(p, b, nb);
    // norm stage of this execute on the norm stream: after the last analysis that read norm set nb (execute
    // k-3, or k-2 with two sets), and after a host raster copy enqueued on the plan's stream since the last
    // execute.  (That analysis's partial-subframe list ran earlier on the norm stream itself.)
    if (p->nfree_pending[nb]) HIPCHK(hipStreamWaitEvent(p->nstream, p->ev_nfree[nb], 0));
    if (p->resync) {  // first pipelined execute after serial ones: after everything on the plan's stream
      HIPCHK(hipEventRecord(p->ev_raster, s));
      for (auto& st : p->astream)
        if (st) HIPCHK(hipStreamWaitEvent(st, p->ev_raster, 0));
      p->raster_dirty = true;
      p->resync = false;
    }
    if (p->raster_dirty) {
      HIPCHK(hipStreamWaitEvent(p->nstream, p->ev_raster, 0));
      p->raster_dirty = false;
    }
    rc = run_group(p, p->groups[0], 0, 1, as, nullptr, nullptr, nullptr, nullptr, nullptr, -1, nullptr, p->pack,
                   p->ev_scan[b], p->nstream, p->ev_norm[b], p->ev_ana[b]);
    if (rc) return rc;
    if ((rc = count_out(p, as))) return rc;
    p->ana_pending[b] = true;
    HIPCHK(hipEventRecord(p->ev_nfree[nb], as));  // (the analysis was the last work on `as`)
    p->nfree_pending[nb] = true;
    HIPCHK(hipEventRecord(p->ev_pack[b], p->pack));
    p->pack_pending[b] = true;
    p->executed = true;
    return FRA_OK;
  }
  if ((rc = drain_pipeline(p))) return rc;
  if (p->timing || p->groups.size() == 1) {
    // serial: the whole plan as one group; timing events bracket each kernel phase
    if (p->timing) HIPCHK(hipEventRecord(p->ev[0], s));
    hipEvent_t* e = p->ev;
    rc = run_group(p, p->timing ? p->all : p->groups[0], 0, 1, s, nullptr, nullptr, p->timing ? e[1] : nullptr,
                   p->timing ? e[2] : nullptr, p->timing ? e[3] : nullptr);
    if (rc) return rc;
    if (p->timing) {
      HIPCHK(hipEventRecord(p->ev[4], s));
      p->pending_times = true;
    }
    if ((rc = count_out(p, s))) return rc;
  } else {
    const int ng = (int)p->groups.size();
    HIPCHK(hipEventRecord(p->gev[0], s));
    for (int g = 1; g < ng; g++) HIPCHK(hipStreamWaitEvent(p->aux[g - 1], p->gev[0], 0));
    for (int g = 0; g < ng; g++) {
      hipStream_t st = g == 0 ? s : p->aux[g - 1];
      rc = run_group(p, p->groups[g], g, ng, st, g ? p->gev[1 + 2 * (g - 1)] : nullptr, p->gev[1 + 2 * g], nullptr,
                     nullptr, nullptr);
      if (rc) return rc;
      if (g) HIPCHK(hipEventRecord(p->gev[2 + 2 * g], st));
    }
    for (int g = 1; g < ng; g++) HIPCHK(hipStreamWaitEvent(s, p->gev[2 + 2 * g], 0));
  }
  p->executed = true;
  return FRA_OK;
}

int fra_plan_sync(fra_plan* p) {
  if (!p) return set_err(FRA_E_INVALID, "null plan");
  (void)hipSetDevice(p->ctx->device);
  if (int rc = plan_sync_all(p)) return rc;
  if (p->timing) collect_times(p);
  return FRA_OK;
}

int fra_plan_result(fra_plan* p, fra_stream_info* infos, uint64_t* total) {
  if (!p) return set_err(FRA_E_INVALID, "null plan");
  if (!p->executed) return set_err(FRA_E_STATE, "plan not executed");
  (void)hipSetDevice(p->ctx->device);
  if (int rc = plan_sync_all(p)) return rc;
  const int nfr = p->args.nframes_total;
  std::vector<unsigned long long> off(nfr + 1);
  HIPCHK(hipMemcpy(off.data(), p->d_foff, sizeof(unsigned long long) * (nfr + 1), hipMemcpyDeviceToHost));
  // exclusive scan of [bytes..., 0]: off[nfr] = total
  if (total) *total = off[nfr];
  if (infos) {
    std::vector<NormDev> nd(p->streams.size());
    if (!nd.empty())
      HIPCHK(hipMemcpy(nd.data(), p->d_norm, sizeof(NormDev) * nd.size(), hipMemcpyDeviceToHost));
    for (size_t s = 0; s < p->streams.size(); s++) {
      const StreamDev& st = p->streams[s];
      fra_stream_info& in = infos[s];
      in.offset = off[st.first_frame];
      in.frame_bytes = off[st.first_frame + st.nframes] - off[st.first_frame];
      in.data_min = p->job.norm ? nd[s].mn : 0.0;
      in.data_max = p->job.norm ? nd[s].mx : 0.0;
      in.sample_rate = st.sample_rate;
      in.bps = st.bps;
      in.channels = st.channels;
      in.nframes = st.nframes;
    }
  }
  return FRA_OK;
}

int fra_plan_download(fra_plan* p, uint8_t* host_out, uint64_t capacity) {
  uint64_t total = 0;
  int rc = fra_plan_result(p, nullptr, &total);
  if (rc) return rc;
  if (capacity < total) return set_err(FRA_E_INVALID, "capacity %llu < %llu", (unsigned long long)capacity,
                                       (unsigned long long)total);
  if (total) HIPCHK(hipMemcpy(host_out, p->d_out, total, hipMemcpyDeviceToHost));
  return FRA_OK;
}

int fra_plan_frame_offsets(fra_plan* p, uint64_t* offsets, uint64_t n) {
  if (!p || !offsets) return set_err(FRA_E_INVALID, "null argument");
  if (!p->executed) return set_err(FRA_E_STATE, "plan not executed");
  const uint64_t nfr = (uint64_t)p->args.nframes_total;
  if (n != nfr + 1) return set_err(FRA_E_INVALID, "frame offsets: n = %llu, plan has %llu frames + 1",
                                   (unsigned long long)n, (unsigned long long)nfr);
  (void)hipSetDevice(p->ctx->device);
  if (int rc = plan_sync_all(p)) return rc;
  static_assert(sizeof(unsigned long long) == sizeof(uint64_t), "u64");
  HIPCHK(hipMemcpy(offsets, p->d_foff, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
  return FRA_OK;
}

int fra_plan_device_output(fra_plan* p, const uint8_t** dev_ptr, uint64_t* capacity) {
  if (!p) return set_err(FRA_E_INVALID, "null plan");
  *dev_ptr = p->d_out;
  *capacity = p->out_cap;
  return FRA_OK;
}

int fra_plan_enable_timing(fra_plan* p, int32_t on) {
  if (!p) return set_err(FRA_E_INVALID, "null plan");
  p->timing = on != 0;
  for (float& m : p->ms) m = 0;
  p->nexec = 0;
  p->pending_times = false;
  return FRA_OK;
}

int fra_plan_timing(fra_plan* p, float* ms4, int32_t* n) {
  if (!p) return set_err(FRA_E_INVALID, "null plan");
  collect_times(p);
  for (int k = 0; k < 4; k++) ms4[k] = p->ms[k];
  *n = p->nexec;
  return FRA_OK;
}

int fra_plan_set_first_frame(fra_plan* p, int32_t first_frame) {
  if (!p || first_frame < 0) return set_err(FRA_E_INVALID, "bad argument");
  (void)hipSetDevice(p->ctx->device);
  // pipelined executes still in flight read frame_number0 on the analysis / pack streams (k_frame_scan):
  // let them finish before the table changes under them
  if (int rc = plan_sync_all(p)) return rc;
  p->job.first_frame = first_frame;
  for (auto& st : p->streams) st.frame_number0 = (uint32_t)first_frame;
  if (!p->streams.empty())  // complete before this call returns, so every later execute reads it
    HIPCHK(hipMemcpyAsync(p->d_streams, p->streams.data(), sizeof(StreamDev) * p->streams.size(),
                          hipMemcpyHostToDevice, p->ctx->stream));
  HIPCHK(hipStreamSynchronize(p->ctx->stream));  // the host array may change again before it is read
  return FRA_OK;
}

int fra_plan_flags(fra_plan* p, int32_t* flags) {
  if (!p || !flags) return set_err(FRA_E_INVALID, "null argument");
  // (vector loads as an execute will decide them: the device raster's alignment, or hipMalloc's for host rasters)
  p->args.vec8 = (p->ld_vec8 && (!p->d_raster || (uintptr_t)p->d_raster % 8 == 0)) ? 1 : 0;
  const char* ek = getenv("FRA_KEEP17");
  const int k17 = (ek && ek[0] == '0') ? 0 : (ek && ek[0] == '1') ? 1 : p->k17;
  *flags = (p->pipe ? FRA_PLAN_PIPELINED : 0) | (wave_path(p) ? FRA_PLAN_WAVE : 0) | (k17 ? FRA_PLAN_KEEP17 : 0);
  return FRA_OK;
}

int fra_plan_capacity(fra_plan* p, uint64_t* capacity, int32_t* host_bands) {
  if (!p) return set_err(FRA_E_INVALID, "null plan");
  if (capacity) *capacity = p->out_cap;
  if (host_bands) *host_bands = (int32_t)p->hbands.size();
  return FRA_OK;
}

// H2D of raster rows [r0, r1) of every band (channel) of the job: one contiguous run per channel for
// band-planar rasters (band_stride >= row_stride), one run for pixel-interleaved ones; clamped to the
// plan's extent (the last row of the last channel may end before row_stride does)
static int copy_rows_h2d(fra_plan* p, const uint8_t* host, int64_t r0, int64_t r1, hipStream_t st) {
  const fra_job& j = p->job;
  const int es = elem_size(j.dtype);
  const int64_t extent = (int64_t)(p->raster_bytes / es);
  const bool planar = j.channels > 1 && j.band_stride >= j.row_stride;
  const int nrun = planar ? j.channels : 1;
  for (int c = 0; c < nrun; c++) {
    const int64_t a = (int64_t)c * (planar ? j.band_stride : 0) + r0 * j.row_stride;
    const int64_t b = std::min(extent, (int64_t)c * (planar ? j.band_stride : 0) + r1 * j.row_stride);
    if (b > a)
      HIPCHK(hipMemcpyAsync((uint8_t*)p->d_raster_owned + a * es, host + a * es, (size_t)(b - a) * es,
                            hipMemcpyHostToDevice, st));
  }
  return FRA_OK;
}

// the bounded-memory input of fra_plan_encode_ring: image row r of channel c at ring row r % rows
struct RingIn {
  const uint8_t* ring;
  int64_t rows;
  volatile int64_t* rows_done;
};
// H2D of raster rows [r0, r1) from the ring: per channel (run) at most two pieces, split where the ring wraps
static int copy_rows_ring_h2d(fra_plan* p, const RingIn& rg, int64_t r0, int64_t r1, hipStream_t st) {
  const fra_job& j = p->job;
  const int es = elem_size(j.dtype);
  const int64_t extent = (int64_t)(p->raster_bytes / es);
  const bool planar = j.channels > 1 && j.band_stride >= j.row_stride;
  const int nrun = planar ? j.channels : 1;
  for (int c = 0; c < nrun; c++) {
    const int64_t dbase = (int64_t)c * (planar ? j.band_stride : 0);
    const int64_t hbase = (int64_t)c * (planar ? rg.rows * j.row_stride : 0);
    for (int64_t r = r0; r < r1;) {
      const int64_t rr = r % rg.rows, n = std::min(r1 - r, rg.rows - rr);
      const int64_t a = dbase + r * j.row_stride;
      const int64_t b = std::min(extent, dbase + (r + n) * j.row_stride);
      if (b > a)
        HIPCHK(hipMemcpyAsync((uint8_t*)p->d_raster_owned + a * es, rg.ring + (hbase + rr * j.row_stride) * es,
                              (size_t)(b - a) * es, hipMemcpyHostToDevice, st));
      r += n;
    }
  }
  return FRA_OK;
}

// page-locked (hipHostMalloc'd or registered) host memory: an async copy to it returns at once
static bool host_pinned(const void* ptr) {
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, ptr) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeHost;
}
// encode_host's D2H copies into a pageable output, on threads of their own (`out` null: off, the caller copies
// itself).  The runtime's own copy into pageable memory stages through one pinned buffer and copies out on the
// calling thread, page faults of a lazily committed buffer included: about 17 GB/s, so C5's 22.4 GB of frames
// outlasted the 34 GB raster's H2D by 0.6 s (profiles/r05_ring_timeline.txt).  Here each of n threads owns a
// 64 MiB piece of page-locked staging: DMA the piece into it at the link rate, then copy it out on that thread,
// so the copy-outs and their page faults run n-wide beside the DMA.  push() takes a byte range whose frames are
// complete on the device.
struct D2HWorker {
  static constexpr uint64_t kPiece = 64ull << 20;
  D2HWorker(int device, uint8_t* out, const uint8_t* dev, uint8_t* stage, const std::vector<hipStream_t>& st)
      : out_(out), dev_(dev) {
    if (!out_) return;
    for (size_t i = 0; i < st.size(); i++)
      th_.emplace_back([this, device, stage, i, s = st[i]]() { run(device, stage + (uint64_t)i * kPiece, s); });
  }
  ~D2HWorker() { finish(); }
  bool on() const { return out_ != nullptr; }
  void push(uint64_t a, uint64_t b) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (uint64_t x = a; x < b; x += kPiece) q_.emplace_back(x, std::min(b, x + kPiece));
    }
    cv_.notify_all();
  }
  // wait for every pushed copy; false if one failed (error())
  bool finish() {
    if (!th_.empty()) {
      { std::lock_guard<std::mutex> lk(mu_); end_ = true; }
      cv_.notify_all();
      for (auto& t : th_) t.join();
      th_.clear();
    }
    return err_.empty();
  }
  const std::string& error() const { return err_; }

 private:
  void run(int device, uint8_t* stage, hipStream_t st) {
    hipError_t e = hipSetDevice(device);
    for (;;) {
      std::pair<uint64_t, uint64_t> r;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return !q_.empty() || end_; });
        if (q_.empty()) break;
        r = q_.front();
        q_.pop_front();
      }
      if (e != hipSuccess) continue;  // drain the queue after a failure
      const size_t n = (size_t)(r.second - r.first);
      e = hipMemcpyAsync(stage, dev_ + r.first, n, hipMemcpyDeviceToHost, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      if (e == hipSuccess) memcpy(out_ + r.first, stage, n);
    }
    if (e != hipSuccess) {
      std::lock_guard<std::mutex> lk(mu_);
      if (err_.empty()) err_ = hipGetErrorString(e);
    }
  }
  uint8_t* out_;
  const uint8_t* dev_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::pair<uint64_t, uint64_t>> q_;
  bool end_ = false;
  std::string err_;  // read after the joins
};
static int encode_host(fra_plan* p, const void* host_raster, uint8_t* host_out, uint64_t capacity,
                       uint64_t* total_bytes, const volatile int64_t* rows_ready, const RingIn* ring = nullptr);
int fra_plan_encode_host(fra_plan* p, const void* host_raster, uint8_t* host_out, uint64_t capacity,
                         uint64_t* total_bytes) {
  return encode_host(p, host_raster, host_out, capacity, total_bytes, nullptr);
}
int fra_plan_encode_host_progress(fra_plan* p, const void* host_raster, uint8_t* host_out, uint64_t capacity,
                                  uint64_t* total_bytes, const volatile int64_t* rows_ready) {
  if (!rows_ready) return set_err(FRA_E_INVALID, "null rows_ready");
  return encode_host(p, host_raster, host_out, capacity, total_bytes, rows_ready);
}
int fra_plan_host_band_rows(fra_plan* p, int64_t* max_rows) {
  if (!p || !max_rows) return set_err(FRA_E_INVALID, "null argument");
  int64_t m = 0;
  for (const auto& hb : p->hbands) m = std::max(m, hb.r1 - hb.r0);
  *max_rows = m;
  return FRA_OK;
}
int fra_plan_encode_ring(fra_plan* p, const void* ring, int64_t ring_rows, uint8_t* host_out, uint64_t capacity,
                         uint64_t* total_bytes, const volatile int64_t* rows_ready, volatile int64_t* rows_done) {
  if (!p || !ring || !rows_ready || !rows_done) return set_err(FRA_E_INVALID, "null argument");
  int64_t mx = 0;
  fra_plan_host_band_rows(p, &mx);
  if (ring_rows < mx || ring_rows < 1)
    return set_err(FRA_E_INVALID, "ring of %lld rows < the tallest host band (%lld rows)", (long long)ring_rows,
                   (long long)mx);
  const RingIn rg{(const uint8_t*)ring, ring_rows, rows_done};
  return encode_host(p, ring, host_out, capacity, total_bytes, rows_ready, &rg);
}
// wait (host) until the producer has published rows [0, r1) of the raster; false if it reported failure.
// `poll` runs on every spin (the ring path publishes finished H2D copies there, which the producer may need
// before it can publish r1)
extern "C++" template <typename F>
static bool wait_rows(const volatile int64_t* rows_ready, int64_t r1, F&& poll) {
  if (!rows_ready) return true;
  for (int spin = 0;; spin++) {
    const int64_t r = __atomic_load_n(const_cast<const int64_t*>(rows_ready), __ATOMIC_ACQUIRE);
    if (r < 0) return false;
    if (r >= r1) return true;
    poll();
    if (spin < 64) continue;
    struct timespec ts = {0, spin < 1024 ? 2000 : 50000};
    nanosleep(&ts, nullptr);
  }
}
static int encode_host(fra_plan* p, const void* host_raster, uint8_t* host_out, uint64_t capacity,
                       uint64_t* total_bytes, const volatile int64_t* rows_ready, const RingIn* ring) {
  if (!p || (!host_raster && p->raster_bytes) || (!host_out && capacity)) return set_err(FRA_E_INVALID, "null argument");
  (void)hipSetDevice(p->ctx->device);
  hipStream_t s = p->ctx->stream;
  const int nb = (int)p->hbands.size();
  if (total_bytes) *total_bytes = 0;
  if (nb == 0) {  // no windows
    p->executed = true;
    return FRA_OK;
  }
  if (int rc = drain_pipeline(p)) return rc;  // the bands below use buffer set 0 on the plan's stream
  if (!p->d_raster_owned && p->raster_bytes) HIPCHK(hipMalloc(&p->d_raster_owned, p->raster_bytes));
  p->d_raster = p->d_raster_owned;
  p->args.raster = p->d_raster;
  p->job.raster = host_raster;
  p->job.raster_on_device = 0;
  p->args.vec8 = (p->ld_vec8 && (uintptr_t)p->d_raster % 8 == 0) ? 1 : 0;
  if (!p->h2d) HIPCHK(hipStreamCreateWithFlags(&p->h2d, hipStreamNonBlocking));
  if (!p->d2h) HIPCHK(hipStreamCreateWithFlags(&p->d2h, hipStreamNonBlocking));
  if (!p->hev_start) HIPCHK(hipEventCreateWithFlags(&p->hev_start, hipEventDisableTiming));
  if ((int)p->hev.size() < 2 * nb) {
    for (auto& e : p->hev)
      if (e) (void)hipEventDestroy(e);
    p->hev.assign(2 * nb, nullptr);
    for (auto& e : p->hev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  if (!p->h_gbase) {
    HIPCHK(hipHostMalloc((void**)&p->h_gbase, sizeof(unsigned long long) * (nb + 1),
                         hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void**)&p->d_gbase_mirror, p->h_gbase, 0));
  }
  // H2D runs at most one band ahead of the oldest band whose D2H is not yet issued (unlimited measured
  // slower on C4: 22.2 vs 21.3 ms)
  constexpr int ahead = 1;
  // the copies must not overwrite the device raster while earlier work of this plan still reads it
  HIPCHK(hipEventRecord(p->hev_start, s));
  HIPCHK(hipStreamWaitEvent(p->h2d, p->hev_start, 0));
  HIPCHK(hipStreamWaitEvent(p->d2h, p->hev_start, 0));
  const uint8_t* host = (const uint8_t*)host_raster;
  // ring path: bands whose H2D copy is enqueued / known complete; completed bands free their ring rows
  int copies = 0, copied = 0;
  auto publish = [&]() {
    if (!ring) return;
    int64_t done = -1;
    while (copied < copies && hipEventQuery(p->hev[2 * copied]) == hipSuccess) done = p->hbands[copied++].r1;
    if (done >= 0) __atomic_store_n(const_cast<int64_t*>(ring->rows_done), done, __ATOMIC_RELEASE);
  };
  auto enqueue_copy = [&](int b) -> int {
    const auto& hb = p->hbands[b];
    if (!wait_rows(rows_ready, hb.r1, publish))
      return set_err(FRA_E_STATE, "the raster producer failed (rows_ready < 0)");
    if (hb.r1 > hb.r0) {
      const int rc = ring ? copy_rows_ring_h2d(p, *ring, hb.r0, hb.r1, p->h2d) : copy_rows_h2d(p, host, hb.r0, hb.r1, p->h2d);
      if (rc) return rc;
    }
    HIPCHK(hipEventRecord(p->hev[2 * b], p->h2d));
    copies = b + 1;
    publish();
    return FRA_OK;
  };
  uint64_t beg = 0;
  int issued = 0;  // bands whose D2H has been enqueued
  bool over = false;
  // a pageable output (the ring path's lazily committed frames): a D2H into it returns only once the runtime has
  // staged the whole copy, which would hold this loop -- and with it the next band's H2D and the producer's ring
  // rows -- for every band's frames; those copies go to worker threads instead
  // (the context's staging and streams: FRA_D2H_THREADS workers, default 4; held for this call -- a concurrent
  // encode on the same context copies through the runtime instead)
  fra_ctx* cx = p->ctx;
  std::unique_lock<std::mutex> stage_lk(cx->stage_mu, std::defer_lock);
  const bool out_pageable = capacity > 0 && !host_pinned(host_out) && stage_lk.try_lock();
  if (out_pageable && !cx->stage) {
    // built in locals and committed to the context only when every piece exists (a half-built staging
    // set would leave a worker pool with no threads that reports success without copying)
    const char* e = getenv("FRA_D2H_THREADS");
    const int n = std::min(std::max(e ? atoi(e) : 4, 1), 16);
    uint8_t* stage = nullptr;
    std::vector<hipStream_t> sts;
    hipError_t he = hipHostMalloc((void**)&stage, D2HWorker::kPiece * n, hipHostMallocPortable);
    for (int i = 0; he == hipSuccess && i < n; i++) {
      hipStream_t st = nullptr;
      he = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
      if (he == hipSuccess) sts.push_back(st);
    }
    if (he != hipSuccess) {
      for (auto st : sts) (void)hipStreamDestroy(st);
      if (stage) (void)hipHostFree(stage);
      return set_err(FRA_E_HIP, "D2H staging: %s", hipGetErrorString(he));
    }
    cx->stage = stage;
    cx->stage_n = n;
    cx->stage_st = std::move(sts);
  }
  D2HWorker dw(cx->device, out_pageable ? host_out : nullptr, p->d_out, cx->stage, cx->stage_st);
  auto enqueue_d2h = [&](int b) -> int {
    const uint64_t end = p->h_gbase[b + 1];
    if (end > capacity) over = true;
    if (!over && end > beg) {
      if (dw.on()) {
        dw.push(beg, end);
      } else {
        HIPCHK(hipStreamWaitEvent(p->d2h, p->hev[2 * b + 1], 0));
        HIPCHK(hipMemcpyAsync(host_out + beg, p->d_out + beg, (size_t)(end - beg), hipMemcpyDeviceToHost, p->d2h));
      }
    }
    beg = end;
    return FRA_OK;
  };
  // an error after work was enqueued (a failed producer, a HIP error): drain the three streams (and the D2H
  // worker) before returning, so no copy still reads or writes the caller's buffers
  auto drained = [&](int code) -> int {
    std::string keep = g_err;
    dw.finish();
    (void)hipStreamSynchronize(p->h2d);
    (void)hipStreamSynchronize(s);
    (void)hipStreamSynchronize(p->d2h);
    g_err = keep;
    return code;
  };
  // (a HIP error once copies are in flight also drains: the caller may free or refill its ring on return)
#define HIPCHK_D(x)                                                                                         \
  do {                                                                                                      \
    hipError_t _e = (x);                                                                                    \
    if (_e != hipSuccess)                                                                                   \
      return drained(set_err(FRA_E_HIP, "%s: %s (%s:%d)", #x, hipGetErrorString(_e), __FILE__, __LINE__)); \
  } while (0)
  int rc = enqueue_copy(0);
  if (rc) return drained(rc);
  for (int b = 0; b < nb; b++) {
    if (b + 1 < nb) {  // the next band's rows go over PCIe meanwhile
      while (ahead > 0 && b + 1 - issued > ahead) {
        HIPCHK_D(hipEventSynchronize(p->hev[2 * issued + 1]));
        if ((rc = enqueue_d2h(issued++))) return drained(rc);
      }
      if ((rc = enqueue_copy(b + 1))) return drained(rc);
    }
    HIPCHK_D(hipStreamWaitEvent(s, p->hev[2 * b], 0));
    // the band's end offset reaches h_gbase by a kernel store (k_group_offsets), not by a copy-engine
    // command that would queue behind the H2D copies
    rc = run_group(p, p->hbands[b].g, b, nb, s, nullptr, nullptr, nullptr, nullptr, nullptr, 0, p->d_gbase_mirror);
    if (rc) return drained(rc);
    HIPCHK_D(hipEventRecord(p->hev[2 * b + 1], s));
    // bands already assembled: their D2H can start now (pageable sources make the H2D enqueue blocking)
    while (issued <= b && hipEventQuery(p->hev[2 * issued + 1]) == hipSuccess)
      if ((rc = enqueue_d2h(issued++))) return drained(rc);
    publish();
  }
  while (issued < nb) {
    HIPCHK_D(hipEventSynchronize(p->hev[2 * issued + 1]));
    if ((rc = enqueue_d2h(issued++))) return drained(rc);
  }
  if (!dw.finish()) return drained(set_err(FRA_E_HIP, "frames D2H: %s", dw.error().c_str()));
  HIPCHK_D(hipStreamSynchronize(p->d2h));
  HIPCHK_D(hipStreamSynchronize(s));
  HIPCHK_D(hipStreamSynchronize(p->h2d));
#undef HIPCHK_D
  publish();
  p->executed = true;
  // a frame the assembly skipped or a frame-scan desync (the device error word) fails the call: the copied
  // frames are not a valid stream
  if ((rc = check_dev_err(p))) return rc;
  if (total_bytes) *total_bytes = beg;
  if (over)
    return set_err(FRA_E_SPACE, "output needs %llu bytes, capacity %llu (frames stay on the device)",
                   (unsigned long long)beg, (unsigned long long)capacity);
  return FRA_OK;
}

int fra_host_alloc(uint64_t bytes, void** ptr) {
  if (!ptr) return set_err(FRA_E_INVALID, "null argument");
  *ptr = nullptr;
  HIPCHK(hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocPortable));
  return FRA_OK;
}
int fra_host_free(void* ptr) {
  if (ptr) HIPCHK(hipHostFree(ptr));
  return FRA_OK;
}
int fra_host_register(void* ptr, uint64_t bytes) {
  if (!ptr || !bytes) return set_err(FRA_E_INVALID, "null argument");
  HIPCHK(hipHostRegister(ptr, bytes, hipHostRegisterPortable));
  return FRA_OK;
}
int fra_host_unregister(void* ptr) {
  if (ptr) HIPCHK(hipHostUnregister(ptr));
  return FRA_OK;
}

int fra_encode(int device, const fra_job* job, uint8_t** out, uint64_t* out_len, fra_stream_info* infos) {
  fra_ctx* ctx = nullptr;
  int rc = fra_ctx_create(device, &ctx);
  if (rc) return rc;
  fra_plan* p = nullptr;
  rc = fra_plan_create(ctx, job, &p);
  if (!rc) rc = fra_plan_execute(p);
  if (!rc) rc = fra_plan_sync(p);
  uint64_t total = 0;
  if (!rc) rc = fra_plan_result(p, infos, &total);
  if (!rc) {
    *out = (uint8_t*)malloc(total ? total : 1);
    if (!*out) rc = set_err(FRA_E_NOMEM, "malloc %llu", (unsigned long long)total);
    else rc = fra_plan_download(p, *out, total);
    if (rc) { free(*out); *out = nullptr; }
    *out_len = total;
  }
  std::string keep = g_err;
  fra_plan_destroy(p);
  fra_ctx_destroy(ctx);
  g_err = keep;
  return rc;
}

int fra_stream_header(uint8_t* o, int32_t channels, int32_t bps, int32_t sample_rate, int32_t blocksize) {
  if (!o || channels < 1 || channels > 8 || bps < 4 || bps > 32 || blocksize < 16 || blocksize > 65535 ||
      sample_rate <= 0 || sample_rate >= (1 << 20))
    return set_err(FRA_E_INVALID, "bad stream header parameters");
  memcpy(o, "fLaC", 4);
  o[4] = 0x00;  // STREAMINFO, not last
  o[5] = 0; o[6] = 0; o[7] = 34;
  uint8_t* si = o + 8;
  memset(si, 0, 34);
  si[0] = (uint8_t)(blocksize >> 8); si[1] = (uint8_t)blocksize;
  si[2] = (uint8_t)(blocksize >> 8); si[3] = (uint8_t)blocksize;
  // bytes 4..9 min/max frame size = 0
  // 20-bit sample rate | 3-bit channels-1 | 5-bit bps-1 | 36-bit total samples (0)
  si[10] = (uint8_t)(sample_rate >> 12);
  si[11] = (uint8_t)(sample_rate >> 4);
  si[12] = (uint8_t)(((sample_rate & 0xF) << 4) | ((channels - 1) << 1) | ((bps - 1) >> 4));
  si[13] = (uint8_t)(((bps - 1) & 0xF) << 4);
  // MD5 zero
  uint8_t* vc = o + 42;
  const uint32_t vlen = (uint32_t)(sizeof(kVendor) - 1);
  const uint32_t blen = 4 + vlen + 4;
  vc[0] = 0x84;  // last | VORBIS_COMMENT
  vc[1] = (uint8_t)(blen >> 16); vc[2] = (uint8_t)(blen >> 8); vc[3] = (uint8_t)blen;
  vc[4] = (uint8_t)vlen; vc[5] = (uint8_t)(vlen >> 8); vc[6] = (uint8_t)(vlen >> 16); vc[7] = (uint8_t)(vlen >> 24);
  memcpy(vc + 8, kVendor, vlen);
  memset(vc + 8 + vlen, 0, 4);
  return FRA_OK;  // 42 + 4 + 40 = 86 bytes
}

int fra_normalize(fra_ctx* ctx, const void* data, int32_t on_device, int32_t dtype, uint64_t n, int32_t bps,
                  const double* data_min, const double* data_max, void* out_host, double* mn_out, double* mx_out) {
  if (!ctx || (!data && n) || (!out_host && n)) return set_err(FRA_E_INVALID, "null argument");
  if (dtype < FRA_U8 || dtype > FRA_F64) return set_err(FRA_E_INVALID, "bad dtype %d", dtype);
  (void)hipSetDevice(ctx->device);
  hipStream_t s = ctx->stream;
  const size_t in_bytes = (size_t)n * elem_size(dtype);
  const size_t out_bytes = (size_t)n * (bps == 16 ? 2 : 4);
  void* d_in = nullptr;
  void* d_out = nullptr;
  NormDev* d_nd = nullptr;
  int rc = FRA_OK;
  auto fail = [&](hipError_t e, const char* what) {
    rc = set_err(FRA_E_HIP, "%s: %s", what, hipGetErrorString(e));
  };
  hipError_t e = hipSuccess;
  if (!on_device && n) {
    if ((e = hipMalloc(&d_in, in_bytes)) != hipSuccess) fail(e, "hipMalloc");
    else if ((e = hipMemcpyAsync(d_in, data, in_bytes, hipMemcpyHostToDevice, s)) != hipSuccess) fail(e, "h2d");
  }
  if (!rc && (e = hipMalloc(&d_out, std::max<size_t>(4, out_bytes))) != hipSuccess) fail(e, "hipMalloc");
  if (!rc && (e = hipMalloc(&d_nd, sizeof(NormDev))) != hipSuccess) fail(e, "hipMalloc");
  if (!rc && (e = launch_normalize_flat(dtype, on_device ? data : d_in, n, bps, d_nd, data_min != nullptr,
                                        data_min ? *data_min : 0.0, data_max != nullptr, data_max ? *data_max : 0.0,
                                        d_out, s)) != hipSuccess)
    fail(e, "normalize kernels");
  NormDev nd{};
  if (!rc && out_bytes && (e = hipMemcpyAsync(out_host, d_out, out_bytes, hipMemcpyDeviceToHost, s)) != hipSuccess)
    fail(e, "d2h");
  if (!rc && (e = hipMemcpyAsync(&nd, d_nd, sizeof(NormDev), hipMemcpyDeviceToHost, s)) != hipSuccess) fail(e, "d2h");
  if (!rc && (e = hipStreamSynchronize(s)) != hipSuccess) fail(e, "sync");
  if (!rc) {
    if (mn_out) *mn_out = nd.mn;
    if (mx_out) *mx_out = nd.mx;
  }
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  (void)hipFree(d_nd);
  return rc;
}

int fra_synth_raster(fra_ctx* ctx, int32_t kind, uint64_t seed, int32_t bands, int32_t height, int32_t width,
                     void* dev_out) {
  if (!ctx || !dev_out || bands < 1 || height < 1 || width < 1 || (kind != 3 && kind != 4 && kind != 5))
    return set_err(FRA_E_INVALID, "bad synth arguments");
  (void)hipSetDevice(ctx->device);
  HIPCHK(launch_synth(kind, seed, bands, height, width, dev_out, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return FRA_OK;
}

int fra_device_alloc(fra_ctx* ctx, uint64_t bytes, void** p) {
  (void)hipSetDevice(ctx->device);
  HIPCHK(hipMalloc(p, bytes ? bytes : 1));
  return FRA_OK;
}
int fra_device_free(fra_ctx* ctx, void* p) {
  (void)hipSetDevice(ctx->device);
  HIPCHK(hipFree(p));
  return FRA_OK;
}
int fra_memcpy_d2h(fra_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
  (void)hipSetDevice(ctx->device);
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return FRA_OK;
}
int fra_memcpy_h2d(fra_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
  (void)hipSetDevice(ctx->device);
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return FRA_OK;
}

}  // extern "C"
