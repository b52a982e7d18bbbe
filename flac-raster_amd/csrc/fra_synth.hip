// fra_synth.hip -- synthetic rasters for the benchmark configurations.
//
// All arithmetic is integer (splitmix64 hashes, fixed-point bilinear value noise, Irwin-Hall
// pseudo-Gaussian), so flac_raster/synth.py reproduces any window bit for bit on the CPU; the C5
// float32 values are one correctly-rounded double division followed by a cast, done identically
// on both sides.  Kinds:
//   3  C3 DEM-like int16            550 + terrain value noise (scales 1024/256) + uniform 0..50
//   4  C4 Sentinel-2-L1C-like uint16 per-band mean + 600*(3-octave value noise 512/128/32)
//                                   + N(0,15)-like DN noise, clip [1, 11672], nodata corner
//   5  C5 reflectance float32        0.15 + 0.1*noise + N(0,0.002)-like, clip [0, 1.2]
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fra {

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ inline uint32_t lattice(uint64_t seed, int b, int oct, uint32_t ix, uint32_t iy) {
  return (uint32_t)(splitmix64(seed ^ ((uint64_t)b << 56) ^ ((uint64_t)oct << 48) ^ ((uint64_t)iy << 24) ^ ix) & 0xFFFFu);
}
// bilinear value noise in [0, 65535] at scale 2^ls
__device__ inline uint32_t vnoise(uint64_t seed, int b, int oct, int ls, uint32_t row, uint32_t col) {
  const uint32_t s = 1u << ls;
  const uint32_t ix = col >> ls, iy = row >> ls, fx = col & (s - 1), fy = row & (s - 1);
  const uint64_t v00 = lattice(seed, b, oct, ix, iy), v10 = lattice(seed, b, oct, ix + 1, iy);
  const uint64_t v01 = lattice(seed, b, oct, ix, iy + 1), v11 = lattice(seed, b, oct, ix + 1, iy + 1);
  const uint64_t top = v00 * (s - fx) + v10 * fx;
  const uint64_t bot = v01 * (s - fx) + v11 * fx;
  return (uint32_t)((top * (s - fy) + bot * fy) >> (2 * ls));
}
// Irwin-Hall(4 bytes) - 510, sigma ~ 147.8
__device__ inline int32_t ih4(uint64_t seed, int b, uint32_t row, uint32_t col) {
  const uint64_t h = splitmix64(seed ^ 0xA5A5A5A5A5A5A5A5ull ^ ((uint64_t)b << 56) ^ ((uint64_t)row << 28) ^ col);
  return (int32_t)((h & 0xFF) + ((h >> 8) & 0xFF) + ((h >> 16) & 0xFF) + ((h >> 24) & 0xFF)) - 510;
}
__device__ inline int32_t tdiv(int64_t a, int64_t b) { return (int32_t)(a / b); }  // C truncation

__global__ void k_synth(int kind, uint64_t seed, int bands, int H, int W, void* out) {
  const int64_t total = (int64_t)bands * H * W;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / ((int64_t)H * W));
    const int64_t rem = e - (int64_t)b * H * W;
    const uint32_t row = (uint32_t)(rem / W), col = (uint32_t)(rem - (int64_t)row * W);
    if (kind == 3) {
      const uint32_t n1 = vnoise(seed, b, 0, 10, row, col), n2 = vnoise(seed, b, 1, 8, row, col);
      const uint64_t h = splitmix64(seed ^ 0x5151515151515151ull ^ ((uint64_t)row << 28) ^ col);
      const int32_t v = 550 + (int32_t)(n1 * 600u / 65535u) + (int32_t)(n2 * 300u / 65535u) + (int32_t)(h % 51u);
      ((int16_t*)out)[e] = (int16_t)v;
    } else if (kind == 4) {
      const int32_t means[4] = {1200, 1100, 1000, 2500};
      const uint32_t nz = 4u * vnoise(seed, b, 0, 9, row, col) + 2u * vnoise(seed, b, 1, 7, row, col) +
                          vnoise(seed, b, 2, 5, row, col);
      const int32_t dn = (int32_t)((uint64_t)nz * 1200u / 458745u) - 600;
      const int32_t g = tdiv((int64_t)ih4(seed, b, row, col) * 15, 148);
      int32_t v = means[b & 3] + dn + g;
      v = v < 1 ? 1 : (v > 11672 ? 11672 : v);
      const int64_t tri = ((int64_t)(H + W) * 158) / 1000;
      if ((int64_t)row + col < tri) v = 0;
      ((uint16_t*)out)[e] = (uint16_t)v;
    } else {
      const int32_t nz = 2 * (int32_t)vnoise(seed, b, 0, 9, row, col) + (int32_t)vnoise(seed, b, 1, 6, row, col) - 3 * 32767;
      const int32_t g = tdiv((int64_t)ih4(seed, b, row, col) * 200, 148);
      int32_t v = 15000 + tdiv((int64_t)nz * 10000, 3 * 65535) + g;
      v = v < 0 ? 0 : (v > 120000 ? 120000 : v);
      ((float*)out)[e] = (float)((double)v / 100000.0);
    }
  }
}

hipError_t launch_synth(int kind, uint64_t seed, int bands, int H, int W, void* out, hipStream_t s) {
  k_synth<<<4096, 256, 0, s>>>(kind, seed, bands, H, W, out);
  return hipGetLastError();
}

}  // namespace fra
