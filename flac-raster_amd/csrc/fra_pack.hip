// fra_pack.hip -- the frame assembly kernel (the per-frame device code, its gather formulation and the
// CRC-16 scheme are in fra_assemble.h): k_assemble4, one frame per wave, four per workgroup.  (r04: the
// background form k_assemble_bg for pipelined 32-bps plans was removed once the 32-bps analysis fills a CU
// with five workgroups -- C5 step 109.3 ms with it, 106.8 with k_assemble4, profiles/r04_ab_c5_assemble4_vs_bg.txt.)
#include <cstdlib>

#include "fra_assemble.h"

namespace fra {
// quads per lane per round (r05: 1, 30 VGPRs -- with the lighter LDS tables, FRA_ASM_LIGHT in fra_assemble.h, three
// workgroups (12 waves) per CU fit beside 4 waves per SIMD of the 16-bit k_analyze_w instead of 8 waves: the assembly of
// a pipelined execute, which gated the next analysis's start (its slots), keeps up -- C4 step 1.461 -> 1.411 ms, C3 /
// C5 quarter / 8-way share neutral, profiles/r05_ab_background.txt 10; alone it is 0.282 -> 0.295 ms)
#ifndef FRA_ASM_U
#define FRA_ASM_U 1
#endif

// four frames per workgroup, one per wave -- the 17.5 KiB of CRC tables are copied to LDS
// once for four frames (a C3 frame is only ~7 KiB) and a frame needs no workgroup barrier.  r03 v20: C4
// k_assemble 0.302 -> 0.272 ms (step 2.03 -> 1.98 ms), C3 0.310 -> 0.209 ms (step 1.38 -> 1.27 ms); two quads
// per thread per round beat four (`profiles/r03_ab_assemble_per_wave_v20.txt`)
__global__ void __launch_bounds__(kThreads, 8) k_assemble4(JobArgs a) {
  __shared__ AssembleSmem S;
  if (FRA_BG_PRIO > 0) __builtin_amdgcn_s_setprio(FRA_BG_PRIO);  // (wave issue priority: fra_internal.h)
  copy_tables(a, S);
  __syncthreads();
  const int i = (int)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  if (i < a.frame_count) assemble_frame<FRA_ASM_U>(a, a.frame_base + i, S);
}

hipError_t launch_assemble(const JobArgs& a, hipStream_t s) {
  if (a.frame_count <= 0) return hipSuccess;
  k_assemble4<<<(unsigned)((a.frame_count + 3) / 4), kThreads, 0, s>>>(a);
  return hipGetLastError();
}

}  // namespace fra
