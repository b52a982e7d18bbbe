// fra_pack.hip -- the frame assembly kernels (the per-frame device code, its gather formulation and the
// CRC-16 scheme are in fra_assemble.h), both one frame per wave:
// * k_assemble4: four frames per workgroup (serial executes, and pipelined 16-bit plans on the pack stream);
// * k_assemble_bg: background form for pipelined 32-bps plans (see below).
#include <cstdlib>

#include "fra_assemble.h"

namespace fra {

// background form for the pipelined execute, where it runs beside the next execute's k_analyze: a
// k_analyze<16-bit> CU holds 6 workgroups of 80 VGPRs and <= 94 SGPRs per wave, leaving per SIMD 32 VGPRs
// and 128 of the 800 SGPRs (ceil(n/16)*16 + 16 per wave), and ~26 KiB of LDS per CU; a 32-bps CU (4
// workgroups) leaves 96 VGPRs and 12.6 KiB.  At <= 32 VGPRs (one quad per thread per round), <= 96 SGPRs
// and 9.3 KiB of LDS one workgroup fits into that remainder instead of taking the place of an analysis
// workgroup; a grid of about one workgroup per CU strides over the frames and copies the CRC tables once.
// (amdgpu_num_vgpr counts pairs of gfx950's unified VGPR/AGPR file: 16 -> 32 VGPRs.)
__global__ void __attribute__((amdgpu_flat_work_group_size(kThreads, kThreads), amdgpu_num_vgpr(16),
                               amdgpu_num_sgpr(96))) k_assemble_bg(JobArgs a) {
  __shared__ AssembleSmemBg S;
  // one frame per wave, each wave striding over the frames on its own (no workgroup barrier per frame)
  copy_tables(a, S);
  __syncthreads();
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  for (int i = (int)blockIdx.x * 4 + w; i < a.frame_count; i += (int)gridDim.x * 4)
    assemble_frame<1>(a, a.frame_base + i, S);
}

// the default: four frames per workgroup, one per wave -- the 17.5 KiB of CRC tables are copied to LDS
// once for four frames (a C3 frame is only ~7 KiB) and a frame needs no workgroup barrier.  r03 v20: C4
// k_assemble 0.302 -> 0.272 ms (step 2.03 -> 1.98 ms), C3 0.310 -> 0.209 ms (step 1.38 -> 1.27 ms); two quads
// per thread per round beat four (`profiles/r03_ab_assemble_per_wave_v20.txt`)
__global__ void __launch_bounds__(kThreads, 8) k_assemble4(JobArgs a) {
  __shared__ AssembleSmem S;
  copy_tables(a, S);
  __syncthreads();
  const int i = (int)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  if (i < a.frame_count) assemble_frame<2>(a, a.frame_base + i, S);
}

hipError_t launch_assemble(const JobArgs& a, hipStream_t s, int bg_blocks) {
  if (a.frame_count <= 0) return hipSuccess;
  if (bg_blocks > 0) k_assemble_bg<<<(unsigned)std::min(bg_blocks, a.frame_count), kThreads, 0, s>>>(a);
  else k_assemble4<<<(unsigned)((a.frame_count + 3) / 4), kThreads, 0, s>>>(a);
  return hipGetLastError();
}

}  // namespace fra
