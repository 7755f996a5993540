// Phase-A stream rate of the c3 fp32 window kernel's LDS-DMA pattern, without its compute: 512
// instances x [256 rows x 4096 fp32] (2 GiB), one 4-wave workgroup per instance, 2 workgroups per CU,
// every wave owning one 16-KiB LDS region (one slab in flight per wave, as consensus_fast_winf.hip).
// Per slab step a wave waits for its DMA, copies 64 words per lane out of LDS, issues the next slab
// and spends `spin` dependent VALU ops (the non-network work of a slab is ~600).
// Variants (what one wave's 16 KiB covers):
//   0: its 16 columns x 256 rows of the step's 64-column slab (64 B per row piece; the kernel today)
//   1: 64 rows x the 64 columns (256 B per row piece); the 4 waves' regions form the workgroup's slab,
//      exchanged through LDS behind two workgroup barriers per step
//   2: 16 KiB contiguous (what a [column tile][row][16 columns] storage layout would give)
// hipcc --offload-arch=gfx950 -O3 -I../../csrc/include dma_rate.hip -o dma_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "svoc/bufload.hpp"

using namespace svoc;

constexpr int N = 256, D = 4096, ROWB = D * 4;

__device__ __forceinline__ void dma16(const BufDesc& rs, uint32_t* region, int vo, int soff_step) {
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)(region + k * 256);
    int keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(vo), "s"(rs.w), "s"(lds), "s"(k * soff_step)
        : "memory");
  }
}

template <int VAR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void stream(const float* vals, uint32_t* out,
                                                                                       int spin) {
  __shared__ uint32_t slab[4 * 64 * 64];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float* inst = vals + (size_t)b * N * D;
  const BufDesc rsd = buf_desc(inst, (uint32_t)(N * ROWB));
  uint32_t* region = slab + wave * 4096;
  // per-lane voffset of piece 0 and the per-piece soffset step, by variant
  int vlane, pstep;
  if (VAR == 0) {          // 4 lanes x 16 B per row, 16 rows per piece; column block 16 * wave
    vlane = (lane / 4) * ROWB + (lane % 4) * 16;
    pstep = 16 * ROWB;
  } else if (VAR == 1) {   // 16 lanes x 16 B per row (256 B), 4 rows per piece; rows 64 * wave
    vlane = (64 * wave + lane / 16) * ROWB + (lane % 16) * 16;
    pstep = 4 * ROWB;
  } else {                 // contiguous: this wave's 16 KiB tile
    vlane = lane * 16;
    pstep = 1024;
  }
  const int nslab = D / 64;
  auto col0 = [&](int s) { return VAR == 0 ? (s * 64 + wave * 16) * 4 : VAR == 1 ? s * 64 * 4 : (s * 4 + wave) * 16384; };
  dma16(rsd, region, vlane + col0(0), pstep);
  uint32_t acc = 0;
  for (int s = 0; s < nslab; ++s) {
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    if (VAR == 1) __syncthreads();
    uint32_t x[64];
    const uint32_t* src = VAR == 1 ? slab + (lane / 16) * 4096 + (lane % 16) : region + lane;
#pragma unroll
    for (int i = 0; i < 64; ++i) x[i] = src[i * 64];
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
    if (VAR == 1) __syncthreads();
    if (s + 1 < nslab) dma16(rsd, region, vlane + col0(s + 1), pstep);
#pragma unroll
    for (int i = 0; i < 64; ++i) acc = acc * 3u + x[i];
    for (int t = 0; t < spin; ++t) acc = (acc ^ (acc >> 3)) + 0x9e3779b9u;
  }
  out[b * 256 + tid] = acc;
}

int main() {
  const int B = 512;
  float* vals;
  uint32_t* out;
  hipMalloc(&vals, (size_t)B * N * D * 4);
  hipMalloc(&out, (size_t)B * 256 * 4);
  hipMemset(vals, 0x3c, (size_t)B * N * D * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int spin : {0, 150, 300}) {
    for (int var = 0; var < 3; ++var) {
      float best = 1e9f;
      for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(e0);
        if (var == 0) hipLaunchKernelGGL(stream<0>, dim3(B), dim3(256), 0, 0, vals, out, spin);
        else if (var == 1) hipLaunchKernelGGL(stream<1>, dim3(B), dim3(256), 0, 0, vals, out, spin);
        else hipLaunchKernelGGL(stream<2>, dim3(B), dim3(256), 0, 0, vals, out, spin);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep && ms < best) best = ms;
      }
      printf("variant %d spin %3d: %.1f us, %.2f TB/s\n", var, spin, best * 1e3, (double)B * N * D * 4 / (best * 1e-3) / 1e12);
    }
  }
  return 0;
}
