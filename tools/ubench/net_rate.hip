// Issue rate of the c3 fp32 window network (window_group<4, 16, 17> on u32 keys, sortnet.hpp) alone, on
// registers: 1 / 2 waves per SIMD.  ns per network per SIMD vs its VALU count (from the ISA) tells
// whether the network itself runs at the pipe rate (profiles/r3_valu_rate_probe.txt: ~1.7 ns / instr).
// hipcc --offload-arch=gfx950 -O3 -I../../csrc/include net_rate.hip -o net_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "svoc/sortnet.hpp"

using namespace svoc;
#define REPS 64

__global__ __launch_bounds__(256) void net(const uint32_t* in, uint32_t* out) {
  const int lane = threadIdx.x & 63, seg = lane / 16;
  uint32_t r[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) r[i] = in[(blockIdx.x * 256 + threadIdx.x) * 64 % 65536 + i];
  uint32_t acc = 0;
  for (int it = 0; it < REPS; ++it) {
    uint32_t w[17], lo, hi;
    uint32_t t[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) t[i] = r[i] ^ (uint32_t)it;
    window_group<4, 16, 17>(t, seg, lane, w, lo, hi);
#pragma unroll
    for (int m = 0; m < 17; ++m) acc += w[m];
    acc ^= lo + hi;
    r[0] += acc;   // keep the inputs changing
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  uint32_t *in, *out;
  hipMalloc(&in, 65536 * 4 + 4096 * 4);
  hipMalloc(&out, 2048 * 1024 * 4);
  hipMemset(in, 0x5a, 65536 * 4 + 4096 * 4);
  for (int wpc : {4, 8}) {   // waves per CU: 1 or 2 per SIMD (256-thread workgroups)
    const int grid = 256 * wpc / 4 * 4;   // 4 rounds of full occupancy
    hipLaunchKernelGGL(net, dim3(grid), dim3(256), 0, 0, in, out);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(net, dim3(grid), dim3(256), 0, 0, in, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double nets_per_simd = (double)grid * 4 * REPS / 1024.0;   // waves x reps / SIMDs
    printf("waves/CU %d: %.3f ms, %.1f ns per network per SIMD\n", wpc, ms, ms * 1e6 / nets_per_simd);
  }
  return 0;
}
