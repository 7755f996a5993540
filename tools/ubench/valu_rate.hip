// VALU issue-rate probe: wave64 min/max (u32), packed u16 min/max, f32 add and permlane32 swaps, with 1, 2
// and 4 waves per SIMD (one 256 / 512 / 1024-thread workgroup per CU).  Cycles per instruction per SIMD =
// elapsed * clock / (instructions per SIMD).  hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REPS 4096
template <int OP>
__global__ void probe(uint32_t* out, uint32_t seed) {
  uint32_t r[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = seed * (threadIdx.x + i * 77u) ^ (i * 0x9e3779b9u);
  for (int it = 0; it < REPS; ++it) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        // even half: pairs (2i, 2i+1); odd half: pairs (i, i+8) -- no register moves between them
        const int ia = h ? i : 2 * i, ib = h ? i + 8 : 2 * i + 1;
        uint32_t a = r[ia], b = r[ib];
        if constexpr (OP == 0) {   // u32 min/max compare-exchange
          r[ia] = a < b ? a : b; r[ib] = a < b ? b : a;
        } else if constexpr (OP == 1) {   // packed u16
          typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
          u16x2 x = __builtin_bit_cast(u16x2, a), y = __builtin_bit_cast(u16x2, b);
          r[ia] = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(x, y));
          r[ib] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, y));
        } else if constexpr (OP == 2) {   // f32 add
          float x = __builtin_bit_cast(float, a), y = __builtin_bit_cast(float, b);
          r[ia] = __builtin_bit_cast(uint32_t, x + y); r[ib] = __builtin_bit_cast(uint32_t, y + x * 0.5f);
        } else if constexpr (OP == 3) {   // permlane32 swap (2 regs) + min/max
          const auto t = __builtin_amdgcn_permlane32_swap(a, b, false, false);
          r[ia] = t[0] < t[1] ? t[0] : t[1]; r[ib] = t[0] < t[1] ? t[1] : t[0];
        } else {   // min3 / max3 (3-input)
          uint32_t c = r[(ib + 3) & 15];
          r[ia] = __builtin_elementwise_min(__builtin_elementwise_min(a, b), c);
          r[ib] = __builtin_elementwise_max(__builtin_elementwise_max(a, b), c);
        }
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc ^= r[i];
  if (acc == 0x12345678u) out[0] = acc;
}

template <int OP>
static void run(const char* name, int threads, uint32_t* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int grid = 256 * 8;   // 8 workgroups per CU over time (fills every CU)
  hipLaunchKernelGGL(probe<OP>, dim3(grid), dim3(threads), 0, 0, d, 1u);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe<OP>, dim3(grid), dim3(threads), 0, 0, d, 2u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double waves = (double)grid * threads / 64;
  const double instr = waves * REPS * 32.0;   // 32 ops per iteration (2 x 8 pairs x 2); perm: +16 swaps
  // per-SIMD instruction rate: 1024 SIMDs
  const double per_simd = instr / 1024.0;
  printf("%-10s threads/WG %4d: %8.3f ms  %.3f ns per wave-instruction per SIMD (x2.1GHz = %.2f cyc)\n", name, threads,
         ms, ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.1);
}

int main() {
  uint32_t* d; hipMalloc(&d, 4);
  for (int t : {256, 512, 1024}) {
    run<0>("min/max", t, d);
    run<1>("pk_u16", t, d);
    run<2>("f32add", t, d);
    run<3>("perm32+mm", t, d);
    run<4>("min3max3", t, d);
  }
  return 0;
}
