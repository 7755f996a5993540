// Round prologue / epilogue: two launches replace ~30 small ATen kernels per step (mask
// arithmetic, status tests, reductions), which cost ~190 us per step on the c2 config.
#include <hip/hip_runtime.h>

#include "svoc/bookkeeping.hpp"

namespace svoc {

__global__ __launch_bounds__(256) void round_prologue_kernel(RoundBook r) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b < r.B) r.active[b] = book_active(r, b);
}

// grid-stride over the instances with at most EPI_BLOCKS workgroups: the four counter atomics per
// workgroup then number a few thousand instead of B/64 (1M instances: 16k same-address atomics)
constexpr int EPI_BLOCKS = 512;

__global__ __launch_bounds__(256) void round_epilogue_kernel(RoundBook r) {
  unsigned long long v[4] = {0, 0, 0, 0};
  for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < r.B; b += (int64_t)gridDim.x * 256) {
    const bool act = r.active[b] != 0;
    const bool ok = book_ok(r, b);
    if (ok) {
      r.consensus_active[b] = 1;
      v[0] += book_rel2_fx(r, b);
      v[1] += 1;
    }
    v[2] += act ? 1 : 0;
    v[3] += (act && !ok) ? 1 : 0;
    r.touched[b] = 0;
  }
  if (r.acc == nullptr) return;
  __shared__ unsigned long long part[4][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    unsigned long long x = v[k];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) part[wave][k] = x;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const unsigned long long s = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] +
                                 part[3][threadIdx.x];
    if (s) atomicAdd(&r.acc[threadIdx.x], s);
  }
}

}  // namespace svoc

using namespace svoc;

extern "C" int svoc_round_prologue(const RoundBook* r, hipStream_t stream) {
  if (r->B <= 0) return 0;
  hipLaunchKernelGGL(round_prologue_kernel, dim3((unsigned)((r->B + 255) / 256)), dim3(256), 0, stream, *r);
  return (int)hipGetLastError();
}

extern "C" int svoc_round_epilogue(const RoundBook* r, hipStream_t stream) {
  if (r->B <= 0) return 0;
  const int64_t blocks = (r->B + 255) / 256;
  hipLaunchKernelGGL(round_epilogue_kernel, dim3((unsigned)(blocks < EPI_BLOCKS ? blocks : EPI_BLOCKS)), dim3(256), 0,
                     stream, *r);
  return (int)hipGetLastError();
}
