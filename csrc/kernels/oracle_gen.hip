// Fused sentiment -> stochastic oracles: one workgroup per comment window (= consensus instance),
// one lane per oracle slot; the slot permutation is built once per window in LDS.
#include <hip/hip_runtime.h>

#include "svoc/bootstrap.hpp"

namespace svoc {

__global__ __launch_bounds__(256) void bootstrap_kernel(BootParams p) {
  __shared__ int perm[256];
  const int w = blockIdx.x;
  if (threadIdx.x == 0) boot_perm(p, w, perm);
  __syncthreads();
  for (int j = threadIdx.x; j < p.N; j += blockDim.x) {
    float v[16];
    boot_slot(p, w, j, v);
    float* dst = p.out + ((int64_t)w * p.N + perm[j]) * p.D;
    for (int d = 0; d < p.D; ++d) dst[d] = v[d];
  }
}

}  // namespace svoc

extern "C" int svoc_bootstrap(const svoc::BootParams* p, hipStream_t s) {
  if (p->W <= 0) return 0;
  if (p->N > 256 || p->D > 16 || p->C > 64) return -1;
  hipLaunchKernelGGL(svoc::bootstrap_kernel, dim3(p->W), dim3(256), 0, s, *p);
  return (int)hipGetLastError();
}
