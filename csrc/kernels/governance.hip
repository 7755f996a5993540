// Batched admin replacement voting: one lane per (instance, action).  A <= 64 admins so the vote
// matrix column is one uint64 and the majority count is one popcount (K7 in the survey).
#include <hip/hip_runtime.h>

#include "svoc/governance.hpp"

namespace svoc {

__global__ __launch_bounds__(256) void governance_kernel(GovState g, GovAction a) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.K) return;
  a.status[k] = gov_apply_one(g, a, k);
}

}  // namespace svoc

extern "C" int svoc_governance(const svoc::GovState* g, const svoc::GovAction* a, hipStream_t s) {
  if (a->K <= 0) return 0;
  hipLaunchKernelGGL(svoc::governance_kernel, dim3((a->K + 255) / 256), dim3(256), 0, s, *g, *a);
  return (int)hipGetLastError();
}
