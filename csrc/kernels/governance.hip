// Batched admin replacement voting: one lane per (instance, action), or one lane per instance's run of
// actions (ordered batches).  A <= 64 admins so the vote
// matrix column is one uint64 and the majority count is one popcount (K7 in the survey).
#include <hip/hip_runtime.h>

#include "svoc/governance.hpp"

namespace svoc {

__global__ __launch_bounds__(256) void governance_kernel(GovState g, GovAction a) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.K) return;
  a.status[k] = gov_apply_one(g, a, k);
}

// Ordered batches: `order` lists the actions sorted stably by instance (a device sort; no host wave split).
// The lane at the head of each instance's run applies that run in submission order -- the reference's
// per-contract transaction order (the sequencer serialises one contract's transactions) -- and every other
// lane exits; instances are independent, so the runs proceed in parallel in one launch.
__global__ __launch_bounds__(256) void governance_seq_kernel(GovState g, GovAction a) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.K) return;
  const int64_t b = a.inst[a.order[p]];
  if (p > 0 && a.inst[a.order[p - 1]] == b) return;   // not the head of its instance's run
  for (int q = p; q < a.K; ++q) {
    const int k = (int)a.order[q];
    if (a.inst[k] != b) break;
    a.status[k] = gov_apply_one(g, a, k);
  }
}

}  // namespace svoc

extern "C" int svoc_governance(const svoc::GovState* g, const svoc::GovAction* a, hipStream_t s) {
  if (a->K <= 0) return 0;
  if (a->order)
    hipLaunchKernelGGL(svoc::governance_seq_kernel, dim3((a->K + 255) / 256), dim3(256), 0, s, *g, *a);
  else
    hipLaunchKernelGGL(svoc::governance_kernel, dim3((a->K + 255) / 256), dim3(256), 0, s, *g, *a);
  return (int)hipGetLastError();
}
