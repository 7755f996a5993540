// Batched update_prediction storage step (contract.cairo:331-343, :588-603): validate each update
// (constrained inputs must lie in [0, 1] / [0, WSAD]: 'interval error', math.cairo:298-310),
// pick the last valid writer per (instance, oracle) with an atomicMax on the update sequence
// number (coalescing is exact: survey §2.8-13), copy the winning rows with 16-B vector stores,
// flip `enabled` and bump n_active_oracles on first commit.  Three launches, no host sync.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svoc/launch.hpp"
#include "svoc/status.hpp"

namespace svoc {

__device__ __forceinline__ bool in_range(const UpdateParams& p, int64_t u, int d) {
  if (p.dtype == 0) {
    const uint16_t raw = ((const uint16_t*)p.upd)[u * p.D + d];
    const float f = __builtin_bit_cast(float, (uint32_t)raw << 16);
    return f >= 0.f && f <= 1.f;
  } else if (p.dtype == 1) {
    const float f = ((const float*)p.upd)[u * p.D + d];
    return f >= 0.f && f <= 1.f;
  }
  const int64_t v = ((const int64_t*)p.upd)[u * p.D + d];
  return v >= 0 && v <= 1000000;
}

__device__ __forceinline__ bool bf16_unit(uint32_t raw16) {  // 0 <= x <= 1 (and -0.0)
  return raw16 <= 0x3f80u || raw16 == 0x8000u;
}

// one wave per update: validate (wave-parallel over D, 16-B loads when rows allow), then claim the
// (instance, oracle) slot with an atomicMax on the update's sequence number
__global__ __launch_bounds__(256) void upd_validate_kernel(UpdateParams p) {
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (u >= p.U) return;
  const int64_t b = p.inst[u], o = p.oracle[u];
  int st = ST_OK;
  if (b < 0 || b >= p.B || o < 0 || o >= p.N) st = ST_NOT_ORACLE;
  if (st == ST_OK && p.constrained) {
    bool ok = true;
    const uint16_t* row = (const uint16_t*)p.upd + u * p.D;
    if (p.dtype == 0 && (p.D & 7) == 0 && (((uintptr_t)row) & 15) == 0) {
      for (int c = lane; c < p.D / 8; c += 64) {
        const uint4 v = ((const uint4*)row)[c];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) ok = ok && bf16_unit(w[k] & 0xffffu) && bf16_unit(w[k] >> 16);
      }
    } else {
      for (int d = lane; d < p.D; d += 64) ok = ok && in_range(p, u, d);
    }
    if (!__all(ok)) st = ST_INTERVAL_INPUT;
  }
  if (lane == 0) {
    p.upd_status[u] = st;
    if (st == ST_OK) atomicMax(&p.winner[b * p.N + o], (int)u);
  }
}

// one workgroup per update: the winner copies its row
__global__ __launch_bounds__(256) void upd_apply_kernel(UpdateParams p) {
  const int64_t u = blockIdx.x;
  if (p.upd_status[u] != ST_OK) return;
  const int64_t b = p.inst[u], o = p.oracle[u];
  if (p.winner[b * p.N + o] != (int)u) return;  // superseded by a later update: coalesced
  const int64_t row_bytes = (int64_t)p.D * p.elem_bytes;
  unsigned char* dst = (unsigned char*)p.values + (b * p.inst_stride + o * p.ld) * p.elem_bytes;
  const unsigned char* src = (const unsigned char*)p.upd + u * row_bytes;
  if (((uintptr_t)dst & 15) == 0 && ((uintptr_t)src & 15) == 0 && (row_bytes & 15) == 0) {
    for (int64_t i = threadIdx.x; i < row_bytes / 16; i += blockDim.x)
      ((uint4*)dst)[i] = ((const uint4*)src)[i];
  } else {
    for (int64_t i = threadIdx.x; i < row_bytes; i += blockDim.x) dst[i] = src[i];
  }
  if (threadIdx.x == 0) {
    if (!p.enabled[b * p.N + o]) {
      p.enabled[b * p.N + o] = 1;
      atomicAdd(&p.n_active[b], 1);
    }
    p.touched[b] = 1;
  }
}

__global__ __launch_bounds__(256) void upd_reset_kernel(UpdateParams p) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= p.U || p.upd_status[u] != ST_OK) return;
  p.winner[p.inst[u] * p.N + p.oracle[u]] = -1;
}

}  // namespace svoc

using namespace svoc;

extern "C" int svoc_apply_updates(const UpdateParams* p, hipStream_t stream) {
  if (p->U <= 0) return 0;
  hipLaunchKernelGGL(upd_validate_kernel, dim3((p->U + 3) / 4), dim3(256), 0, stream, *p);
  hipLaunchKernelGGL(upd_apply_kernel, dim3(p->U), dim3(256), 0, stream, *p);
  hipLaunchKernelGGL(upd_reset_kernel, dim3((p->U + 255) / 256), dim3(256), 0, stream, *p);
  return (int)hipGetLastError();
}
