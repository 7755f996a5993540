// Batched update_prediction storage step (contract.cairo:331-343, :588-603): validate each update
// (constrained inputs must lie in [0, 1] / [0, WSAD]: 'interval error', math.cairo:298-310),
// pick the last valid writer per (instance, oracle) with an atomicMax on the update sequence
// number (coalescing is exact: survey §2.8-13), copy the winning rows with 16-B vector stores,
// flip `enabled` and bump n_active_oracles on first commit.  Three launches, no host sync; each
// update gets L lanes sized to its row, so tiny rows pack 64 updates per wave.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svoc/launch.hpp"
#include "svoc/status.hpp"

namespace svoc {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bool in_range(const UpdateParams& p, int64_t u, int d) {
  if (p.dtype == 0) {
    const uint16_t raw = ((const uint16_t*)p.upd)[u * p.D + d];
    const float f = __builtin_bit_cast(float, (uint32_t)raw << 16);
    return f >= 0.f && f <= 1.f;
  } else if (p.dtype == 1) {
    const float f = ((const float*)p.upd)[u * p.D + d];
    return f >= 0.f && f <= 1.f;
  }
  const int64_t v = p.dtype == 3 ? (int64_t)((const int32_t*)p.upd)[u * p.D + d] : ((const int64_t*)p.upd)[u * p.D + d];
  return v >= 0 && v <= 1000000;
}

__device__ __forceinline__ bool bf16_unit(uint32_t raw16) {  // 0 <= x <= 1 (and -0.0)
  return raw16 <= 0x3f80u || raw16 == 0x8000u;
}

// unconstrained float values must be finite (the wsad domain has no NaN / inf)
__device__ __forceinline__ bool finite_at(const UpdateParams& p, int64_t u, int d) {
  if (p.dtype == 0) return (((const uint16_t*)p.upd)[u * p.D + d] & 0x7f80u) != 0x7f80u;
  if (p.dtype == 1) return (__builtin_bit_cast(uint32_t, ((const float*)p.upd)[u * p.D + d]) & 0x7f800000u) != 0x7f800000u;
  return true;
}

// L lanes per update (L = power of two covering the row in 16-B chunks, capped at 64): a wave
// serves 64/L updates, so the deployed 7 x 6 config (12-B rows) runs 64 updates per wave instead of
// one, and wide rows (c3: 8 KiB) get a whole wave each.  True iff all L lanes of the group agree.
template <int L>
__device__ __forceinline__ bool group_all(bool ok) {
  const uint64_t bad = __ballot(!ok);
  const int lane = threadIdx.x & 63;
  const uint64_t gm = (L == 64) ? ~0ull : (((1ull << (L & 63)) - 1ull) << (lane & ~(L - 1)));
  return (bad & gm) == 0;
}

// The transaction's status in the contract's check order (contract.cairo:588-596): the prediction's
// interval check (finite values, unconstrained floats) before the caller's oracle lookup -- an update
// failing both reports INTERVAL_INPUT, as the reference does.
__device__ __forceinline__ int row_status(bool ok, bool fin, bool bad) {
  return !ok ? ST_INTERVAL_INPUT : !fin ? ST_NON_FINITE : bad ? ST_NOT_ORACLE : ST_OK;
}

// validate every update, then claim its (instance, oracle) slot with an atomicMax on the update's
// sequence number: the last valid writer wins (coalescing is exact: survey §2.8-13)
template <int L>
__global__ __launch_bounds__(256) void upd_validate_kernel(UpdateParams p) {
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) / L;
  const int sub = threadIdx.x & (L - 1);
  const bool in = u < p.U;
  bool bad = false;   // unknown instance / oracle: reported after the row checks (see row_status)
  int64_t b = 0, o = 0;
  if (in) {
    b = p.inst[u];
    o = p.oracle[u];
    bad = b < 0 || b >= p.B || o < 0 || o >= p.N;
  }
  bool ok = true;
  if (in && p.constrained) {
    const uint16_t* row = (const uint16_t*)p.upd + u * p.D;
    if (p.dtype == 0 && (p.D & 7) == 0 && (((uintptr_t)row) & 15) == 0) {
      for (int c = sub; c < p.D / 8; c += L) {
        const uint4 v = ((const uint4*)row)[c];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) ok = ok && bf16_unit(w[k] & 0xffffu) && bf16_unit(w[k] >> 16);
      }
    } else {
      for (int d = sub; d < p.D; d += L) ok = ok && in_range(p, u, d);
    }
  }
  bool fin = true;
  if (in && !p.constrained && p.dtype <= 1)
    for (int d = sub; d < p.D; d += L) fin = fin && finite_at(p, u, d);
  ok = group_all<L>(ok);  // all lanes reach the ballots (no early return above)
  fin = group_all<L>(fin);
  if (in && sub == 0) {
    const int st = row_status(ok, fin, bad);
    p.upd_status[u] = st;
    if (p.saved_en) p.saved_en[u] = kNotSaved;   // the winner's apply overwrites it
    if (st == ST_OK) atomicMax(&p.winner[b * p.N + o], (int)u);
  }
}

// Row copy src -> dst by the L lanes of an update (16-B vectors when aligned); with `sv` (transactional
// streaming) every chunk of dst is first copied to sv -- loaded before the chunk is overwritten by the
// same lane, so the saved row is the pre-update one.
template <int L>
__device__ __forceinline__ void copy_row(unsigned char* dst, const unsigned char* src, unsigned char* sv,
                                         int64_t row_bytes, int sub) {
  if (((uintptr_t)dst & 15) == 0 && ((uintptr_t)src & 15) == 0 && (!sv || ((uintptr_t)sv & 15) == 0) &&
      (row_bytes & 15) == 0) {
    for (int64_t i = sub; i < row_bytes / 16; i += L) {
      if (sv) ((uint4*)sv)[i] = ((const uint4*)dst)[i];
      ((uint4*)dst)[i] = ((const uint4*)src)[i];
    }
  } else if (((uintptr_t)dst & 3) == 0 && ((uintptr_t)src & 3) == 0 && (!sv || ((uintptr_t)sv & 3) == 0) &&
             (row_bytes & 3) == 0) {
    for (int64_t i = sub; i < row_bytes / 4; i += L) {
      if (sv) ((uint32_t*)sv)[i] = ((const uint32_t*)dst)[i];
      ((uint32_t*)dst)[i] = ((const uint32_t*)src)[i];
    }
  } else {
    for (int64_t i = sub; i < row_bytes; i += L) {
      if (sv) sv[i] = dst[i];
      dst[i] = src[i];
    }
  }
}

// first commit of an (instance, oracle) slot: enabled + n_active (contract.cairo:331-343); the old flag
// goes to saved_en (transactional streaming)
__device__ __forceinline__ void commit_flags(const UpdateParams& p, int64_t u, int64_t b, int64_t o) {
  const uint8_t was = p.enabled[b * p.N + o];
  if (p.saved_en) p.saved_en[u] = was;
  if (!was) {
    p.enabled[b * p.N + o] = 1;
    atomicAdd(&p.n_active[b], 1);
  }
  p.touched[b] = 1;
}

// the winner of each slot copies its row (16-B vectors when aligned), flips `enabled`, bumps
// n_active_oracles on an oracle's first commit (contract.cairo:331-343) and marks the instance
template <int L>
__global__ __launch_bounds__(256) void upd_apply_kernel(UpdateParams p) {
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) / L;
  const int sub = threadIdx.x & (L - 1);
  if (u >= p.U || p.upd_status[u] != ST_OK) return;
  const int64_t b = p.inst[u], o = p.oracle[u];
  if (p.winner[b * p.N + o] != (int)u) return;  // superseded by a later update: coalesced
  const int64_t row_bytes = (int64_t)p.D * p.elem_bytes;
  unsigned char* dst = (unsigned char*)p.values + (b * p.inst_stride + o * p.ld) * p.elem_bytes;
  const unsigned char* src = (const unsigned char*)p.upd + u * row_bytes;
  unsigned char* sv = p.saved ? (unsigned char*)p.saved + u * row_bytes : nullptr;
  copy_row<L>(dst, src, sv, row_bytes, sub);
  if (sub == 0) commit_flags(p, u, b, o);
}

// unique (instance, oracle) pairs (e.g. a synthetic stream, one bootstrap batch per window): no
// last-writer resolution needed, so validation and the row copy run in one pass over the updates
// (one read of the update rows instead of two)
// SAVE (transactional streaming, p.saved set): the rows being overwritten are loaded with the new ones and
// saved; a separate instantiation, so the plain form keeps its register footprint (the save path's
// conditional loads took the L = 64, RB = 8 kernel from 57 to 276 VGPRs when they shared one body)
template <int L, int RB, bool SAVE>
__global__ __launch_bounds__(256) void upd_fused_unique_kernel(UpdateParams p) {
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) / L;
  const int sub = threadIdx.x & (L - 1);
  const bool in = u < p.U;
  bool bad = false;   // unknown instance / oracle: reported after the row checks (row_status)
  int64_t b = 0, o = 0;
  if (in) {
    b = p.inst[u];
    o = p.oracle[u];
    bad = b < 0 || b >= p.B || o < 0 || o >= p.N;
  }
  const int64_t row_bytes = (int64_t)p.D * p.elem_bytes;
  const unsigned char* src = (const unsigned char*)p.upd + u * row_bytes;
  unsigned char* dst = (unsigned char*)p.values + (b * p.inst_stride + o * p.ld) * p.elem_bytes;
  const bool vec = (row_bytes & 15) == 0 && (((uintptr_t)src) & 15) == 0 && (((uintptr_t)dst) & 15) == 0;
  // bf16 / fp32 rows of <= RB*L 16-B chunks (c3: 8 KiB bf16 rows, 8 chunks per lane; 16 KiB fp32
  // rows, RB = 16): every chunk is loaded once into registers (all loads in flight together,
  // non-temporal: the update batch is read once), validated there and stored from there, so the row
  // is never re-read
  const int64_t nch = row_bytes / 16;
  if (p.dtype <= 1 && vec && nch <= (int64_t)RB * L) {  // uniform over the launch
    uint4 v[RB];
    u32x4 old[SAVE ? RB : 1];   // transactional: the row being overwritten, loaded in the same batch
    bool ok = true, fin = true;
    const bool live = in;
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const int64_t i = sub + (int64_t)k * L;
      u32x4 t = {0u, 0u, 0u, 0u};
      if (live && i < nch) t = __builtin_nontemporal_load((const u32x4*)src + i);
      v[k] = uint4{t.x, t.y, t.z, t.w};
    }
    if constexpr (SAVE) {
      // (bad indices: the row address is not dereferenced -- a clamped in-bounds slot is read instead)
      const unsigned char* ds = bad ? (const unsigned char*)p.values : dst;
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const int64_t i = sub + (int64_t)k * L;
        old[k] = (live && i < nch) ? ((const u32x4*)ds)[i] : u32x4{0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (p.dtype == 1) {   // fp32: 0 <= x <= 1 (and -0.0) / finite
          if (p.constrained) ok = ok && (w[j] <= 0x3f800000u || w[j] == 0x80000000u);
          else fin = fin && ((w[j] & 0x7f800000u) != 0x7f800000u);
        } else {
          if (p.constrained) ok = ok && bf16_unit(w[j] & 0xffffu) && bf16_unit(w[j] >> 16);
          else fin = fin && ((w[j] & 0x7f80u) != 0x7f80u) && ((w[j] & 0x7f800000u) != 0x7f800000u);
        }
      }
    }
    ok = group_all<L>(ok);
    fin = group_all<L>(fin);
    if (!in) return;
    const int st = row_status(ok, fin, bad);
    if (sub == 0) {
      p.upd_status[u] = st;
      if (st != ST_OK && p.saved_en) p.saved_en[u] = kNotSaved;
    }
    if (st != ST_OK) return;
    if constexpr (SAVE) {   // the old row, saved beside the update
      u32x4* sv = (u32x4*)((unsigned char*)p.saved + u * row_bytes);
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const int64_t i = sub + (int64_t)k * L;
        if (i < nch) __builtin_nontemporal_store(old[k], sv + i);   // read back only on a revert
      }
    }
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const int64_t i = sub + (int64_t)k * L;
      if (i < nch) ((uint4*)dst)[i] = v[k];
    }
  } else if (L == 1 && p.dtype == 0 && (row_bytes & 3) == 0 && row_bytes <= 16 && (((uintptr_t)p.upd) & 3) == 0 &&
             (((uintptr_t)p.values) & 3) == 0 && (p.inst_stride & 1) == 0 && (p.ld & 1) == 0) {
    // short bf16 rows (the deployed 7 x 6: 12 B): the row's words are loaded with the instance / oracle
    // indices (their addresses do not depend on them), validated and stored from registers -- one
    // memory round trip before the stores instead of three (profiles/r2_pmc_c5.md)
    const int nw = (int)(row_bytes >> 2);
    uint32_t w[4], old[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (in && k < nw) ? ((const uint32_t*)src)[k] : 0u;
    // the slot's old words and enabled flag, loaded together (one round trip after the indices; the
    // stores below could alias them, so loaded any later they would wait for those stores)
    const bool slot = in && !bad;
#pragma unroll
    for (int k = 0; k < 4; ++k) old[k] = (slot && p.saved && k < nw) ? ((const uint32_t*)dst)[k] : 0u;
    const uint8_t was = slot ? p.enabled[b * p.N + o] : (uint8_t)1;
    bool ok = true, fin = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= nw) continue;
      if (p.constrained) ok = ok && bf16_unit(w[k] & 0xffffu) && bf16_unit(w[k] >> 16);
      else fin = fin && ((w[k] & 0x7f80u) != 0x7f80u) && ((w[k] & 0x7f800000u) != 0x7f800000u);
    }
    if (!in) return;
    const int st = row_status(ok, fin, bad);
    p.upd_status[u] = st;
    if (st != ST_OK) {
      if (p.saved_en) p.saved_en[u] = kNotSaved;
      return;
    }
    if (p.saved) {
      uint32_t* sv = (uint32_t*)((unsigned char*)p.saved + u * row_bytes);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < nw) __builtin_nontemporal_store(old[k], sv + k);   // read back only on a revert
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < nw) ((uint32_t*)dst)[k] = w[k];
    if (p.saved_en) p.saved_en[u] = was;
    if (!was) {
      p.enabled[b * p.N + o] = 1;
      atomicAdd(&p.n_active[b], 1);
    }
    p.touched[b] = 1;
    return;
  } else {
    bool ok = true, fin = true;
    if (in) {
      if (p.dtype == 0 && vec) {
        for (int64_t i = sub; i < nch; i += L) {
          const uint4 v = ((const uint4*)src)[i];
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (p.constrained) ok = ok && bf16_unit(w[k] & 0xffffu) && bf16_unit(w[k] >> 16);
            else fin = fin && ((w[k] & 0x7f80u) != 0x7f80u) && ((w[k] & 0x7f800000u) != 0x7f800000u);
          }
        }
      } else {
        for (int d = sub; d < p.D; d += L) {
          if (p.constrained) ok = ok && in_range(p, u, d);
          else if (p.dtype <= 1) fin = fin && finite_at(p, u, d);
        }
      }
    }
    ok = group_all<L>(ok);   // every lane reaches the ballots
    fin = group_all<L>(fin);
    if (!in) return;
    const int st = row_status(ok, fin, bad);
    if (sub == 0) {
      p.upd_status[u] = st;
      if (st != ST_OK && p.saved_en) p.saved_en[u] = kNotSaved;
    }
    if (st != ST_OK) return;
    // the row was just read by these lanes: the copy re-reads it from L2
    copy_row<L>(dst, src, p.saved ? (unsigned char*)p.saved + u * row_bytes : nullptr, row_bytes, sub);
  }
  if (sub == 0) commit_flags(p, u, b, o);
}

// Roll back the reverted instances' updates (RestoreParams).  One thread per update, grid-stride over a
// small grid: the check is a few loads per update and reverts are rare, so the kernel must not need many
// workgroup slots -- it runs right after its range's round, beside the other range's round kernel, which
// holds every slot it can get (a one-wave-per-update form took ~85 us there, on the step's critical path).
// A reverted update's row is copied back by its own thread (16-B vectors when aligned).
__global__ __launch_bounds__(256) void upd_restore_kernel(RestoreParams p) {
  const int64_t row_bytes = (int64_t)p.D * p.elem_bytes;
  for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < p.U; u += (int64_t)gridDim.x * 256) {
    if (p.upd_status[u] != ST_OK) continue;
    const int64_t b = p.inst[u], o = p.oracle[u];
    if (b < 0 || b >= p.B || o < 0 || o >= p.N) continue;
    const int rst = p.status[b];
    if (!p.active[b]) {
      if (p.inactive_status >= 0) p.upd_status[u] = p.inactive_status;
      continue;
    }
    if (rst == ST_OK) continue;
    const uint8_t was = p.saved_en[u];
    if (was != kNotSaved) {
      unsigned char* dst = (unsigned char*)p.values + (b * p.inst_stride + o * p.ld) * p.elem_bytes;
      const unsigned char* sv = (const unsigned char*)p.saved + u * row_bytes;
      if (((uintptr_t)dst & 15) == 0 && ((uintptr_t)sv & 15) == 0 && (row_bytes & 15) == 0) {
        for (int64_t i = 0; i < row_bytes / 16; ++i) ((uint4*)dst)[i] = ((const uint4*)sv)[i];
      } else {
        for (int64_t i = 0; i < row_bytes; ++i) dst[i] = sv[i];
      }
      if (was == 0) {
        p.enabled[b * p.N + o] = 0;
        atomicSub(&p.n_active[b], 1);
      }
    }
    p.upd_status[u] = rst;   // the transaction reverted with the round's code
  }
}

__global__ __launch_bounds__(256) void upd_reset_kernel(UpdateParams p) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= p.U || p.upd_status[u] != ST_OK) return;
  p.winner[p.inst[u] * p.N + p.oracle[u]] = -1;
}

template <int L>
static int launch_updates(const UpdateParams& p, hipStream_t stream) {
  const int64_t blocks = ((int64_t)p.U * L + 255) / 256;
  if (p.unique) {
    // registers for the whole row: 8 16-B chunks per lane, 16 for rows past 8 * L chunks (fp32 c3)
    const int64_t nch = (int64_t)p.D * p.elem_bytes / 16;
    const bool big = L == 64 && nch > 8 * L;
    if (p.saved) {
      if (big) hipLaunchKernelGGL((upd_fused_unique_kernel<L, 16, true>), dim3((unsigned)blocks), dim3(256), 0, stream, p);
      else hipLaunchKernelGGL((upd_fused_unique_kernel<L, 8, true>), dim3((unsigned)blocks), dim3(256), 0, stream, p);
    } else {
      if (big) hipLaunchKernelGGL((upd_fused_unique_kernel<L, 16, false>), dim3((unsigned)blocks), dim3(256), 0, stream, p);
      else hipLaunchKernelGGL((upd_fused_unique_kernel<L, 8, false>), dim3((unsigned)blocks), dim3(256), 0, stream, p);
    }
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(upd_validate_kernel<L>, dim3((unsigned)blocks), dim3(256), 0, stream, p);
  hipLaunchKernelGGL(upd_apply_kernel<L>, dim3((unsigned)blocks), dim3(256), 0, stream, p);
  hipLaunchKernelGGL(upd_reset_kernel, dim3((unsigned)((p.U + 255) / 256)), dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}

static int launch_restore(const RestoreParams& p, hipStream_t stream) {
  // at least 64 workgroups (the pipelined c3 ranges: 32 k updates, 2 per thread), 2 updates per thread
  // past that (a flat 64-workgroup grid left the c5 stream's 1M updates per step at 64 dependent
  // iterations per thread: +0.14 ms per step)
  const int64_t need = ((int64_t)p.U + 255) / 256;
  int64_t blocks = (need + 1) / 2;
  if (blocks < 64) blocks = need < 64 ? need : 64;
  hipLaunchKernelGGL(upd_restore_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}


// Commit of a fused transactional step: the round kernel read the updated rows from the batch and wrote
// every update's transaction status; the accepted rows (status OK) are copied into the state here, one
// update per L lanes, the row's 16-B chunks loaded together (non-temporal: read once) and stored.
template <int L, int RB>
__global__ __launch_bounds__(256) void upd_commit_kernel(const unsigned char* __restrict__ rows,
                                                         const int64_t* __restrict__ oracle,
                                                         const int32_t* __restrict__ upd_status,
                                                         unsigned char* __restrict__ values, int64_t inst_stride,
                                                         int N, int D, int ld, int U, int64_t n_upd, int elem_bytes) {
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) / L;
  const int sub = threadIdx.x & (L - 1);
  if (u >= n_upd || upd_status[u] != ST_OK) return;
  const int64_t o = oracle[u];
  if (o < 0 || o >= N) return;
  const int64_t b = u / U;
  const int64_t row_bytes = (int64_t)D * elem_bytes;
  const unsigned char* src = rows + u * row_bytes;
  unsigned char* dst = values + (b * inst_stride + o * ld) * elem_bytes;
  const int64_t nch = row_bytes / 16;
  if ((row_bytes & 15) == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0 && nch <= (int64_t)RB * L) {
    u32x4 v[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const int64_t i = sub + (int64_t)k * L;
      v[k] = i < nch ? __builtin_nontemporal_load((const u32x4*)src + i) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const int64_t i = sub + (int64_t)k * L;
      if (i < nch) ((u32x4*)dst)[i] = v[k];
    }
  } else {
    for (int64_t i = sub; i < row_bytes; i += L) dst[i] = src[i];
  }
}

template <int L>
static int launch_commit(const void* rows, const int64_t* oracle, const int32_t* st, void* values, int64_t inst_stride,
                         int N, int D, int ld, int U, int64_t n_upd, int eb, hipStream_t stream) {
  const int64_t blocks = (n_upd * L + 255) / 256;
  const int64_t nch = (int64_t)D * eb / 16;
  if (nch > 8 * L)
    hipLaunchKernelGGL((upd_commit_kernel<L, 16>), dim3((unsigned)blocks), dim3(256), 0, stream,
                       (const unsigned char*)rows, oracle, st, (unsigned char*)values, inst_stride, N, D, ld, U, n_upd, eb);
  else
    hipLaunchKernelGGL((upd_commit_kernel<L, 8>), dim3((unsigned)blocks), dim3(256), 0, stream,
                       (const unsigned char*)rows, oracle, st, (unsigned char*)values, inst_stride, N, D, ld, U, n_upd, eb);
  return (int)hipGetLastError();
}

}  // namespace svoc

using namespace svoc;

extern "C" int svoc_apply_updates(const UpdateParams* p, hipStream_t stream) {
  if (p->U <= 0) return 0;
  if ((int64_t)p->U * 64 / 256 >= 0x7fffffffll) return -1;
  const int64_t chunks = ((int64_t)p->D * p->elem_bytes + 15) / 16;  // 16-B pieces per row
  if (chunks <= 1) return launch_updates<1>(*p, stream);
  if (chunks <= 2) return launch_updates<2>(*p, stream);
  if (chunks <= 4) return launch_updates<4>(*p, stream);
  if (chunks <= 8) return launch_updates<8>(*p, stream);
  if (chunks <= 16) return launch_updates<16>(*p, stream);
  if (chunks <= 32) return launch_updates<32>(*p, stream);
  return launch_updates<64>(*p, stream);
}

extern "C" int svoc_restore_updates(const RestoreParams* p, hipStream_t stream) {
  if (p->U <= 0) return 0;
  return launch_restore(*p, stream);
}

extern "C" int svoc_commit_updates(const void* rows, const int64_t* oracle, const int32_t* upd_status, void* values,
                                   int64_t inst_stride, int N, int D, int ld, int U, int64_t n_upd, int elem_bytes,
                                   hipStream_t stream) {
  if (n_upd <= 0) return 0;
  if (U <= 0 || n_upd * 64 / 256 >= 0x7fffffffll) return -1;
  const int64_t chunks = ((int64_t)D * elem_bytes + 15) / 16;
  if (chunks <= 4) return launch_commit<4>(rows, oracle, upd_status, values, inst_stride, N, D, ld, U, n_upd, elem_bytes, stream);
  if (chunks <= 16) return launch_commit<16>(rows, oracle, upd_status, values, inst_stride, N, D, ld, U, n_upd, elem_bytes, stream);
  return launch_commit<64>(rows, oracle, upd_status, values, inst_stride, N, D, ld, U, n_upd, elem_bytes, stream);
}
