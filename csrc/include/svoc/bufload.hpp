// Raw buffer loads over one instance's [N, ld] bf16 table (shared by the register-streaming kernels).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svoc/sortnet.hpp"

namespace svoc {

// Buffer resource over one instance: row offsets ride in SGPRs (soffset), the lane's column-pair
// offset in one VGPR (voffset); rows past N fall outside num_records and read as 0 (no clamping).
SVOC_DEV __amdgpu_buffer_rsrc_t instance_rsrc(const void* base, uint32_t bytes) {
  const uint64_t pa = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)pa);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(pa >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// The same descriptor as four SGPR words, for inline asm (buffer_load ... lds): words 0-1 base, 2
// num_records, 3 the flags make_buffer_rsrc sets.
typedef int v4i_t __attribute__((ext_vector_type(4)));
struct BufDesc {
  v4i_t w;
};
SVOC_DEV BufDesc buf_desc(const void* base, uint32_t bytes) {
  const uint64_t pa = (uint64_t)base;
  return BufDesc{v4i_t{(int)__builtin_amdgcn_readfirstlane((uint32_t)pa),
                       (int)(__builtin_amdgcn_readfirstlane((uint32_t)(pa >> 32)) & 0xffffu),
                       (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000}};
}

SVOC_DEV uint32_t bload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}
// with a cache-policy operand (gfx950: 1 = sc0, 2 = nt, 16 = sc1)
template <int AUX>
SVOC_DEV uint32_t bload_p(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, AUX);
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
SVOC_DEV void bstore(__amdgpu_buffer_rsrc_t r, uint32_t v, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, soff, 0);
}
SVOC_DEV void bstore2(__amdgpu_buffer_rsrc_t r, f32x2 v, int voff, int soff) {
  const float a = v.x, b = v.y;  // element copies first (see fand2 in sortnet.hpp: clang bit_cast of v.y)
  const u32x2 u = {__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b)};
  __builtin_amdgcn_raw_buffer_store_b64(u, r, voff, soff, 0);
}
SVOC_DEV float bloadf(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// Staged pass-2 outputs (launch.hpp, fast_work_words): [3][D2] floats (consensus, skewness,
// kurtosis) at byte offset `stg` of the instance's workspace.
SVOC_DEV void stage_out(__amdgpu_buffer_rsrc_t ws, int stg, int D2, int which, int col, float v) {
  bstore(ws, __builtin_bit_cast(uint32_t, v), col * 4, stg + which * D2 * 4);
}
// Copy of the staged outputs of one instance to consensus / skew / kurt (the round's status is OK),
// by all NT threads of the workgroup after a barrier.  sc0 loads: the words were stored by other
// waves of this workgroup (workgroup-scope coherence, as in the LLVM AMDGPU memory model).
template <int NT>
SVOC_DEV void commit_staged(__amdgpu_buffer_rsrc_t ws, int stg, int D2, int D, int tid, float* cons, float* skew,
                            float* kurt) {
  for (int c = tid; c < D; c += NT) {
    const uint32_t a = __builtin_amdgcn_raw_buffer_load_b32(ws, c * 4, stg, 1);
    const uint32_t s = __builtin_amdgcn_raw_buffer_load_b32(ws, c * 4, stg + D2 * 4, 1);
    const uint32_t k = __builtin_amdgcn_raw_buffer_load_b32(ws, c * 4, stg + 2 * D2 * 4, 1);
    cons[c] = __builtin_bit_cast(float, a);
    skew[c] = __builtin_bit_cast(float, s);
    kurt[c] = __builtin_bit_cast(float, k);
  }
}

// Sort keys of two bf16 columns: constrained values ([0, 1]) by one XOR, general bf16 otherwise.
template <bool CONS>
SVOC_DEV u16x2 to_key(uint32_t raw) {
  if constexpr (CONS) return pos_to_key(raw);
  else return bf16x2_to_key(raw);
}
template <bool CONS>
SVOC_DEV uint32_t from_key(u16x2 k) {
  if constexpr (CONS) return key_to_pos(k);
  else return key_to_bf16x2(k);
}

}  // namespace svoc
