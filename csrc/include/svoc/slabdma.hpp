// Phase-A streaming of an instance table through LDS by LDS-DMA, shared by the one-network window
// kernels (consensus_fast_winf.hip: fp32, one column per lane; consensus_fast_win.hip: bf16, one column
// pair per 32-bit word).  A lane group of NSEG lanes owns a column (pair), 64 rows per lane.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svoc/bufload.hpp"

namespace svoc {

// The lane's 64 raw rows as two 32-wide vectors (one SSA value each): a plain array is split by SROA into
// a promoted part and a scratch part when several code paths read it.
typedef uint32_t u32x32_t __attribute__((ext_vector_type(32)));
struct RawRows {
  u32x32_t lo, hi;   // rows 0..31, 32..63
  SVOC_DEV uint32_t at(int i) const { return i < 32 ? lo[i] : hi[i - 32]; }
};

// Phase-A streaming by LDS-DMA (buffer_load_dwordx4 ... lds: no VGPR destination).  Every wave owns a
// 16-KiB LDS region holding its next slab -- its P columns x the NPAD rows -- so a wave waits for its
// own pieces only (no workgroup barrier in phase A).  Region layout: LDS row q = NSEG * (r % 64) + r / 64
// of global row r, P words per row: the NSEG rows a reader instruction touches (r, r + 64, ...; one per
// lane-group segment) are adjacent, i.e. on 64 distinct banks.  One DMA instruction (piece) writes 1 KiB
// lane-linearly = RPI consecutive LDS rows; 16 pieces fill the region.
template <int NSEG>
struct SlabDma {
  static constexpr int P = 64 / NSEG, CPR = P / 4, RPI = 64 / CPR;
  int vlane;   // this lane's part of every piece's voffset
  int row0;    // global row this lane loads in piece 0 (piece k: row0 + k * RPI / NSEG)
  int colb;    // this lane's byte offset within the row piece
  SVOC_DEV SlabDma(int lane, int rowb) {
    const int j = lane / CPR;   // LDS row of the piece this lane fills
    row0 = (j % NSEG) * 64 + j / NSEG;
    colb = (lane % CPR) * 16;
    vlane = row0 * rowb + colb;
  }
  SVOC_DEV int row_of(int k) const { return row0 + k * (RPI / NSEG); }
  // the region's LDS byte address (cast once per slab: per piece, the generic -> LDS cast's null test and a
  // 64-bit add cost four SALU)
  static SVOC_DEV uint32_t lds_addr(uint32_t* region) {
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)region;
  }
  // issue this wave's 16 pieces of the slab whose first word (of this wave: an fp32 column, a bf16 column
  // pair) is col0.  Inline asm: the
  // __builtin_amdgcn_raw_ptr_buffer_load_lds form crashes ROCm 7.2's instruction selection in this
  // kernel; M0 is saved and restored around the piece (the compiler reserves it).
  SVOC_DEV void issue(const BufDesc& rs, uint32_t* region, int rowb, int col0) const {
    const int vo = vlane + col0 * 4;
    const uint32_t lds0 = lds_addr(region);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t lds = lds0 + k * 1024u;
      int keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\t"
          "s_mov_b32 m0, %3\n\t"
          "s_nop 0\n\t"
          "buffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
          "s_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(vo), "s"(rs.w), "s"(lds), "s"(k * (RPI / NSEG) * rowb)
          : "memory");
    }
  }
  // The same slab, with per-piece row sources (fused transactional streaming): piece k is issued twice
  // under complementary exec masks -- the lanes whose row comes from the update batch (sel(k) != 0) read
  // byte offset off_b(k) of rb, the others the state rows exactly as issue() does (one voffset for the
  // slab, the piece's row step in soffset: no per-piece VALU).  The masks are switched inside the asm (exec
  // restored before it ends), so the compiler sees no divergent control flow around the loads (which cost
  // the kernel ~27 spilled VGPRs when written as if / else).
  template <class Sel, class OffB>
  SVOC_DEV void issue_mapped(const BufDesc& rs, const BufDesc& rb, uint32_t* region, int rowb, int col0, Sel sel,
                             OffB off_b) const {
    const int vo = vlane + col0 * 4;
    const uint32_t lds0 = lds_addr(region);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t lds = lds0 + k * 1024u;
      const uint32_t fb = sel(k);
      const int vb = off_b(k, fb);
      int keep;
      uint64_t sx;
      // (the exec masks come from a compare inside the asm: ballots outside it were scheduled early and
      // held as 16 SGPR pairs -- hundreds of spilled SGPRs; s_nop 4: VALU-written VCC read by SALU)
      asm volatile(
          "s_mov_b32 %0, m0\n\t"
          "s_mov_b32 m0, %7\n\t"
          "s_mov_b64 %1, exec\n\t"
          "v_cmp_ne_u32 vcc, 0, %4\n\t"
          "s_nop 4\n\t"
          "s_andn2_b64 exec, %1, vcc\n\t"
          "s_nop 0\n\t"
          "buffer_load_dwordx4 %2, %5, %8 offen lds\n\t"
          "s_and_b64 exec, %1, vcc\n\t"
          "s_nop 0\n\t"
          "buffer_load_dwordx4 %3, %6, 0 offen lds\n\t"
          "s_mov_b64 exec, %1\n\t"
          "s_mov_b32 m0, %0"
          : "=&s"(keep), "=&s"(sx)
          : "v"(vo), "v"(vb), "v"(fb), "s"(rs.w), "s"(rb.w), "s"(lds), "s"(k * (RPI / NSEG) * rowb)
          : "vcc", "memory");
    }
  }
};

}  // namespace svoc
