// Fused two-pass robust consensus, fast mode, "window" variant: ONE sorting network and ONE read of
// the instance per round.
//
// Semantics: contract/src/contract.cairo:442-503 (constrained) / :370-434 (unconstrained), as in
// consensus_fast_reg.hip.  The pass-2 smooth median (over the R = N - f reliable rows, ranks
// R/2 - 1 and R/2, math.cairo:113-126) is an order statistic of the FULL column shifted by at most
// f ranks: with a = N/2 - R/2 it lies at sorted position R/2 - 1 + j of the full column for the
// smallest j with  #{removed keys <= w_j} <= j  (w = the full column's sorted keys from position
// R/2 - 1 on).  So:
//   pass 1 (phase A): the register-streaming median network of consensus_fast_reg.hip, extended to
//     keep H keys on either side of the median (window_group, sortnet.hpp), written to a workspace;
//     the qr loop (the reg kernel's) also accumulates the all-row power sums of d = x - c1;
//   rank mask: unchanged (sort by (qr asc, idx desc), the first R are reliable);
//   pass 2 (phase B, one lane per column pair): only the f removed rows are read.  Their keys
//     (f + 2 <= 2H slots with -inf / +inf sentinels around them) are sorted by a small network and
//     compared slot by slot with the window:
//       med_lo = min{ w_j : w_j < u'_j },  med_hi = min{ w_j : w_j < u'_(j-1) }
//     (u' = the sorted removed keys shifted by the sentinel count, so slot j pairs with window
//     position j).  The reliable rows' power sums are the all-row sums minus the removed rows'.
//     When that difference would cancel (all-row second / fourth sums more than win_cancel x the
//     reliable ones: far outliers around a tight cluster, or zero variance) the column goes on the
//     instance's list, and the workgroup recomputes those columns exactly over the reliable rows
//     (one wave per column) before it finishes.
// Versus the reg kernel: no second 64*NSEG-key network, no second read of the instance (HBM: the
// pass-1 read + the window round trip + the removed rows).  Valid for f <= 32 with a + 1 <= H and
// f - a + 1 <= H (H = 5 or 17); the dispatcher falls back to consensus_fast_reg.hip otherwise.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "svoc/bufload.hpp"
#include "svoc/launch.hpp"
#include "svoc/rankmask.hpp"
#include "svoc/sortnet.hpp"
#include "svoc/status.hpp"

namespace svoc {

// The reliable sums are trusted when sum_all(d^2) <= C * sum_R(d^2) and likewise for d^4, C =
// p.win_cancel (default 64, SVOC_WIN_CANCEL): the fp32 error of the difference is then <= C x the
// all-row sums' own relative error (~1e-6 worst case, ~1e-7 typical).

SVOC_DEV u16x2 win_cand(u16x2 wt, u16x2 zt) {  // wt < zt ? wt : 0xFFFF, per 16-bit half
  // four packed instructions (written with the elementwise builtins, LLVM split the halves into compares and
  // selects: ~7 VALU per candidate, 20 candidates per column pair in pass 2)
  const uint32_t one = 0x00010001u;
  uint32_t d;
  asm("v_pk_sub_u16 %0, %1, %2 clamp\n\t"
      "v_pk_min_u16 %0, %0, %3\n\t"
      "v_pk_sub_u16 %0, %0, %3"
      : "=&v"(d)
      : "v"(as_u32(zt)), "v"(as_u32(wt)), "v"(one));
  return as_k(as_u32(wt) | d);   // d: 0 where wt < zt, 0xFFFF otherwise
}

// Skewness / sample-adjusted excess kurtosis (math.cairo:320-363) of n values from power sums of
// d = x - shift; returns false for zero variance (the contract's sqrt(0) -> div-by-zero revert).  The
// n-only factors are formed once per instance (MomK); per column one IEEE division (1 / mu2) and one
// v_rsq_f32 remain of the ~10 divisions (each a div_scale / rcp / fma / div_fmas / div_fixup sequence) the
// direct formulas cost -- a third of the c2 pass-2 loop.  (Within a few ulp of the direct form.)
struct MomK {
  float n, in, k3, k4a, k4b, ik4c;
};
SVOC_DEV MomK mom_k(float n) {
  return MomK{n, 1.f / n, n / ((n - 1.f) * (n - 2.f)), n * (n + 1.f) / (n - 1.f), 3.f * (n - 1.f) * (n - 1.f),
              1.f / ((n - 2.f) * (n - 3.f))};
}
SVOC_DEV bool moments_from_sums(const MomK& K, float t1, float t2, float t3, float t4, float& dl, float& sk, float& ku) {
#pragma clang fp contract(off)
  dl = t1 * K.in;
  const float e2 = t2 * K.in, e3 = t3 * K.in, e4 = t4 * K.in;
  const float mu2 = e2 - dl * dl;
  const float mu3 = e3 - 3.f * dl * e2 + 2.f * dl * dl * dl;
  const float mu4 = e4 - 4.f * dl * e3 + 6.f * dl * dl * e2 - 3.f * dl * dl * dl * dl;
  sk = 0.f;
  ku = 0.f;
  if (!(mu2 > 0.f)) return false;
  const float r = 1.f / mu2;
  sk = K.n * mu3 * r * __builtin_amdgcn_rsqf(mu2) * K.k3;
  ku = (K.n * mu4 * (r * r) * K.k4a - K.k4b) * K.ik4c;
  return true;
}

// qr partials of the lane's 64 rows reduced across the wave's column pairs (the reg kernel's
// transposing butterfly: stage L exchanges with lane ^ (P >> L) and halves the row set), evaluated
// depth-first so only O(log) partials are live instead of 64; the leaves also accumulate the rows'
// power sums of d = x - c1.  MASKW: slab with columns past D (their halves masked to +0, centre +0);
// MASKROWS: rows >= N (read as 0 past the buffer end) are masked out of the power sums.
struct QrCtx {
  int nvl, lane;
  f32x2 c2;
};
template <int L, int I, int P, bool MASKROWS>
SVOC_DEV float qr_tree(const QrCtx& c, const uint32_t (&wv)[64], f32x2& s1, f32x2& s2, f32x2& s3, f32x2& s4) {
  // (no implicit contraction: every instantiation must round identically -- only the explicit fmas below;
  // left to the backend, y * y + s2 was fused in some instantiations and not in others.  The fmas are
  // written out: unfused mul + add took the N <= 64 kernel from 5 to 36 VGPR spills,
  // profiles/r4_win_bf16_qr_fma_ab.txt)
#pragma clang fp contract(off)
  if constexpr (L == 0) {
    f32x2 y = bf16x2_to_f32x2(wv[I]) - c.c2;
    f32x2 q = y * y;
    const float part = __builtin_fmaf(y.x, y.x, q.y);
    if (MASKROWS) {
      const uint32_t rm = lt_mask(I, c.nvl);
      y = fand2(y, rm);
      q = fand2(q, rm);
    }
    s1 += y;
    s2 = __builtin_elementwise_fma(y, y, s2);
    s3 = __builtin_elementwise_fma(q, y, s3);
    s4 = __builtin_elementwise_fma(q, q, s4);
    return part;
  } else {
    constexpr int msk = P >> L;
    const float lo_v = qr_tree<L - 1, I, P, MASKROWS>(c, wv, s1, s2, s3, s4);
    const float hi_v = qr_tree<L - 1, I + (64 >> L), P, MASKROWS>(c, wv, s1, s2, s3, s4);
    if constexpr (msk == 32 || msk == 16) {
      // one v_permlane{32,16}_swap: the lower lane ends with (own lo, partner's lo), the upper lane with
      // (partner's hi, own hi) -- the same sums as the select form below, no selects
      uint32_t x = __builtin_bit_cast(uint32_t, lo_v), y = __builtin_bit_cast(uint32_t, hi_v);
      xswap<msk>(x, y);
      return __builtin_bit_cast(float, x) + __builtin_bit_cast(float, y);
    } else {
      const bool up = (c.lane & msk) != 0;
      const float send = up ? lo_v : hi_v;
      const float keep = up ? hi_v : lo_v;
      return keep + xor_lane<msk>(send);
    }
  }
}
// One butterfly tree (final slot I): its 64/KEEP rows I, I + KEEP, ... are loaded together (all in
// flight at once), then reduced depth-first; an empty asm closes the tree so the next tree's loads
// are not hoisted into this one (only one tree's words live: no spills at NSEG 4).
template <int P, int I, bool MASKW, bool MASKROWS>
SVOC_DEV void qr_tree_slot(__amdgpu_buffer_rsrc_t rs, int vo, int rowb, uint32_t mW, const QrCtx& c, float* acc,
                           f32x2& s1, f32x2& s2, f32x2& s3, f32x2& s4) {
  constexpr int KEEP = 64 / P;
  uint32_t wv[64];
#pragma unroll
  for (int m = 0; m < 64 / KEEP; ++m) {
    const int i = I + KEEP * m;
    wv[i] = bload(rs, vo, i * rowb);
    if (MASKW) wv[i] &= mW;
  }
  constexpr int S = __builtin_ctz(P);   // butterfly stages: log2(P)
  acc[I] += qr_tree<S, I, P, MASKROWS>(c, wv, s1, s2, s3, s4);
  asm volatile("" : "+v"(acc[I]), "+v"(s1), "+v"(s2), "+v"(s3), "+v"(s4));
}
template <int P, bool MASKW, bool MASKROWS, int... Is>
SVOC_DEV void qr_moments_seq(__amdgpu_buffer_rsrc_t rs, int vo, int rowb, uint32_t mW, const QrCtx& c, float* acc,
                             f32x2& s1, f32x2& s2, f32x2& s3, f32x2& s4, std::integer_sequence<int, Is...>) {
  (qr_tree_slot<P, Is, MASKW, MASKROWS>(rs, vo, rowb, mW, c, acc, s1, s2, s3, s4), ...);
}
template <int P, bool MASKW, bool MASKROWS>
SVOC_DEV void qr_moments(__amdgpu_buffer_rsrc_t rs, int vo, int rowb, uint32_t mW, const QrCtx& c, float* acc,
                         f32x2& s1, f32x2& s2, f32x2& s3, f32x2& s4) {
  qr_moments_seq<P, MASKW, MASKROWS>(rs, vo, rowb, mW, c, acc, s1, s2, s3, s4,
                                     std::make_integer_sequence<int, 64 / P>{});
}

// qr pass with half of the slab staged in LDS (N = NPAD = 256, constrained): trees 0 and 1 (rows
// i % 4 < 2, 32 rows) were written to the wave's LDS region as keys right after the pass-1 load; trees
// 2 and 3 (32 rows) are re-read from memory, all 32 loads issued first so their latency overlaps the
// LDS trees.  Same trees, same order of accumulation as qr_moments: bit-identical results.
template <int P, bool MASKW>
SVOC_DEV void qr_moments_staged(__amdgpu_buffer_rsrc_t rs, int vo, int rowb, uint32_t mW, uint32_t kp,
                                const uint32_t* st, int lane, const QrCtx& c, float* acc, f32x2& s1, f32x2& s2,
                                f32x2& s3, f32x2& s4) {
  static_assert(P == 16, "staging layout: KEEP = 4 trees of 16 rows");
  constexpr int KEEP = 4, S = 4;
  uint32_t wm[64];   // trees 2 and 3 from memory (indices i % 4 >= 2)
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    wm[2 + KEEP * m] = bload(rs, vo, (2 + KEEP * m) * rowb);
    wm[3 + KEEP * m] = bload(rs, vo, (3 + KEEP * m) * rowb);
  }
  {
    uint32_t wv[64];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      wv[KEEP * m] = st[(2 * m) * 64 + lane] ^ kp;
      if (MASKW) wv[KEEP * m] &= mW;
    }
    acc[0] += qr_tree<S, 0, P, false>(c, wv, s1, s2, s3, s4);
    asm volatile("" : "+v"(acc[0]), "+v"(s1), "+v"(s2), "+v"(s3), "+v"(s4));
  }
  {
    uint32_t wv[64];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      wv[1 + KEEP * m] = st[(2 * m + 1) * 64 + lane] ^ kp;
      if (MASKW) wv[1 + KEEP * m] &= mW;
    }
    acc[1] += qr_tree<S, 1, P, false>(c, wv, s1, s2, s3, s4);
    asm volatile("" : "+v"(acc[1]), "+v"(s1), "+v"(s2), "+v"(s3), "+v"(s4));
  }
  if (MASKW) {
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      wm[2 + KEEP * m] &= mW;
      wm[3 + KEEP * m] &= mW;
    }
  }
  acc[2] += qr_tree<S, 2, P, false>(c, wm, s1, s2, s3, s4);
  asm volatile("" : "+v"(acc[2]), "+v"(s1), "+v"(s2), "+v"(s3), "+v"(s4));
  acc[3] += qr_tree<S, 3, P, false>(c, wm, s1, s2, s3, s4);
}

// qr pass with half of the slab staged in LDS for N <= 128 (NSEG 1 and 2, constrained): the even rows
// (tree 0 when KEEP = 2, read into its own array so only that tree's words are live next to the 32
// in-flight loads; the first butterfly half of the single tree when KEEP = 1) come from the wave's
// LDS region, the odd rows are re-read from memory with all 32 loads issued before the LDS reads.
// Same trees, same leaf order as qr_moments: bit-identical results.
template <int P, bool MASKW>
SVOC_DEV void qr_moments_staged_even(__amdgpu_buffer_rsrc_t rs, int vo, int rowb, uint32_t mW, uint32_t kp,
                                     const uint32_t* st, int lane, const QrCtx& c, float* acc, f32x2& s1,
                                     f32x2& s2, f32x2& s3, f32x2& s4) {
  constexpr int KEEP = 64 / P, S = __builtin_ctz(P);
  static_assert(KEEP <= 2, "even-row staging: one or two trees");
  if constexpr (KEEP == 1) {
    uint32_t wv[64];
#pragma unroll
    for (int m = 0; m < 32; ++m) wv[2 * m + 1] = bload(rs, vo, (2 * m + 1) * rowb);
#pragma unroll
    for (int m = 0; m < 32; ++m) wv[2 * m] = st[m * 64 + lane] ^ kp;
    if (MASKW) {
#pragma unroll
      for (int i = 0; i < 64; ++i) wv[i] &= mW;
    }
    acc[0] += qr_tree<S, 0, P, false>(c, wv, s1, s2, s3, s4);
  } else {
    uint32_t wm[64];   // tree 1 (odd rows) from memory, loads issued first
#pragma unroll
    for (int m = 0; m < 32; ++m) wm[2 * m + 1] = bload(rs, vo, (2 * m + 1) * rowb);
    {
      uint32_t wv[64];
#pragma unroll
      for (int m = 0; m < 32; ++m) {
        wv[2 * m] = st[m * 64 + lane] ^ kp;
        if (MASKW) wv[2 * m] &= mW;
      }
      acc[0] += qr_tree<S, 0, P, false>(c, wv, s1, s2, s3, s4);
      asm volatile("" : "+v"(acc[0]), "+v"(s1), "+v"(s2), "+v"(s3), "+v"(s4));
    }
    if (MASKW) {
#pragma unroll
      for (int m = 0; m < 32; ++m) wm[2 * m + 1] &= mW;
    }
    acc[1] += qr_tree<S, 1, P, false>(c, wm, s1, s2, s3, s4);
  }
}

template <int NSEG, int WAVES, int H, bool CONS, int MODE>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(4))) void consensus_fast_win_kernel(FastParams p) {
#pragma clang fp contract(off)   // (as qr_tree: every instantiation rounds the same way)
  constexpr int P = 64 / NSEG;          // column pairs per wave (phase A)
  constexpr int NPAD = 64 * NSEG;
  constexpr int W = WAVES * P * 2;      // columns per workgroup step (phase A)
  constexpr int NT = WAVES * 64;
  constexpr int KEEP = 64 / P;
  // constrained: half of each slab (32 rows x 64 lanes, keys) staged per wave for the qr pass
  // (N = 256: rows i % 4 < 2; N <= 128: even rows; profiles/r1_stage_ab.txt)
  constexpr bool STAGE = CONS && MODE != 2;
  __shared__ uint32_t stage[STAGE ? WAVES * 32 * 64 : 1];
  __shared__ __attribute__((aligned(16))) float qr_part[WAVES * NPAD];   // (then the rank keys: 2 NPAD words)
  __shared__ float qr_lds[NPAD];
  __shared__ uint64_t relmask[4];
  __shared__ int urow[32];      // removed rows, index order
  __shared__ float misc_f[2];
  __shared__ int misc_i[3];     // status, zero-variance flag, cleanup list length

  const int b = blockIdx.x;
  if (p.active && !p.active[b]) return;   // (no round, no rollback: the instance keeps its updates)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < 32) urow[tid] = 0;  // f < 32: unused slots still name a valid row
  if (tid == 0) misc_i[2] = 0;
  const int seg = lane / P, pair_w = lane % P;
  const int cp = wave * P + pair_w;
  const int N = p.N, D = p.D;
  const int rowb = p.ld * 2;
  const uint16_t* inst = (const uint16_t*)p.values + (int64_t)b * p.inst_stride;
  const __amdgpu_buffer_rsrc_t rs = instance_rsrc(inst, (uint32_t)(N * rowb));
  const int nslab = (D + W - 1) / W;
  const int Dp = p.work_pairs;
  // this instance's workspace (buffer ops, 32-bit offsets): [H][2][Dp] window keys, then at byte
  // offset MOM the [4][Dp] float2 all-row power sums, then at LST the [2 Dp] cleanup column list
  const __amdgpu_buffer_rsrc_t ws = instance_rsrc(p.work + (int64_t)b * p.work_stride, (uint32_t)(p.work_stride * 4));
  const int MOM = 2 * H * Dp * 4;
  const int LST = MOM + 4 * Dp * 8;
  const int lo1 = (NPAD - N + 1) >> 1;
  const int nv = N - seg * 64;
  const int nl = N + lo1 - seg * 64;
  const int seg_off = seg * 64 * rowb;
  const uint32_t pol = group_polarity<NSEG>(seg);
  const uint32_t kp = 0x80008000u ^ pol;   // constrained key = raw ^ kp
  uint32_t* const stw = stage + (STAGE ? wave * 32 * 64 : 0);
  // a reverting round's exit (uniform over the workgroup): the status, and with FastParams.rst_saved the
  // rollback of this instance's saved update batch (launch.hpp)
  auto revert = [&](int st) __attribute__((always_inline)) {
    if (tid == 0) p.status[b] = st;
    if (MODE != 0 || !p.rst_saved) return;
    const int U = p.rst_U;
    const int64_t u0 = (int64_t)b * U;
    uint16_t* const vals = (uint16_t*)p.values + (int64_t)b * p.inst_stride;
    for (int j = 0; j < U; ++j) {   // (uniform: every thread reads the same update)
      const int64_t u = u0 + j;
      if (p.rst_status[u] != ST_OK) continue;
      const int64_t o = p.rst_oracle[u];
      const uint8_t was = p.rst_saved_en[u];
      if (o < 0 || o >= N || was == kNotSaved) continue;
      const uint16_t* src = (const uint16_t*)p.rst_saved + u * D;
      uint16_t* dst = vals + o * p.ld;
      for (int c = tid; c < D; c += NT) dst[c] = src[c];
      if (was == 0 && tid == 0) {
        p.rst_enabled[(int64_t)b * N + o] = 0;
        p.rst_n_active[b] -= 1;
      }
    }
    __syncthreads();   // (every thread has read the statuses above)
    for (int j = tid; j < U; j += NT) {
      const int64_t u = u0 + j, o = p.rst_oracle[u];
      if (p.rst_status[u] == ST_OK && o >= 0 && o < N) p.rst_status[u] = st;
    }
  };

  float acc[KEEP];
#pragma unroll
  for (int i = 0; i < KEEP; ++i) acc[i] = 0.f;

  // ------------------------------------------------------------ phase A: pass 1
  const int pass1_slabs = MODE == 2 ? 0 : nslab;
#pragma nounroll
  for (int s = 0; s < pass1_slabs; ++s) {
    const int colA = s * W + 2 * cp;
    const int pg = s * (W / 2) + cp;    // workspace pair index
    const bool vA = colA < D, vB = colA + 1 < D;
    const int vo = seg_off + (vA ? colA * 2 : 0);
    int nvl = nv, nll = nl;
    asm volatile("" : "+v"(nvl), "+v"(nll));
    float cA, cB;
    const uint32_t mW = vA ? (vB ? 0xffffffffu : 0x0000ffffu) : 0u;
    {
      u16x2 r[64];
      if (N == NPAD) {
        if (CONS) {
#pragma unroll
          for (int i = 0; i < 64; ++i) r[i] = as_k(bload(rs, vo, i * rowb) ^ kp);
          if constexpr (STAGE && NSEG == 4) {
#pragma unroll
            for (int m = 0; m < 16; ++m) {
              stw[(2 * m) * 64 + lane] = as_u32(r[4 * m]);
              stw[(2 * m + 1) * 64 + lane] = as_u32(r[4 * m + 1]);
            }
          } else if constexpr (STAGE) {
#pragma unroll
            for (int m = 0; m < 32; ++m) stw[m * 64 + lane] = as_u32(r[2 * m]);
          }
        } else {
#pragma unroll
          for (int i = 0; i < 64; ++i) r[i] = as_k(as_u32(to_key<CONS>(bload(rs, vo, i * rowb))) ^ pol);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          const uint32_t hi_m = ~lt_mask(i, nll);
          r[i] = as_k(((as_u32(to_key<CONS>(bload(rs, vo, i * rowb))) & (lt_mask(i, nvl) | hi_m)) | hi_m) ^ pol);
        }
      }
      u16x2 klo, khi;
      if constexpr (CONS) {
        u16x2 wk[NSEG == 1 ? 2 * H : H];
        window_group<NSEG, P, H>(r, seg, lane, wk, klo, khi);
        if constexpr (NSEG == 1) {
#pragma unroll
          for (int m = 0; m < H; ++m) {
            bstore(ws, as_u32(wk[m]), pg * 4, 2 * m * Dp * 4);
            bstore(ws, as_u32(wk[H + m]), (Dp + pg) * 4, 2 * m * Dp * 4);
          }
        } else {
          constexpr int slo = NSEG == 2 ? 0 : 1;
          if (seg == slo || seg == slo + 1) {
            const int part = seg - slo;
#pragma unroll
            for (int m = 0; m < H; ++m) bstore(ws, as_u32(wk[m]), (part * Dp + pg) * 4, 2 * m * Dp * 4);
          }
        }
      } else {
        median_group<NSEG>(r, klo, khi);
      }
      const uint32_t lo = from_key<CONS>(klo), hi = from_key<CONS>(khi);
      cA = 0.5f * (bf16_lo(lo) + bf16_lo(hi));
      cB = 0.5f * (bf16_hi(lo) + bf16_hi(hi));
    }
    if (seg == 0) {
      if (vA) p.c1[(int64_t)b * D + colA] = cA;
      if (vB) p.c1[(int64_t)b * D + colA + 1] = cB;
    }
    __builtin_amdgcn_sched_barrier(0);
    // the re-read's offset depends on the network's result (empty asm): otherwise the 64 loads are
    // hoisted above the network and both 64-register arrays are live at once (spills)
    int vo2 = vo;
    asm volatile("" : "+v"(vo2) : "v"(cA), "v"(cB));
    const QrCtx qc{nvl, lane, f32x2{vA ? cA : 0.f, vB ? cB : 0.f}};
    f32x2 s1 = {0.f, 0.f}, s2 = s1, s3 = s1, s4 = s1;
    if (STAGE && N == NPAD) {
      if constexpr (STAGE && NSEG == 4) {
        if ((s + 1) * W <= D) qr_moments_staged<P, false>(rs, vo2, rowb, mW, kp, stw, lane, qc, acc, s1, s2, s3, s4);
        else qr_moments_staged<P, true>(rs, vo2, rowb, mW, kp, stw, lane, qc, acc, s1, s2, s3, s4);
      } else if constexpr (STAGE) {
        if ((s + 1) * W <= D) qr_moments_staged_even<P, false>(rs, vo2, rowb, mW, kp, stw, lane, qc, acc, s1, s2, s3, s4);
        else qr_moments_staged_even<P, true>(rs, vo2, rowb, mW, kp, stw, lane, qc, acc, s1, s2, s3, s4);
      }
    } else if ((s + 1) * W <= D) {
      if (N == NPAD) qr_moments<P, false, false>(rs, vo2, rowb, mW, qc, acc, s1, s2, s3, s4);
      else qr_moments<P, false, true>(rs, vo2, rowb, mW, qc, acc, s1, s2, s3, s4);
    } else {
      if (N == NPAD) qr_moments<P, true, false>(rs, vo2, rowb, mW, qc, acc, s1, s2, s3, s4);
      else qr_moments<P, true, true>(rs, vo2, rowb, mW, qc, acc, s1, s2, s3, s4);
    }
    if constexpr (NSEG == 4) {
      s1.x += xor_lane<16>(s1.x); s1.y += xor_lane<16>(s1.y); s2.x += xor_lane<16>(s2.x); s2.y += xor_lane<16>(s2.y);
      s3.x += xor_lane<16>(s3.x); s3.y += xor_lane<16>(s3.y); s4.x += xor_lane<16>(s4.x); s4.y += xor_lane<16>(s4.y);
    }
    if constexpr (NSEG >= 2) {
      s1.x += xor_lane<32>(s1.x); s1.y += xor_lane<32>(s1.y); s2.x += xor_lane<32>(s2.x); s2.y += xor_lane<32>(s2.y);
      s3.x += xor_lane<32>(s3.x); s3.y += xor_lane<32>(s3.y); s4.x += xor_lane<32>(s4.x); s4.y += xor_lane<32>(s4.y);
    }
    if (seg == 0) {
      bstore2(ws, s1, pg * 8, MOM);
      bstore2(ws, s2, pg * 8, MOM + Dp * 8);
      bstore2(ws, s3, pg * 8, MOM + 2 * Dp * 8);
      bstore2(ws, s4, pg * 8, MOM + 3 * Dp * 8);
    }
  }

  // ------------------------------------------------------------ qr reduction
  {
    int base = 0;
#pragma unroll
    for (int h = 32, msk = P / 2; msk >= 1; h >>= 1, msk >>= 1) base += (lane & msk) ? h : 0;
#pragma unroll
    for (int i = 0; i < KEEP; ++i) qr_part[wave * NPAD + seg * 64 + base + i] = acc[i];
  }
  __syncthreads();
  for (int t = tid; t < NPAD; t += NT) {
    float q = 0.f;
    if (MODE == 2) {
      q = t < N ? p.qr[(int64_t)b * N + t] : 0.f;
    } else {
#pragma unroll
      for (int w = 0; w < WAVES; ++w) q += qr_part[w * NPAD + t];
    }
    qr_lds[t] = q;
  }
  __syncthreads();
  if (MODE == 1) {
    for (int t = tid; t < N; t += NT) p.qr[(int64_t)b * N + t] = qr_lds[t];
    if (tid == 0) p.status[b] = ST_OK;
    return;
  }

  // ------------------------------------------------------------ rank mask (contract.cairo:345-363)
  const int f = p.n_failing;
  const int R = N - f;
  if constexpr (CONS) {
    static_assert(WAVES >= 2, "rank keys in qr_part");
    rank_mask_nonneg<NT, NPAD>(qr_lds, reinterpret_cast<uint64_t*>(qr_part), N, R, tid, relmask);
  } else
  for (int base = 0; base < NPAD; base += NT) {
    const int t = base + tid;
    bool rel = false;
    if (t < N) {
      const float myq = qr_lds[t];
      int rank = 0;
      const int n4 = N & ~3;
      for (int j = 0; j < n4; j += 4) {
        const float4 q4 = *(const float4*)(qr_lds + j);
        rank += (q4.x < myq || (q4.x == myq && j > t)) ? 1 : 0;
        rank += (q4.y < myq || (q4.y == myq && j + 1 > t)) ? 1 : 0;
        rank += (q4.z < myq || (q4.z == myq && j + 2 > t)) ? 1 : 0;
        rank += (q4.w < myq || (q4.w == myq && j + 3 > t)) ? 1 : 0;
      }
      for (int j = n4; j < N; ++j) {
        const float qj = qr_lds[j];
        rank += (qj < myq || (qj == myq && j > t)) ? 1 : 0;
      }
      rel = rank < R;
    }
    const uint64_t bal = __ballot(rel);
    if (lane == 0 && (t >> 6) < 4) relmask[t >> 6] = bal;
  }
  __syncthreads();
  // removed rows in index order (pass 2 reads only these)
  for (int t = tid; t < N; t += NT) {
    const int w = t >> 6;
    const uint64_t nr = ~relmask[w];
    if ((nr >> (t & 63)) & 1) {
      int cnt = __popcll(nr & ((1ull << (t & 63)) - 1));
      for (int v = 0; v < w; ++v) cnt += __popcll(~relmask[v]);
      if (cnt < 32) urow[cnt] = t;
    }
  }
  if (tid < 64) {
    float s_all = 0.f, s_rel = 0.f;
    for (int t = tid; t < N; t += 64) {
      const float q = qr_lds[t];
      s_all += q;
      s_rel += ((relmask[t >> 6] >> (t & 63)) & 1) ? q : 0.f;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      s_all += __shfl_xor(s_all, o);
      s_rel += __shfl_xor(s_rel, o);
    }
    if (tid == 0) {
      int st = ST_OK;
      const float rd = p.legacy ? 1.f : (float)(p.rel_dim > 0 ? p.rel_dim : D);
      float rel1, rel2 = 0.f;
      if (CONS) rel1 = 1.f - 2.f * sqrtf(s_all / (float)N / rd);
      else rel1 = 1.f - fminf(p.max_spread, sqrtf(s_all / (float)N)) / p.max_spread;
      if (!(rel1 >= 0.f && rel1 <= 1.f)) st = ST_RELIABILITY_INTERVAL;
      else if (R < 2) st = R <= 0 ? ST_USIZE_UNDERFLOW : ST_INDEX_OOB;
      else {
        if (CONS) rel2 = 1.f - 2.f * sqrtf(s_rel / (float)R / rd);
        else rel2 = 1.f - fminf(p.max_spread, sqrtf(s_rel / (float)R)) / p.max_spread;
        if (!(rel2 >= 0.f && rel2 <= 1.f)) st = ST_RELIABILITY_INTERVAL;
        else if (R < 4 && !p.legacy) st = ST_TOO_FEW_RELIABLE;
      }
      misc_f[0] = rel1;
      misc_f[1] = rel2;
      misc_i[0] = st;
      misc_i[1] = 0;
    }
  }
  __syncthreads();
  if (misc_i[0] != ST_OK) {
    revert(misc_i[0]);
    return;
  }
  const int npairs = (D + 1) >> 1;

  // ------------------------------------------------------------ zero-variance pre-check (constrained)
  // A reliable column of zero variance reverts the whole round (sqrt(0) -> wsad_div by zero,
  // math.cairo:322,331; contract.cairo:588-603).  Fast mode: ZERO_VARIANCE <=> the reliable values of
  // some column are all equal.  It is decided here, before any output is written.  The R equal values
  // would form a sorted run covering positions [f, N - f - 1]; when f + H <= N/2 that run contains the
  // whole pass-1 window, so only columns whose window is constant (lowest key == highest key) qualify
  // -- usually none -- and only those are compared against the reliable rows.  Otherwise every
  // column is.  (Unconstrained rounds stage their outputs instead: no window.)
  if (CONS && !p.legacy) {
    const bool inwin = f + H <= N / 2;
    int fr = 0;   // first reliable row
    for (int w = 0; w < 4; ++w)
      if (relmask[w]) { fr = 64 * w + __builtin_ctzll(relmask[w]); break; }
    bool zv = false;
#pragma nounroll
    for (int base = wave * 64; base < npairs; base += WAVES * 64) {
      const int pair = base + lane;
      const int pr = pair < npairs ? pair : npairs - 1;
      bool cA = pair < npairs, cB = pair < npairs && 2 * pair + 1 < D;
      if (inwin) {
        // compared as values: a run of +0.0 and -0.0 is constant, but its keys differ
        const uint32_t lo = key_to_pos(as_k(bload(ws, pr * 4, 0))), hi = key_to_pos(~as_k(bload(ws, (Dp + pr) * 4, 0)));
        cA = cA && bf16_lo(lo) == bf16_lo(hi);
        cB = cB && bf16_hi(lo) == bf16_hi(hi);
      }
      if (__ballot(cA || cB)) {   // rare: compare the reliable rows with the first one
        const uint32_t w0 = bload(rs, pr * 4, fr * rowb);
        const float rA = bf16_lo(w0), rB = bf16_hi(w0);
        for (int i = fr + 1; i < N; ++i) {
          if (!((relmask[i >> 6] >> (i & 63)) & 1)) continue;   // uniform
          const uint32_t w = bload(rs, pr * 4, i * rowb);
          cA = cA && bf16_lo(w) == rA;
          cB = cB && bf16_hi(w) == rB;
        }
        zv = zv || cA || cB;
      }
    }
    if (zv) misc_i[1] = 1;
    __syncthreads();
    if (misc_i[1]) {
      revert(ST_ZERO_VARIANCE);
      return;
    }
  }
  if (CONS) {
    for (int t = tid; t < N; t += NT) {
      p.reliable[(int64_t)b * N + t] = (relmask[t >> 6] >> (t & 63)) & 1;
      p.qr[(int64_t)b * N + t] = qr_lds[t];
    }
  }
  // unconstrained: pass-2 outputs are staged in the workspace and committed at the end
  const int D2 = 2 * Dp;
  const int STG = Dp * (2 * 17 + 8 + 2) * 4;   // launch.hpp: fast_work_stage_word

  // ------------------------------------------------------------ phase B: pass 2 (contract.cairo:476-500)
  // one lane per column pair: the removed keys are sorted once (true key order) and ranked against
  // both window halves; packed power sums for the two columns
  const float n = (float)R;
  const MomK mk = mom_k(n);
  const int sh = H - 1 - (N / 2 - R / 2);   // -inf sentinels in front of the removed keys
  const int64_t ob = (int64_t)b * D;
  bool zv = false;
#pragma nounroll
  for (int base = wave * 64; base < npairs; base += WAVES * 64) {
    const int pair = base + lane;
    const int pr = pair < npairs ? pair : npairs - 1;
    const int vo = pr * 4;
    const float c1A = p.c1[ob + 2 * pr];
    const float c1B = 2 * pr + 1 < D ? p.c1[ob + 2 * pr + 1] : 0.f;
    const f32x2 c2 = {c1A, c1B};
    // opaque per-iteration copies: otherwise LICM hoists the 2H slot offsets / masks (uniform,
    // loop-invariant) out of the pair loop and keeps them live in VGPRs (spills)
    int shl = sh, fl = f;
    asm volatile("" : "+s"(shl), "+s"(fl));
    // the removed rows' words, all loads in flight at once (uniform row offsets).  Constrained: the
    // 2H network slots (slot t = removed row t - sh; the others become sentinels below);
    // unconstrained: the f <= 32 removed rows
    constexpr int NS = CONS ? 2 * H : 32;
    const int s0 = CONS ? shl : 0;
    // slot bit masks (uniform): real = a removed row, low = a -inf sentinel
    const uint64_t realm = ((fl >= 64 ? ~0ull : (1ull << fl) - 1)) << s0;
    const uint64_t lowm = (1ull << s0) - 1;
    uint32_t uw[NS];
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      const int row = t - s0;
      const bool real = (realm >> t) & 1;
      uw[t] = 0u;
      if (CONS || real) uw[t] = bload(rs, vo, __builtin_amdgcn_readfirstlane(urow[real ? row : 0]) * rowb);
    }
    // removed rows' power sums of d = x - c1 (both columns, packed)
    f32x2 u1 = {0.f, 0.f}, u2 = u1, u3 = u1, u4 = u1;
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      if ((realm >> t) & 1) {   // uniform
        const f32x2 y = bf16x2_to_f32x2(uw[t]) - c2;
        const f32x2 q = y * y;
        u1 += y;
        u2 += q;
        u3 = __builtin_elementwise_fma(q, y, u3);
        u4 = __builtin_elementwise_fma(q, q, u4);
      }
    }

    uint32_t medw = 0u;   // pass-2 middle pair (true keys) of both columns: lo, hi
    uint32_t mhw = 0u;
    if constexpr (CONS && H == 5) {
      // c2's shape (N = 64, f = 8, sentinel shift 0): U' = the f sorted removed keys, then +inf -- an 8-key network
      // instead of the 64-slot one (at H = 17 the 32-key form took the 128-VGPR kernel to scratch:
      // profiles/r6_rank_key_ab.txt); other shapes the general form below
      auto cands = [&](const auto& z) __attribute__((always_inline)) {
        u16x2 clo = as_k(~0u), chi = as_k(~0u);
#pragma unroll
        for (int m = 0; m < H; ++m) {
          const u16x2 wl = as_k(bload(ws, pr * 4, 2 * m * Dp * 4));
          const u16x2 wu = ~as_k(bload(ws, (Dp + pr) * 4, 2 * m * Dp * 4));
          clo = kmin(clo, win_cand(wl, z(m)));
          if (m) chi = kmin(chi, win_cand(wl, z(m - 1)));
          clo = kmin(clo, win_cand(wu, z(2 * H - 1 - m)));
          chi = kmin(chi, win_cand(wu, z(2 * H - 2 - m)));
        }
        medw = key_to_pos(clo);
        mhw = key_to_pos(chi);
      };
      constexpr int NF = 8;
      if (s0 == 0 && fl == NF) {   // (uniform)
        u16x2 z[NF];
#pragma unroll
        for (int t = 0; t < NF; ++t) z[t] = as_k(uw[t < NS ? t : 0] ^ 0x80008000u);
        sort_oem<NF>(z);
        cands([&](int t) __attribute__((always_inline)) { return t < NF ? z[t < NF ? t : 0] : as_k(~0u); });
      } else {
        u16x2 z[64];
#pragma unroll
        for (int t = 0; t < 64; ++t) {
          if (t < 2 * H) {
            const uint32_t mreal = 0u - (uint32_t)((realm >> t) & 1);
            const uint32_t kx = (0x80008000u & mreal) | (~mreal & (0u - (uint32_t)(((~lowm) >> t) & 1)));
            z[t] = as_k((uw[t] & mreal) ^ kx);
          } else {
            z[t] = as_k(~0u);
          }
        }
        sort_oem<64>(z);
        cands([&](int t) __attribute__((always_inline)) { return z[t]; });
      }
    } else if constexpr (CONS) {
      // removed keys + sentinels: U'[t], t < 2H, ascending true keys
      u16x2 z[64];
#pragma unroll
      for (int t = 0; t < 64; ++t) {
        if (t < 2 * H) {
          // scalar masks only: real slot -> key, else the -inf (0) / +inf (~0) sentinel
          const uint32_t mreal = 0u - (uint32_t)((realm >> t) & 1);
          const uint32_t kx = (0x80008000u & mreal) | (~mreal & (0u - (uint32_t)(((~lowm) >> t) & 1)));
          z[t] = as_k((uw[t] & mreal) ^ kx);
        } else {
          z[t] = as_k(~0u);
        }
      }
      sort_oem<64>(z);
      // lower window half: position c - H + m pairs with U'[m] (lo) / U'[m - 1] (hi); upper half
      // (stored complemented, position c + H - 1 - m): U'[2H - 1 - m] (lo) / U'[2H - 2 - m] (hi)
      u16x2 clo = as_k(~0u), chi = as_k(~0u);
#pragma unroll
      for (int m = 0; m < H; ++m) {
        const u16x2 wl = as_k(bload(ws, pr * 4, 2 * m * Dp * 4));
        const u16x2 wu = ~as_k(bload(ws, (Dp + pr) * 4, 2 * m * Dp * 4));
        clo = kmin(clo, win_cand(wl, z[m]));
        if (m) chi = kmin(chi, win_cand(wl, z[m - 1]));
        clo = kmin(clo, win_cand(wu, z[2 * H - 1 - m]));
        chi = kmin(chi, win_cand(wu, z[2 * H - 2 - m]));
      }
      medw = key_to_pos(clo);
      mhw = key_to_pos(chi);
    }

    // reliable rows' power sums = all-row sums (phase A) - removed rows' sums
    const int mo = pr * 8;
    const f32x2 sa1 = {bloadf(ws, mo, MOM), bloadf(ws, mo + 4, MOM)};
    const f32x2 sa2 = {bloadf(ws, mo, MOM + Dp * 8), bloadf(ws, mo + 4, MOM + Dp * 8)};
    const f32x2 sa3 = {bloadf(ws, mo, MOM + 2 * Dp * 8), bloadf(ws, mo + 4, MOM + 2 * Dp * 8)};
    const f32x2 sa4 = {bloadf(ws, mo, MOM + 3 * Dp * 8), bloadf(ws, mo + 4, MOM + 3 * Dp * 8)};
    const f32x2 t1 = sa1 - u1, t2 = sa2 - u2, t3 = sa3 - u3, t4 = sa4 - u4;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int col = 2 * pr + h;
      if (!(pair < npairs && col < D)) continue;
      const float a2 = h ? sa2.y : sa2.x, a4 = h ? sa4.y : sa4.x;
      const float r2 = h ? t2.y : t2.x, r4 = h ? t4.y : t4.x;
      // trusted: no deep cancellation in the all-minus-removed difference, and the reliable mean
      // within 2 sigma of the shift c1 (moments about a far shift cancel like (dl^2 / mu2)^2)
      const float rdl = (h ? t1.y : t1.x) * mk.in, rmu2 = r2 * mk.in - rdl * rdl;
      const bool good = r2 > 0.f && a2 <= p.win_cancel * r2 && a4 <= p.win_cancel * r4 && rdl * rdl <= 4.f * rmu2;
      if (CONS) {
        p.consensus[ob + col] = h ? 0.5f * (bf16_hi(medw) + bf16_hi(mhw)) : 0.5f * (bf16_lo(medw) + bf16_lo(mhw));
        if (MODE == 0 && p.c1_out) p.c1_out[ob + col] = h ? c1B : c1A;   // (no revert after the pre-check)
      }
      if (good) {
        float dl, sk, ku;
        const bool nz = moments_from_sums(mk, h ? t1.y : t1.x, r2, h ? t3.y : t3.x, r4, dl, sk, ku);
        if (CONS) {
          p.skew[ob + col] = p.legacy ? 0.f : sk;
          p.kurt[ob + col] = p.legacy ? 0.f : ku;
        } else {
          stage_out(ws, STG, D2, 0, col, (h ? c1B : c1A) + dl);
          stage_out(ws, STG, D2, 1, col, p.legacy ? 0.f : sk);
          stage_out(ws, STG, D2, 2, col, p.legacy ? 0.f : ku);
          zv |= !nz;
        }
      } else {
        // exact recomputation over the reliable rows below (each column listed once: <= D entries)
        const int k = atomicAdd(&misc_i[2], 1);
        bstore(ws, (uint32_t)col, k * 4, LST);
      }
    }
  }
  if (!CONS && zv && !p.legacy) misc_i[1] = 1;
  __syncthreads();
  // cleanup: one wave per listed column, lanes stride the rows, two-pass wave reductions
  // (math.cairo:320-363): the reliable mean first, then the power sums about it (no cancellation)
  const int nredo = misc_i[2];
  if (nredo) {
    for (int k = wave; k < nredo; k += WAVES) {
      // (sc0: read through the vL1D -- the entry was written by another wave of this workgroup)
      const int col = (int)__builtin_amdgcn_readfirstlane(__builtin_amdgcn_raw_buffer_load_b32(ws, 0, LST + k * 4, 1));
      const float cc = p.c1[ob + col];
      const uint16_t* xc = inst + col;
      float y[NSEG];
      float t1 = 0.f;
#pragma unroll
      for (int g = 0; g < NSEG; ++g) {
        const int i = g * 64 + lane;
        const bool use = i < N && ((relmask[g] >> lane) & 1);
        y[g] = use ? __builtin_bit_cast(float, (uint32_t)xc[(int64_t)i * p.ld] << 16) - cc : 0.f;
        t1 += y[g];
      }
      t1 += xor_lane<1>(t1); t1 += xor_lane<2>(t1); t1 += xor_lane<4>(t1);
      t1 += xor_lane<8>(t1); t1 += xor_lane<16>(t1); t1 += xor_lane<32>(t1);
      const float mu = t1 / n;   // reliable mean - c1
      float c1s = 0.f, t2 = 0.f, t3 = 0.f, t4 = 0.f;
#pragma unroll
      for (int g = 0; g < NSEG; ++g) {
        const int i = g * 64 + lane;
        const bool use = i < N && ((relmask[g] >> lane) & 1);
        const float d = use ? y[g] - mu : 0.f;
        const float q = d * d;
        c1s += d;
        t2 += q;
        t3 = fmaf(q, d, t3);
        t4 = fmaf(q, q, t4);
      }
      c1s += xor_lane<1>(c1s); t2 += xor_lane<1>(t2); t3 += xor_lane<1>(t3); t4 += xor_lane<1>(t4);
      c1s += xor_lane<2>(c1s); t2 += xor_lane<2>(t2); t3 += xor_lane<2>(t3); t4 += xor_lane<2>(t4);
      c1s += xor_lane<4>(c1s); t2 += xor_lane<4>(t2); t3 += xor_lane<4>(t3); t4 += xor_lane<4>(t4);
      c1s += xor_lane<8>(c1s); t2 += xor_lane<8>(t2); t3 += xor_lane<8>(t3); t4 += xor_lane<8>(t4);
      c1s += xor_lane<16>(c1s); t2 += xor_lane<16>(t2); t3 += xor_lane<16>(t3); t4 += xor_lane<16>(t4);
      c1s += xor_lane<32>(c1s); t2 += xor_lane<32>(t2); t3 += xor_lane<32>(t3); t4 += xor_lane<32>(t4);
      if (lane == 0) {
        float dl, sk, ku;
        const bool nz = moments_from_sums(mk, c1s, t2, t3, t4, dl, sk, ku);
        if (CONS) {
          p.skew[ob + col] = p.legacy ? 0.f : sk;
          p.kurt[ob + col] = p.legacy ? 0.f : ku;
        } else {
          stage_out(ws, STG, D2, 0, col, cc + mu + dl);
          stage_out(ws, STG, D2, 1, col, p.legacy ? 0.f : sk);
          stage_out(ws, STG, D2, 2, col, p.legacy ? 0.f : ku);
          if (!nz && !p.legacy) misc_i[1] = 1;
        }
      }
    }
    __syncthreads();
  }
  // ------------------------------------------------------------ commit
  // (constrained: the outputs were written in place -- the pre-check ruled out every revert;
  // unconstrained: copied from the staging area, only when the round succeeded)
  if (!CONS) {
    if (misc_i[1]) {
      revert(ST_ZERO_VARIANCE);
      return;
    }
    commit_staged<NT>(ws, STG, D2, D, tid, p.consensus + ob, p.skew + ob, p.kurt + ob);
    if (MODE == 0 && p.c1_out)
      for (int c = tid; c < D; c += NT) p.c1_out[ob + c] = p.c1[ob + c];
    for (int t = tid; t < N; t += NT) {
      p.reliable[(int64_t)b * N + t] = (relmask[t >> 6] >> (t & 63)) & 1;
      p.qr[(int64_t)b * N + t] = qr_lds[t];
    }
  }
  if (tid == 0) {
    p.rel[2 * (int64_t)b] = misc_f[0];
    p.rel[2 * (int64_t)b + 1] = misc_f[1];
    p.status[b] = ST_OK;
  }
}

template <int NSEG, int WAVES, int H, bool CONS>
static void launch_win_w(const FastParams& p, hipStream_t stream) {
  if (p.mode == 1) hipLaunchKernelGGL((consensus_fast_win_kernel<NSEG, WAVES, H, CONS, 1>), dim3(p.B), dim3(WAVES * 64), 0, stream, p);
  else if (p.mode == 2) hipLaunchKernelGGL((consensus_fast_win_kernel<NSEG, WAVES, H, CONS, 2>), dim3(p.B), dim3(WAVES * 64), 0, stream, p);
  else hipLaunchKernelGGL((consensus_fast_win_kernel<NSEG, WAVES, H, CONS, 0>), dim3(p.B), dim3(WAVES * 64), 0, stream, p);
}

// Waves per workgroup.  One workgroup per instance; 4 waves x 4 workgroups per CU (LDS and the
// 128-VGPR cap) fill the 4 wave slots of every SIMD only from B = 4 x CUs instances on, and c3's
// pipelined step launches ranges of 256-512.  For N > 128, 8 waves (half the slabs per wave, 75 KiB of
// LDS, 2 workgroups per CU) fill the SIMDs from 2 x CUs instances on and measured faster at every range
// count, also at 1024 instances (c3: 4 waves 763 k / 771 k / 690 k rounds/s at 1 / 2 / 4 ranges,
// 8 waves 784 k / 782 k / 803 k, 16 waves 757 k / 775 k / 728 k; profiles/r2_win_waves_ab.jsonl).
// N <= 64 (c2: the grid is full) stays at 4 (profiles/r2_win_waves_c2.jsonl).
static int win_waves(const FastParams& p, int nseg) {
  constexpr int W8 = 8 * 16 * 2;   // columns per 8-wave slab
  return nseg == 4 && p.D >= 2 * W8 ? 8 : 4;
}

template <int NSEG, int H, bool CONS>
static void launch_win_c(const FastParams& p, hipStream_t stream) {
  if constexpr (NSEG == 4) {
    if (win_waves(p, NSEG) == 8) return launch_win_w<NSEG, 8, H, CONS>(p, stream);
  }
  launch_win_w<NSEG, 4, H, CONS>(p, stream);
}

template <int NSEG>
static void launch_win(const FastParams& p, int H, hipStream_t stream) {
  if (!p.constrained) launch_win_c<NSEG, 5, false>(p, stream);   // no window: H = 5 keeps the layout
  else if (H == 5) launch_win_c<NSEG, 5, true>(p, stream);
  else launch_win_c<NSEG, 17, true>(p, stream);
}

}  // namespace svoc

using namespace svoc;

// Returns -2 when the window kernel does not apply (no workspace, f > 32, ...): the caller falls back.
extern "C" int svoc_fast_round_bf16_win(const FastParams* p, hipStream_t stream) {
  if (p->B <= 0) return 0;
  if (!p->work || p->N < 2 || p->N > 256 || p->ld % 8 != 0 || p->D > p->ld) return -2;
  if (p->mode == 2 && p->work_fresh) return -2;   // pass 1 ran elsewhere: no windows to read
  if (p->n_failing < 0 || p->n_failing > 32 || p->n_failing > p->N - 2) return -2;
  const int H = fast_win_h(p->N, p->n_failing);
  if (H == 0) return -2;
  if (p->work_pairs < fast_work_pairs(p->D) || p->work_pairs % 256 != 0 || p->work_stride < fast_work_words(p->D))
    return -1;
  if (p->N <= 64) launch_win<1>(*p, H, stream);
  else if (p->N <= 128) launch_win<2>(*p, H, stream);
  else launch_win<4>(*p, H, stream);
  return (int)hipGetLastError();
}

extern "C" int svoc_fast_round_bf16_reg(const FastParams* p, hipStream_t stream);
extern "C" int svoc_fast_round_bf16_small(const FastParams* p, hipStream_t stream);

// The bf16-storage fast round: which kernel runs.
//   small instances (N <= 16, D <= 128, whole round): several instances per wave, registers only
//     (consensus_fast_small.hip);
//   default: this one-network window kernel where it applies (workspace given, f <= 32, N <= 256);
//   otherwise, and for wave_hint -7 (tests: the cross-check), the two-network register-streaming kernel
//     (consensus_fast_reg.hip).
//   c1 (mode 0 with c1_out): the window and small kernels commit it themselves; after the others,
//   commit_rows does.
extern "C" int svoc_fast_round_bf16(const FastParams* p, hipStream_t stream) {
  if (p->B <= 0) return 0;
  int rc;
  if (p->upd_rows) return -3;   // fused transactional streaming: the fp32 window kernel only
  if (p->wave_hint == 0 && p->mode == 0 && p->N <= 16 && p->D <= 128) {
    if (p->rst_saved) return -3;   // in-kernel rollback: the window kernel only
    return svoc_fast_round_bf16_small(p, stream);   // (commits c1 into c1_out itself)
  } else {
    if (p->wave_hint != -7) {
      rc = svoc_fast_round_bf16_win(p, stream);
      if (rc != -2) return rc;
    }
    if (p->rst_saved) return -3;
    rc = svoc_fast_round_bf16_reg(p, stream);
  }
  if (rc == 0 && p->mode == 0 && p->c1_out)
    rc = svoc_commit_rows(p->c1, p->c1_out, p->status, p->active, p->B, p->D, stream);
  return rc;
}
