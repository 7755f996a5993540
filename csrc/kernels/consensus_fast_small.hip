// Fused two-pass consensus, fast mode, for SMALL instances (N <= 16 oracles, D <= 128 dims):
// several instances per wave, everything in registers, one launch, no LDS, no barrier.
//
// Semantics and outputs are those of consensus_fast_reg.hip (contract/src/contract.cairo:442-503
// constrained / :370-434 unconstrained; smooth median math.cairo:113-126; tie rule sort.cairo:96-101).
// The deployed configuration is 7 oracles x 6 dims (contract/README.md:43-61, client/common.py:8-9,31);
// the general kernels pad every column to 64 rows, i.e. sort 9x more keys than exist.  Here:
//
//   * a group of G lanes (G = next power of two >= ceil(D/2)) owns one instance; lane g of the group
//     holds column pair (2g, 2g+1) of all NR (8 or 16) padded rows in NR VGPRs -- 64/G instances per
//     wave, 256/G per 4-wave workgroup;
//   * pass 1: keys with the sentinel split of the padding rows (median at the fixed positions
//     NR/2-1, NR/2), an odd-even merge network pruned by DCE to those two outputs;
//   * qr: per-lane partial over its column pair, xor-butterfly sum over the group (every lane ends
//     with the bit-identical qr vector: fp add is commutative, so both partners compute a+b);
//   * rank mask, rel1/rel2 and the status are computed redundantly by the G lanes of the group;
//   * pass 2 reuses the raw words still in registers: no second read of the instance.
// The instance is read from HBM exactly once; the kernel is bound by its ~100 B/instance of I/O.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svoc/launch.hpp"
#include "svoc/sortnet.hpp"
#include "svoc/status.hpp"

namespace svoc {

// Butterfly all-reduce over the G lanes of a group on DPP (no LDS crossbar): quad_perm [1,0,3,2]
// and [2,3,0,1] (xor 1, xor 2), row_half_mirror (pairs each quad with the other quad of its 8-lane
// half), row_ror:8 (xor 8 in a 16-lane row); xor 16 / 32 by ds_bpermute.  Every step adds two
// partner values in both lanes, so all G lanes end with the bit-identical sum (fp add commutes).
template <int CTRL>
SVOC_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
SVOC_DEV int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_ROR8 = 0x128;

template <int G>
SVOC_DEV float group_sum(float v) {
  if constexpr (G >= 2) v += dpp_f<DPP_XOR1>(v);
  if constexpr (G >= 4) v += dpp_f<DPP_XOR2>(v);
  if constexpr (G >= 8) v += dpp_f<DPP_HALF_MIRROR>(v);
  if constexpr (G >= 16) v += dpp_f<DPP_ROR8>(v);
  if constexpr (G >= 32) v += __shfl_xor(v, 16);
  if constexpr (G >= 64) v += __shfl_xor(v, 32);
  return v;
}

template <int G>
SVOC_DEV int group_or(int v) {
  if constexpr (G >= 2) v |= dpp_i<DPP_XOR1>(v);
  if constexpr (G >= 4) v |= dpp_i<DPP_XOR2>(v);
  if constexpr (G >= 8) v |= dpp_i<DPP_HALF_MIRROR>(v);
  if constexpr (G >= 16) v |= dpp_i<DPP_ROR8>(v);
  if constexpr (G >= 32) v |= __shfl_xor(v, 16);
  if constexpr (G >= 64) v |= __shfl_xor(v, 32);
  return v;
}

template <bool CONS>
SVOC_DEV uint32_t small_key(uint32_t w) {
  if constexpr (CONS) return as_u32(pos_to_key(w));
  else return as_u32(bf16x2_to_key(w));
}
template <bool CONS>
SVOC_DEV uint32_t small_unkey(u16x2 k) {
  if constexpr (CONS) return key_to_pos(k);
  else return key_to_bf16x2(k);
}

template <int NR, int G, bool CONS>
__global__ __launch_bounds__(256) void consensus_fast_small_kernel(FastParams p) {
  constexpr int IPW = 64 / G;  // instances per wave
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t b = ((int64_t)blockIdx.x * 4 + wave) * IPW + lane / G;
  const int g = lane % G;
  const int N = p.N, D = p.D;
  // no early exit: the group's butterflies need all G lanes; out-of-range groups compute on
  // instance 0 and write nothing
  const bool live = b < p.B && (p.active == nullptr || p.active[b] != 0);
  const int64_t bi = b < p.B ? b : 0;
  const int colA = 2 * g;
  const bool vA = colA < D, vB = colA + 1 < D;
  const uint32_t mW = vA ? (vB ? 0xffffffffu : 0x0000ffffu) : 0u;
  const uint32_t* base = (const uint32_t*)((const uint16_t*)p.values + bi * p.inst_stride) + (vA ? g : 0);
  const int ldw = p.ld >> 1;  // row stride in dwords (ld % 8 == 0)

  uint32_t w[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) w[i] = i < N ? base[(int64_t)i * ldw] & mW : 0u;

  // ---- pass 1: smooth median of all N rows (sentinel split puts ranks N/2-1, N/2 at NR/2-1, NR/2)
  const int lo1 = (NR - N + 1) >> 1;
  float cA, cB;
  {
    u16x2 r[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const uint32_t k = small_key<CONS>(w[i]);
      r[i] = as_k(i < N ? k : (i < N + lo1 ? 0u : 0xffffffffu));
    }
    sort_oem<NR>(r);
    const uint32_t lo = small_unkey<CONS>(r[NR / 2 - 1]), hi = small_unkey<CONS>(r[NR / 2]);
    cA = 0.5f * (bf16_lo(lo) + bf16_lo(hi));
    cB = 0.5f * (bf16_hi(lo) + bf16_hi(hi));
  }
  // c1: with c1_out (mode 0) written at the commit below, where the round succeeded (no staging row and
  // no commit_rows launch after this kernel); without it, into the row the caller passed
  if (live && !p.c1_out) {
    if (vA) p.c1[b * D + colA] = cA;
    if (vB) p.c1[b * D + colA + 1] = cB;
  }
  // ---- quadratic risk per oracle (math.cairo:225-238), summed over the group's column pairs
  const f32x2 c2 = {vA ? cA : 0.f, vB ? cB : 0.f};
  float qr[NR];
  float s_all = 0.f;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const f32x2 y = bf16x2_to_f32x2(w[i]) - c2;
    const f32x2 q = y * y;
    qr[i] = group_sum<G>(i < N ? q.x + q.y : 0.f);
    s_all += qr[i];
  }
  // ---- rank mask (qr asc, idx desc; contract.cairo:345-363), branch-free: with padding rows at
  // +inf, rank_i = #{j < i : qr_j < qr_i} + #{j > i : qr_j <= qr_i}; each pair is compared once
  // (for j < i: c = qr_j < qr_i counts for i, and !c = qr_i <= qr_j counts for j)
  const int R = N - p.n_failing;
  float qk[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) qk[i] = i < N ? qr[i] : __builtin_inff();
  int rank[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) rank[i] = 0;
#pragma unroll
  for (int i = 1; i < NR; ++i)
#pragma unroll
    for (int j = 0; j < i; ++j) {
      const int c = qk[j] < qk[i] ? 1 : 0;
      rank[i] += c;
      rank[j] += 1 - c;
    }
  uint32_t relbits = 0;
  float s_rel = 0.f;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const bool rel = i < N && rank[i] < R;
    relbits |= rel ? (1u << i) : 0u;
    s_rel += rel ? qr[i] : 0.f;
  }
  // divisors are launch-uniform: one reciprocal each instead of a full-precision division per use
  // (the divisions were ~20% of this kernel's VALU instructions; profiles/r2_pmc_c5.md)
  const float rd = p.legacy ? 1.f : (float)(p.rel_dim > 0 ? p.rel_dim : D);
  const float inv_nrd = 1.f / ((float)N * rd), inv_rrd = 1.f / ((float)R * rd);
  const float inv_ms = 1.f / p.max_spread;
  int st = ST_OK;
  float rel1, rel2 = 0.f;
  if (CONS) rel1 = 1.f - 2.f * sqrtf(s_all * inv_nrd);
  else rel1 = 1.f - fminf(p.max_spread, sqrtf(s_all * (1.f / (float)N))) * inv_ms;
  if (!(rel1 >= 0.f && rel1 <= 1.f)) st = ST_RELIABILITY_INTERVAL;
  else if (R < 2) st = R <= 0 ? ST_USIZE_UNDERFLOW : ST_INDEX_OOB;
  else {
    if (CONS) rel2 = 1.f - 2.f * sqrtf(s_rel * inv_rrd);
    else rel2 = 1.f - fminf(p.max_spread, sqrtf(s_rel * (1.f / (float)R))) * inv_ms;
    if (!(rel2 >= 0.f && rel2 <= 1.f)) st = ST_RELIABILITY_INTERVAL;
    else if (R < 4 && !p.legacy) st = ST_TOO_FEW_RELIABLE;
  }
  if (st != ST_OK) {  // revert: only the status is written (and the pass-1 c1 when the caller took it unstaged)
    if (live && g == 0) p.status[b] = st;
    return;           // uniform over the group
  }
  // ---- pass 2 (contract.cairo:476-500) from the words still in registers
  int first_rel = 0;
#pragma unroll
  for (int i = NR - 1; i >= 0; --i)
    if ((relbits >> i) & 1u) first_rel = i;
  uint32_t w0 = w[0];
#pragma unroll
  for (int i = 1; i < NR; ++i) w0 = first_rel == i ? w[i] : w0;
  const f32x2 sh = bf16x2_to_f32x2(w0);
  f32x2 s1 = {0.f, 0.f}, s2 = s1, s3 = s1, s4 = s1;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const uint32_t mk = 0u - ((relbits >> i) & 1u);
    const f32x2 y = fand2(bf16x2_to_f32x2(w[i]) - sh, mk);
    const f32x2 q = y * y;
    s1 += y;
    s2 += q;
    s3 = __builtin_elementwise_fma(q, y, s3);
    s4 = __builtin_elementwise_fma(q, q, s4);
  }
  float medA = 0.f, medB = 0.f;
  if (CONS) {
    // reliable rows keep their key; the first ceil((NR-R)/2) others (row order) become -inf
    const int lo2 = (NR - R + 1) >> 1;
    u16x2 r[NR];
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const bool rel = (relbits >> i) & 1u;
      const uint32_t sent = cnt < lo2 ? 0u : 0xffffffffu;
      r[i] = as_k(rel ? small_key<CONS>(w[i]) : sent);
      cnt += rel ? 0 : 1;
    }
    sort_oem<NR>(r);
    const uint32_t lo = key_to_pos(r[NR / 2 - 1]), hi = key_to_pos(r[NR / 2]);
    medA = 0.5f * (bf16_lo(lo) + bf16_lo(hi));
    medB = 0.5f * (bf16_hi(lo) + bf16_hi(hi));
  }
  // ---- moments (math.cairo:208-222, 320-398) from the shifted power sums
  const float n = (float)R, inv_n = 1.f / n;
  const float k3 = n / ((n - 1.f) * (n - 2.f));
  const float k4a = n * (n + 1.f) / (n - 1.f), k4b = 3.f * (n - 1.f) * (n - 1.f), ik4c = 1.f / ((n - 2.f) * (n - 3.f));
  int zv = 0;
  float cons_o[2], sk_o[2], ku_o[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const bool v = h ? vB : vA;
    const float a1 = h ? s1.y : s1.x, a2 = h ? s2.y : s2.x, a3 = h ? s3.y : s3.x, a4 = h ? s4.y : s4.x;
    const float shh = h ? sh.y : sh.x, med = h ? medB : medA;
    const float dl = a1 * inv_n, e2 = a2 * inv_n, e3 = a3 * inv_n, e4 = a4 * inv_n;
    const float mu2 = e2 - dl * dl;
    const float mu3 = e3 - 3.f * dl * e2 + 2.f * dl * dl * dl;
    const float mu4 = e4 - 4.f * dl * e3 + 6.f * dl * dl * e2 - 3.f * dl * dl * dl * dl;
    float sk = 0.f, ku = 0.f;
    if (mu2 > 0.f) {
      const float sd = sqrtf(mu2);
      const float z3 = n * mu3 * __builtin_amdgcn_rcpf(mu2 * sd), z4 = n * mu4 * __builtin_amdgcn_rcpf(mu2 * mu2);
      sk = z3 * k3;
      ku = (z4 * k4a - k4b) * ik4c;
    } else if (v) {
      zv = 1;
    }
    cons_o[h] = CONS ? med : shh + dl;
    sk_o[h] = p.legacy ? 0.f : sk;
    ku_o[h] = p.legacy ? 0.f : ku;
  }
  zv = group_or<G>(zv);
  if (!live) return;
  if (zv && !p.legacy) {   // revert: no output is written (contract.cairo:588-603)
    if (g == 0) p.status[b] = ST_ZERO_VARIANCE;
    return;
  }
  // ---- commit: the whole round succeeded
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (!(h ? vB : vA)) continue;
    const int64_t o = b * D + colA + h;
    p.consensus[o] = cons_o[h];
    p.skew[o] = sk_o[h];
    p.kurt[o] = ku_o[h];
    if (p.c1_out) p.c1_out[o] = h ? cB : cA;
  }
#pragma unroll
  for (int i = 0; i < NR; ++i)  // constant register indices only (a runtime index spills to scratch)
    if (i < N && i % G == g) {
      p.reliable[b * N + i] = (relbits >> i) & 1u;
      p.qr[b * N + i] = qr[i];
    }
  if (g == 0) {
    p.rel[2 * b] = rel1;
    p.rel[2 * b + 1] = rel2;
    p.status[b] = ST_OK;
  }
}

template <int NR, int G>
static int launch_small_g(const FastParams& p, hipStream_t stream) {
  constexpr int IPB = 4 * (64 / G);  // instances per 256-thread workgroup
  const int64_t blocks = ((int64_t)p.B + IPB - 1) / IPB;
  if (blocks > 0x7fffffff) return -1;
  auto k = p.constrained ? consensus_fast_small_kernel<NR, G, true> : consensus_fast_small_kernel<NR, G, false>;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}

template <int NR>
static int launch_small(const FastParams& p, hipStream_t stream) {
  const int pairs = (p.D + 1) / 2;
  if (pairs <= 1) return launch_small_g<NR, 1>(p, stream);
  if (pairs <= 2) return launch_small_g<NR, 2>(p, stream);
  if (pairs <= 4) return launch_small_g<NR, 4>(p, stream);
  if (pairs <= 8) return launch_small_g<NR, 8>(p, stream);
  if (pairs <= 16) return launch_small_g<NR, 16>(p, stream);
  if (pairs <= 32) return launch_small_g<NR, 32>(p, stream);
  return launch_small_g<NR, 64>(p, stream);
}

}  // namespace svoc

using namespace svoc;

// Eligible: full round (mode 0), 2 <= N <= 16, D <= 128.
extern "C" int svoc_fast_round_bf16_small(const FastParams* p, hipStream_t stream) {
  if (p->B <= 0) return 0;
  if (p->mode != 0 || p->N < 2 || p->N > 16 || p->D < 1 || p->D > 128 || p->ld % 8 != 0 || p->D > p->ld)
    return -1;
  return p->N <= 8 ? launch_small<8>(*p, stream) : launch_small<16>(*p, stream);
}
