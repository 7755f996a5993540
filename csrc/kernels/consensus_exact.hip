// Bit-exact (wsad, i128 arithmetic) consensus round on the GPU: one group of GS lanes per instance
// (a whole wave, or 8/16/32 lanes so small instances share a wave), lane = oracle row (RPL rows per
// lane for N > 64), loops over columns.  Every integer operation is the same
// csrc/include/svoc/wsad.hpp routine the CPU golden engine uses, evaluated in the same stage order
// (all c1, qr, rel1, rank mask, all consensus, rel2, all means, all variances, all skewness, all
// kurtosis -- contract/src/contract.cairo:451-500), so the outputs and the first-error status match
// csrc/engine/reference_cpu.cpp bit for bit.  Per-column intermediates live in LDS; outputs are
// only written when the whole round succeeds (transaction-revert semantics).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svoc/launch.hpp"
#include "svoc/status.hpp"
#include "svoc/wsad.hpp"

namespace svoc {

// loops over a lane's rows: unrolled (arrays in VGPRs) up to 16 rows per lane (N <= 1024); the 32 / 64
// rows-per-lane instantiations for N <= 4096 keep them in private memory and loop
#pragma clang diagnostic ignored "-Wcuda-compat"   // (a parenthesised, template-dependent unroll count)
#define SVOC_UNROLL_RPL _Pragma("unroll (RPL <= 16 ? RPL : 1)")

__device__ __forceinline__ int64_t shfl64(int64_t v, int src) {
  const int lo = __shfl((int)(uint32_t)v, src), hi = __shfl((int)(uint32_t)(v >> 32), src);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ i128 shfl128(i128 v, int src) {
  const u128 u = (u128)v;
  const uint64_t lo = (uint64_t)shfl64((int64_t)(uint64_t)u, src);
  const uint64_t hi = (uint64_t)shfl64((int64_t)(uint64_t)(u >> 64), src);
  return (i128)(((u128)hi << 64) | lo);
}

// A group of GS lanes = one instance (GS = 64: one instance per wave; GS = 8/16/32: 64/GS instances
// share a wave).  One wave per workgroup, so __syncthreads never waits on another wave and groups
// may leave the column loops at different iterations.
template <int GS>
struct Grp {
  int lane, gl, base;
  uint64_t mask;
  __device__ Grp() {
    lane = threadIdx.x;
    gl = lane % GS;
    base = lane - gl;
    mask = GS == 64 ? ~0ull : (((1ull << GS) - 1ull) << base);
  }
  __device__ bool all(bool v) const { return (__ballot(!v) & mask) == 0; }
  __device__ int count(bool v) const { return __popcll(__ballot(v) & mask); }
  __device__ int any_or(int v) const {
#pragma unroll
    for (int o = GS / 2; o >= 1; o >>= 1) v |= __shfl_xor(v, o);
    return v;
  }
  // s + the group's values in lane (= row) order, checked as the contract's running sum: it adds in row
  // order and reverts on any i128 overflow of a partial sum.  With |s| < 2^126 and every term below
  // 2^120 in magnitude no partial sum of the <= 64 terms can overflow in ANY order, so a butterfly gives
  // the identical integer; otherwise the terms are added one by one onto s, as the CPU engine does.
  // (Summing each group from 0 and adding the group total to s would miss an overflow of a partial
  // sum inside a group once s is large -- possible with several rows per lane.)
  __device__ i128 accum(i128 s, i128 v, int& st) const {
    const i128 lim = (i128)1 << 120, slim = (i128)1 << 126;
    if (s < slim && s > -slim && all(v < lim && v > -lim)) {
#pragma unroll
      for (int o = GS / 2; o >= 1; o >>= 1) v += shfl128(v, lane ^ o);
      return s + v;
    }
    i128 acc = s;
    for (int l = 0; l < GS; ++l) acc = add(acc, shfl128(v, base + l), st);
    return acc;
  }
};

template <int RPL>
struct Rows {
  int64_t x[RPL];
  bool on[RPL];  // row exists and takes part
};

// Column scratch in LDS (one per group): the group's rows are published once, then every lane ranks
// its own rows against them with broadcast LDS reads, both middle ranks in the same pass.
template <int NR>
struct ColScratch {
  int64_t x[NR];
  uint8_t on[NR];
  int64_t pick[2];
};

// stable ranks mid-1 and mid among the rows with on[] set (math.cairo:113-126 via MergeSort)
template <int RPL, int GS>
__device__ void middle_values(const Rows<RPL>& r, const Grp<GS>& g, int n_rows, int mid, ColScratch<RPL * GS>& cs,
                              i128& a, i128& b) {
SVOC_UNROLL_RPL
  for (int j = 0; j < RPL; ++j) {
    const int row = j * GS + g.gl;
    if (row < n_rows) {
      cs.x[row] = r.x[j];
      cs.on[row] = r.on[j] ? 1 : 0;
    }
  }
  __syncthreads();
SVOC_UNROLL_RPL
  for (int j = 0; j < RPL; ++j) {
    const int me = j * GS + g.gl;
    if (me < n_rows && r.on[j]) {
      const int64_t xm = r.x[j];
      int rank = 0;
#pragma unroll 8   // (several broadcast LDS reads in flight: one wave per SIMD at large N)
      for (int k = 0; k < n_rows; ++k) {
        const int64_t xk = cs.x[k];
        rank += (cs.on[k] && (xk < xm || (xk == xm && k < me))) ? 1 : 0;
      }
      if (rank == mid - 1) cs.pick[0] = xm;
      if (rank == mid) cs.pick[1] = xm;
    }
  }
  __syncthreads();
  a = cs.pick[0];
  b = cs.pick[1];
  __syncthreads();  // the scratch is reused by the next column
}

// N > 256 (8+ rows per lane, a whole wave per instance): ranking every row against the column costs
// N^2 / 64 LDS reads per lane; instead the k-th smallest (0-based) value of the on-rows comes from an
// 8-bit radix select over the order-preserving unsigned image of the int64 keys (a 256-bin LDS
// histogram per byte, the bin holding rank k found by a wave prefix scan).  Tied keys are equal
// values, so the picked value is the stable sort's value at that rank.
constexpr int kRadixRpl = 8;
// per-column int64 workspace slots: c1, consensus, mean, variance (two for int64 values), skew, kurt
__host__ __device__ constexpr int ws_cols(bool v128) { return v128 ? kExactWsCols : kExactWsCols - 1; }
template <int RPL>
__device__ int64_t radix_select(const Rows<RPL>& r, int lane, int k, uint32_t* hist) {
  uint64_t prefix = 0, pmask = 0;
#pragma unroll 1
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int t = lane; t < 256; t += 64) hist[t] = 0u;
    __syncthreads();
SVOC_UNROLL_RPL
    for (int j = 0; j < RPL; ++j) {
      const uint64_t u = (uint64_t)r.x[j] ^ 0x8000000000000000ull;
      if (r.on[j] && (u & pmask) == prefix) atomicAdd(&hist[(uint32_t)(u >> shift) & 255u], 1u);
    }
    __syncthreads();
    const uint32_t c = hist[4 * lane] + hist[4 * lane + 1] + hist[4 * lane + 2] + hist[4 * lane + 3];
    int incl = (int)c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    const int L = __builtin_ctzll(__ballot(incl > k));   // exists: k < the number of on-rows
    int below = __shfl(incl, L) - __shfl((int)c, L);
    int bin = 4 * L;
    for (int hb = (int)hist[bin]; below + hb <= k; hb = (int)hist[bin]) { below += hb; ++bin; }
    k -= below;
    prefix |= (uint64_t)bin << shift;
    pmask |= 0xffull << shift;
    __syncthreads();   // every lane's reads done before the next byte clears the histogram
  }
  return (int64_t)(prefix ^ 0x8000000000000000ull);
}

template <int RPL, int GS, int NR>
__device__ i128 smooth_median_w(const Rows<RPL>& r, const Grp<GS>& g, int n_rows, int count,
                                ColScratch<NR>& cs, uint32_t* hist, int& st) {
  if (count == 0) { fail(st, ST_USIZE_UNDERFLOW); return 0; }
  if (count == 1) { fail(st, ST_INDEX_OOB); return 0; }
  i128 a, b;
  if constexpr (RPL >= kRadixRpl) {
    static_assert(GS == 64, "radix select: one wave per instance");
    a = radix_select<RPL>(r, g.gl, count / 2 - 1, hist);
    b = radix_select<RPL>(r, g.gl, count / 2, hist);
  } else {
    middle_values<RPL, GS>(r, g, n_rows, count / 2, cs, a, b);
  }
  return idiv_pos64(add(a, b, st), 2, st);
}

template <int RPL, int GS, class T>
__global__ __launch_bounds__(64) void consensus_exact_kernel(ExactParams p) {
  constexpr int IPW = 64 / GS;  // instances per wave (= per workgroup)
  extern __shared__ __attribute__((aligned(16))) int64_t lds[];
  constexpr bool RADIX = RPL >= kRadixRpl;
  __shared__ ColScratch<RADIX ? 1 : RPL * GS> css[IPW];
  __shared__ __attribute__((aligned(16))) uint32_t hist[RADIX ? 256 : 1];
  const Grp<GS> g;
  const int gi = threadIdx.x / GS;
  const int b = blockIdx.x * IPW + gi;
  if (b >= p.B || (p.active && !p.active[b])) return;
  const int gl = g.gl;
  auto& cs = css[gi];
  const int N = p.N, D = p.D;
  // per-column intermediates: LDS, or a [B, kExactWsCols, D] global workspace when they exceed the LDS
  // (int64 values: the variance can pass 2^63 and takes two slots; int32 values: one)
  constexpr bool V128 = sizeof(T) == 8;
  constexpr int WSC = ws_cols(V128);
  int64_t* const ws = p.work ? p.work + (int64_t)b * kExactWsCols * D : lds + (int64_t)gi * WSC * D;
  int64_t* c1 = ws;
  int64_t* cons = ws + D;
  int64_t* means = ws + 2 * D;
  int64_t* vars = ws + 3 * D;   // V128: (lo, hi) per column
  int64_t* sk = ws + (WSC - 2) * D;
  int64_t* ku = ws + (WSC - 1) * D;
  const T* X = (const T*)p.values + (int64_t)b * N * D;
  int st = ST_OK;  // group-uniform by construction (every lane runs the same checked reductions)

  Rows<RPL> rows;
  i128 qr[RPL];
  if (p.mode == 2) {
    // D-sharded second half: this shard's c1 and the all-reduced qr come in; a shard whose first half
    // failed has already set the (all-reduced) status
    if (p.status[b] != ST_OK) return;
    for (int d = gl; d < D; d += GS) c1[d] = p.c1[(int64_t)b * D + d];
SVOC_UNROLL_RPL
    for (int j = 0; j < RPL; ++j) {
      const int row = j * GS + gl;
      qr[j] = row < N ? (i128)p.qr[(int64_t)b * N + row] : 0;
    }
    __syncthreads();
  } else {
    // ---- pass 1: c1 per column
    for (int d = 0; d < D && st == ST_OK; ++d) {
SVOC_UNROLL_RPL
      for (int j = 0; j < RPL; ++j) {
        const int row = j * GS + gl;
        rows.on[j] = row < N;
        rows.x[j] = row < N ? X[(int64_t)row * D + d] : 0;
      }
      const i128 c = smooth_median_w<RPL, GS>(rows, g, N, N, cs, hist, st);
      if (gl == 0) c1[d] = (int64_t)c;
    }
    __syncthreads();
    if (st != ST_OK) { if (gl == 0) p.status[b] = st; return; }
    // quadratic risk per row (lane-local), then the checked mean
    int lst = ST_OK;
SVOC_UNROLL_RPL
    for (int j = 0; j < RPL; ++j) {
      const int row = j * GS + gl;
      i128 acc = 0;
      if (row < N)
        for (int d = 0; d < D; ++d) acc = add(acc, qdev(X[(int64_t)row * D + d], c1[d], lst), lst);
      qr[j] = acc;
    }
    // any lane's overflow reverts (qr can only fail with OVERFLOW)
    if (g.any_or(lst != ST_OK)) st = ST_OVERFLOW;
    if (p.mode == 1) {   // D-sharded first half: c1 and the qr partials out, nothing else
      bool big = false;
SVOC_UNROLL_RPL
      for (int j = 0; j < RPL; ++j) big = big || qr[j] >= (i128)kExactQrPartialMax || qr[j] <= -(i128)kExactQrPartialMax;
      if (g.any_or(big)) st = ST_OVERFLOW;
      if (st == ST_OK) {
        for (int d = gl; d < D; d += GS) p.c1[(int64_t)b * D + d] = c1[d];
SVOC_UNROLL_RPL
        for (int j = 0; j < RPL; ++j) {
          const int row = j * GS + gl;
          if (row < N) p.qr[(int64_t)b * N + row] = (int64_t)qr[j];
        }
      }
      if (gl == 0) p.status[b] = st;
      return;
    }
  }
  i128 sum_qr = 0;
SVOC_UNROLL_RPL
  for (int j = 0; j < RPL; ++j) sum_qr = g.accum(sum_qr, qr[j], st);
  const i128 mean_qr = idiv(sum_qr, (i128)N, st);
  // obsolete contracts: no /D (contract_nd.cairo:418); D-sharded rounds: the global D
  const int64_t rdim = p.legacy ? 1 : (p.rel_dim > 0 ? p.rel_dim : D);
  const i128 rel1 = p.constrained ? constrained_reliability(mean_qr, rdim, st)
                                  : unconstrained_reliability(wsqrt(mean_qr, st), p.max_spread, st);
  if (st == ST_OK && !in_unit_interval(rel1)) st = ST_RELIABILITY_INTERVAL;
  if (st == ST_OK && p.n_failing > N) st = ST_USIZE_UNDERFLOW;
  if (st != ST_OK) { if (gl == 0) p.status[b] = st; return; }
  // rank mask: (qr asc, idx desc) (sort.cairo:96-101)
  const int threshold = N - p.n_failing;
  bool rel[RPL];
SVOC_UNROLL_RPL
  for (int j = 0; j < RPL; ++j) {
    const int me = j * GS + gl;
    int rank = 0;
SVOC_UNROLL_RPL
    for (int jj = 0; jj < RPL; ++jj)
      for (int l = 0; l < GS; ++l) {
        const int k = jj * GS + l;
        const i128 qk = shfl128(qr[jj], g.base + l);
        if (k < N) rank += (qk < qr[j] || (qk == qr[j] && k > me)) ? 1 : 0;
      }
    rel[j] = me < N && rank < threshold;
  }
  int R = 0;
SVOC_UNROLL_RPL
  for (int j = 0; j < RPL; ++j) R += g.count(rel[j]);
  // ---- pass 2: consensus per column over the reliable rows
  for (int d = 0; d < D && st == ST_OK; ++d) {
SVOC_UNROLL_RPL
    for (int j = 0; j < RPL; ++j) {
      const int row = j * GS + gl;
      rows.on[j] = rel[j];
      rows.x[j] = row < N ? X[(int64_t)row * D + d] : 0;
    }
    i128 c;
    if (p.constrained) {
      c = smooth_median_w<RPL, GS>(rows, g, N, R, cs, hist, st);
    } else {
      i128 s = 0;
SVOC_UNROLL_RPL
      for (int j = 0; j < RPL; ++j) s = g.accum(s, rows.on[j] ? (i128)rows.x[j] : 0, st);
      c = idiv(s, (i128)R, st);
    }
    if (gl == 0) cons[d] = (int64_t)c;
  }
  i128 s2 = 0;
SVOC_UNROLL_RPL
  for (int j = 0; j < RPL; ++j) s2 = g.accum(s2, rel[j] ? qr[j] : 0, st);
  const i128 mean_qr2 = idiv(s2, (i128)R, st);
  const i128 rel2 = p.constrained ? constrained_reliability(mean_qr2, rdim, st)
                                  : unconstrained_reliability(wsqrt(mean_qr2, st), p.max_spread, st);
  if (st == ST_OK && !in_unit_interval(rel2)) st = ST_RELIABILITY_INTERVAL;
  if (p.legacy) {  // obsolete contracts store no moments
    for (int d = gl; d < D; d += GS) sk[d] = ku[d] = 0;
  }
  // ---- moments (math.cairo:208-222, 320-398), stage by stage like the CPU engine
  for (int d = 0; d < D && st == ST_OK && !p.legacy; ++d) {
    i128 s = 0;
SVOC_UNROLL_RPL
    for (int j = 0; j < RPL; ++j) {
      const int row = j * GS + gl;
      s = g.accum(s, rel[j] ? (i128)X[(int64_t)row * D + d] : 0, st);
    }
    const i128 mu = idiv(s, (i128)R, st);
    if (gl == 0) means[d] = (int64_t)mu;
  }
  __syncthreads();
  for (int d = 0; d < D && st == ST_OK && !p.legacy; ++d) {
    i128 s = 0;
    int l2 = ST_OK;
SVOC_UNROLL_RPL
    for (int j = 0; j < RPL; ++j) {
      const int row = j * GS + gl;
      const i128 q = rel[j] ? qdev(X[(int64_t)row * D + d], means[d], l2) : 0;
      if (g.any_or(l2 != ST_OK)) fail(st, ST_OVERFLOW);
      s = g.accum(s, q, st);
    }
    const i128 v = idiv(s, (i128)R, st);
    if (gl == 0) {
      if constexpr (V128) {
        vars[2 * d] = (int64_t)(uint64_t)(u128)v;
        vars[2 * d + 1] = (int64_t)(v >> 64);
      } else {
        vars[d] = (int64_t)v;
      }
    }
  }
  __syncthreads();
  for (int pass = 0; pass < 2 && !p.legacy; ++pass) {  // 0: skewness for all d, 1: kurtosis for all d
    for (int d = 0; d < D && st == ST_OK; ++d) {
      const i128 var = V128 ? (i128)(((u128)(uint64_t)vars[2 * d + 1] << 64) | (uint64_t)vars[2 * d]) : (i128)vars[d];
      const i128 sd = wsqrt(var, st);
      i128 s = 0;
      int l2 = ST_OK;
SVOC_UNROLL_RPL
      for (int j = 0; j < RPL; ++j) {
        const int row = j * GS + gl;
        i128 t = 0;
        if (rel[j] && st == ST_OK) {
          const i128 z = wdiv(sub(X[(int64_t)row * D + d], means[d], l2), sd, l2);
          const i128 z2 = wmul(z, z, l2);
          t = pass == 0 ? wmul(z2, z, l2) : wmul(z2, z2, l2);
        }
        // first error in row order, as the CPU loop: smallest failing row's code wins
        for (int l = 0; l < GS; ++l) {
          const int c = __shfl(l2, g.base + l);
          if (c != ST_OK) { fail(st, c); break; }
        }
        s = g.accum(s, t, st);
      }
      const i128 out = pass == 0 ? skew_from_sum(s, R, st) : kurt_from_sum(s, R, st);
      if (gl == 0) (pass == 0 ? sk : ku)[d] = (int64_t)out;
    }
  }
  __syncthreads();
  if (st != ST_OK) { if (gl == 0) p.status[b] = st; return; }
  // ---- commit
  for (int d = gl; d < D; d += GS) {
    const int64_t o = (int64_t)b * D + d;
    p.consensus[o] = cons[d];
    p.skew[o] = sk[d];
    p.kurt[o] = ku[d];
    if (p.c1) p.c1[o] = c1[d];
  }
SVOC_UNROLL_RPL
  for (int j = 0; j < RPL; ++j) {
    const int row = j * GS + gl;
    if (row < N) {
      p.reliable[(int64_t)b * N + row] = rel[j] ? 1 : 0;
      p.qr[(int64_t)b * N + row] = (int64_t)qr[j];
    }
  }
  if (gl == 0) {
    p.rel[2 * (int64_t)b] = (int64_t)rel1;
    p.rel[2 * (int64_t)b + 1] = (int64_t)rel2;
    p.status[b] = ST_OK;
  }
}

template <int RPL, int GS>
static int launch_exact(const ExactParams& p, hipStream_t stream) {
  constexpr int IPW = 64 / GS;
  const size_t lds = p.work ? 0 : (size_t)IPW * p.D * ws_cols(!p.val32) * sizeof(int64_t);
  if (lds > 64 * 1024) return -2;  // the binding passes a global workspace for wide instances
  auto k = p.val32 ? consensus_exact_kernel<RPL, GS, int32_t> : consensus_exact_kernel<RPL, GS, int64_t>;
  hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k, dim3((unsigned)((p.B + IPW - 1) / IPW)), dim3(64), lds, stream, p);
  return (int)hipGetLastError();
}

}  // namespace svoc

using namespace svoc;

extern "C" int svoc_exact_round_wsad(const ExactParams* p, hipStream_t stream);
extern "C" int svoc_exact_round_wsadx(const ExactParams* p, hipStream_t stream);

// i128 kernel over every active instance (the reference-order path; any status).  Lane group per
// instance: the smallest of 8 / 16 / 32 lanes holding one row each (several instances per wave, e.g.
// the deployed 7 x 6 config runs 8 per wave), else a full wave with 1 or 4 rows per lane.  Wide
// instances (6*D int64 > LDS budget) use the HBM workspace and a full wave.
static int exact_round_i128(const ExactParams* p, hipStream_t stream) {
  const size_t per_inst = (size_t)p->D * ws_cols(!p->val32) * sizeof(int64_t);
  if (!p->work) {
    if (p->N <= 8 && 8 * per_inst <= 64 * 1024) return launch_exact<1, 8>(*p, stream);
    if (p->N <= 16 && 4 * per_inst <= 64 * 1024) return launch_exact<1, 16>(*p, stream);
    if (p->N <= 32 && 2 * per_inst <= 64 * 1024) return launch_exact<1, 32>(*p, stream);
  }
  if (p->N <= 64) return launch_exact<1, 64>(*p, stream);
  if (p->N <= 256) return launch_exact<4, 64>(*p, stream);
  if (p->N <= 512) return launch_exact<8, 64>(*p, stream);
  if (p->N <= 1024) return launch_exact<16, 64>(*p, stream);
  if (p->N <= 2048) return launch_exact<32, 64>(*p, stream);
  return launch_exact<64, 64>(*p, stream);
}

// Exact round: the column-parallel kernel (consensus_wsad.hip) takes every instance it can prove
// bit-exact in fp64 / int64 arithmetic (constrained or obsolete-contract rounds, values in [0, 1e6], a
// successful round); the others -- any revert, out-of-domain values, unconstrained rounds -- are
// flagged and run through the i128 kernel right after it on the same stream.
extern "C" int svoc_exact_round(const ExactParams* p, hipStream_t stream) {
  if (p->B <= 0) return 0;
  if (p->N < 1 || p->N > kExactMaxN || p->D < 1) return -1;
  if (p->stage && p->fallback) {
    const int rc = svoc_exact_round_wsad(p, stream);
    if (rc != -2) {
      if (rc != 0 || p->skip_fallback) return rc;
      // flagged unconstrained rounds over wide columns: the int64 column kernel first (it clears the flags of
      // the rounds it commits; consensus_wsadx.hip), the i128 kernel for the rest
      const int rx = svoc_exact_round_wsadx(p, stream);
      if (rx != 0 && rx != -2) return rx;
      ExactParams q = *p;
      q.active = p->fallback;
      return exact_round_i128(&q, stream);
    }
  }
  return exact_round_i128(p, stream);
}
