// Column-parallel exact (wsad) consensus round: bit-identical to the i128 kernel (consensus_exact.hip)
// and to the CPU golden engine (csrc/engine/reference_cpu.cpp) on every round it accepts.
//
// Semantics: contract/src/contract.cairo:442-503 (constrained) in the exact integer arithmetic of
// signed_decimal.cairo:52-116 and math.cairo:113-398 (smooth median, quadratic risk, reliability,
// rank mask, mean, variance, sqrt, skewness, kurtosis; Appendix A.2 of SURVEY.md).  Accepted:
// constrained rounds (the obsolete N-D contract's too: no moments, reliability without /D) over values
// in [0, 1e6] (the interval the contract enforces on every update, contract.cairo:591-593) that
// succeed, reliable outliers included (their z-power products are summed in int64), and the reverting
// ones: the kernel reports the reference's stage-ordered status (reliability interval after each pass,
// usize underflow / index OOB for R < 2, too few reliable, division by zero of a zero-variance column)
// and writes nothing else.  Out-of-domain values and unconstrained rounds are flagged in p.fallback
// and recomputed right after by the i128 kernel.
//
// Why it is fast: the i128 kernel gives each instance one wave and loops over the columns with a
// group reduction per column per statistic (5 GB/s at 64 x 1024).  Here a lane owns a COLUMN (NSEG
// lanes of 64 rows each for N > 64: the fast kernels' lane-group layout, one 32-bit key per lane
// instead of a bf16 pair), every per-column statistic is lane-local, and the integer arithmetic runs
// in fp64 on integral values (wsad_fast.hpp: exact under bounds the constrained domain guarantees):
//   pass 1: smooth median per column (median_group on u32 keys with the sentinel split), the
//           column's quadratic deviations qdev(x, c1), summed over the wave's columns by a
//           transposing butterfly -> per-oracle qr (u64, exact) in LDS;
//   rank mask (qr asc, idx desc; sort.cairo:96-101), rel1 / rel2 by the wsad.hpp routines;
//   pass 2: smooth median of the reliable rows (the others become sentinels), then from the same
//           registers: mean, variance, wsqrt, z = wsad_div(x - mean, sd), wsad_mul powers ->
//           skewness / kurtosis.  Per-column results are staged in p.stage and copied to the outputs
//           only after every column passed its checks: a flagged instance leaves them untouched.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "svoc/bufload.hpp"
#include "svoc/launch.hpp"
#include "svoc/sortnet.hpp"
#include "svoc/status.hpp"
#include "svoc/wsad.hpp"
#include "svoc/wsad_fast.hpp"

#ifndef SVOC_WSAD_BATCH_QR
#define SVOC_WSAD_BATCH_QR 1   // N <= 64 too: batched qr / mean re-reads (226 VGPRs, c2 exact +27%)
#endif

namespace svoc {

constexpr uint32_t kWsadMax = 1000000u;
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// The lane's column value in row `soff` (bytes): int32, or the low word of an int64 (`hiw` gets its
// high word, which must be 0 for a value in [0, 1e6]).
template <bool V32>
SVOC_DEV uint32_t wload(__amdgpu_buffer_rsrc_t rs, int voff, int soff, uint32_t& hiw) {
  if constexpr (V32) {
    hiw = 0;
    return bload(rs, voff, soff);
  } else {
    const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
    hiw = v[1];
    return v[0];
  }
}

// Low 32-bit words of the lane's 64 rows of one column (int32 values, or the low word of int64 values
// whose high words pass 1 / the first pass-2 read validated), every load issued before any is
// consumed.  Written inline, each re-read loop waited on its load before issuing the next (one load in
// flight); the opaque stride keeps the 64 row soffsets from being hoisted into live SGPRs.
SVOC_DEV void load_lo(__amdgpu_buffer_rsrc_t rs, int vo, int rowb, uint32_t (&x)[64]) {
  asm volatile("" : "+s"(rowb));
#pragma unroll
  for (int i = 0; i < 64; ++i) x[i] = bload(rs, vo, i * rowb);
  __builtin_amdgcn_sched_barrier(0);
}
// The re-read offset made to depend on v (empty asm, as the window kernel's vo2): the loads cannot be
// issued before v exists.  Without it LLVM hoists every re-read above the sort network (nothing else
// orders them) and holds 256 loaded words at once.
template <class T>
SVOC_DEV int after(int vo, T v) {
  asm volatile("" : "+v"(vo) : "v"(v));
  return vo;
}

// Transposing butterfly over the wave's P columns (the fast kernels' qr tree, exact u32 sums):
// stage L exchanges with lane ^ (P >> L); the lane ends with rows I + base(lane) of all P columns.
template <int L, int I, int P>
SVOC_DEV uint32_t qtree(const uint32_t (&q)[64], int lane) {
  if constexpr (L == 0) {
    return q[I];
  } else {
    constexpr int msk = P >> L;
    const uint32_t lo_v = qtree<L - 1, I, P>(q, lane);
    const uint32_t hi_v = qtree<L - 1, I + (64 >> L), P>(q, lane);
    const bool up = (lane & msk) != 0;
    const uint32_t send = up ? lo_v : hi_v;
    const uint32_t keep = up ? hi_v : lo_v;
    return keep + xor_lane_u32<msk>(send);
  }
}
template <int P, int... Is>
SVOC_DEV void qtree_all(const uint32_t (&q)[64], int lane, uint64_t* acc, std::integer_sequence<int, Is...>) {
  ((acc[Is] += qtree<__builtin_ctz(P), Is, P>(q, lane)), ...);
}

// the same butterfly for the high words of 43-bit terms (unconstrained wide deviations): acc += sum << 32
template <int P, int... Is>
SVOC_DEV void qtree_hi_all(const uint32_t (&q)[64], int lane, uint64_t* acc, std::integer_sequence<int, Is...>) {
  ((acc[Is] += (uint64_t)qtree<__builtin_ctz(P), Is, P>(q, lane) << 32), ...);
}
// low / high 32-bit words of an integral double 0 <= q < 2^43
SVOC_DEV uint32_t q_hi(double q) { return (uint32_t)(q * 0x1p-32); }
SVOC_DEV uint32_t q_lo(double q) { return (uint32_t)(q - (double)q_hi(q) * 0x1p32); }
// |d| >= 2^25 for an int32 d (the narrow qdev forms' bound)
SVOC_DEV bool wide25(uint32_t d) { return d + (1u << 25) >= (1u << 26); }

// |x - c| < 2^25 for int32 x, c, in integer arithmetic (the unconstrained domain check; fp64 forms of it
// held the 64 rows' conversions live and cost ~120 VGPRs): both within 2^30 of 0, so x - c cannot wrap
SVOC_DEV bool near25(uint32_t x, uint32_t c) {
  const bool small = (x + (1u << 30)) < (1u << 31) && (c + (1u << 30)) < (1u << 31);
  return small && (x - c + ((1u << 25) - 1u)) < ((1u << 26) - 1u);
}

// The same butterfly with 64-bit partial sums (unconstrained: a deviation's qdev may reach 2^31)
template <int L, int I, int P>
SVOC_DEV uint64_t qtree64(const uint32_t (&q)[64], int lane) {
  if constexpr (L == 0) {
    return q[I];
  } else {
    constexpr int msk = P >> L;
    const uint64_t lo_v = qtree64<L - 1, I, P>(q, lane);
    const uint64_t hi_v = qtree64<L - 1, I + (64 >> L), P>(q, lane);
    const bool up = (lane & msk) != 0;
    const uint64_t send = up ? lo_v : hi_v;
    const uint64_t keep = up ? hi_v : lo_v;
    const uint32_t rlo = xor_lane_u32<msk>((uint32_t)send), rhi = xor_lane_u32<msk>((uint32_t)(send >> 32));
    return keep + (((uint64_t)rhi << 32) | rlo);
  }
}
template <int P, int... Is>
SVOC_DEV void qtree64_all(const uint32_t (&q)[64], int lane, uint64_t* acc, std::integer_sequence<int, Is...>) {
  ((acc[Is] += qtree64<__builtin_ctz(P), Is, P>(q, lane)), ...);
}

// Inclusive prefix sum of one value per thread over a 256-thread workgroup (wave scans + the wave totals);
// `wsum` is 4 words of LDS.  Every thread returns its inclusive prefix; `total` gets the sum.
SVOC_DEV uint32_t block_scan_256(uint32_t v, uint32_t* wsum, int tid, uint32_t& total) {
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = (uint32_t)__shfl_up((int)v, o);
    if (lane >= o) v += u;
  }
  if (lane == 63) wsum[wave] = v;
  __syncthreads();
  uint32_t before = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) before += w < wave ? wsum[w] : 0u;
  total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  return v + before;
}

// Rank mask for the wide lane groups (N up to 4096; sort.cairo:9-103 + contract.cairo:345-363): instead of
// ranking every row against every other (N^2 / 256 LDS reads per thread), T = the (R-1)-th smallest qr is found
// by an 8-pass radix select (one 256-bin LDS histogram per byte, thread = bin), rows below T are reliable and
// the rows AT T by index descending (the merge sort's tie rule) until R rows are.  Thread tid owns the
// contiguous rows [tid RPT, tid RPT + RPT).  256 threads.
template <int NPAD>
SVOC_DEV void rank_mask_select(const uint64_t* qr, int N, int R, uint64_t* relmask, uint32_t* hist, uint32_t* wsum,
                               uint32_t* sel, int tid) {
  constexpr int RPT = NPAD / 256;
  static_assert(RPT >= 1 && 64 % RPT == 0, "rows per thread within one mask word");
  for (int w = tid; w < NPAD / 64; w += 256) relmask[w] = 0ull;
  uint64_t prefix = 0ull, pmask = 0ull;
  uint32_t k = (uint32_t)(R - 1);   // target rank among the rows matching the prefix
  for (int byte = 7; byte >= 0; --byte) {
    hist[tid] = 0u;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int t = tid * RPT + i;
      if (t < N) {
        const uint64_t q = qr[t];
        if ((q & pmask) == prefix) atomicAdd(&hist[(uint32_t)(q >> (8 * byte)) & 255u], 1u);
      }
    }
    __syncthreads();
    const uint32_t c = hist[tid];
    uint32_t tot;
    const uint32_t incl = block_scan_256(c, wsum, tid, tot);
    if (incl - c <= k && k < incl) {   // this bin holds the target
      sel[0] = (uint32_t)tid;
      sel[1] = k - (incl - c);
    }
    __syncthreads();
    prefix |= (uint64_t)sel[0] << (8 * byte);
    pmask |= 0xffull << (8 * byte);
    k = sel[1];
    __syncthreads();
  }
  const uint64_t T = prefix;
  uint32_t lt = 0, ties = 0;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int t = tid * RPT + i;
    if (t < N) {
      const uint64_t q = qr[t];
      lt += q < T ? 1u : 0u;
      ties += q == T ? 1u : 0u;
    }
  }
  uint32_t lt_tot, tie_tot;
  (void)block_scan_256(lt, wsum, tid, lt_tot);
  const uint32_t tie_incl = block_scan_256(ties, wsum, tid, tie_tot);
  const uint32_t need = (uint32_t)R - lt_tot;              // tie rows taken, largest indices first
  uint32_t above = tie_tot - tie_incl;                     // tie rows after this thread's block
  uint64_t bits = 0ull;
#pragma unroll
  for (int i = RPT - 1; i >= 0; --i) {
    const int t = tid * RPT + i;
    if (t < N) {
      const uint64_t q = qr[t];
      bool rel = q < T;
      if (q == T) {
        rel = above < need;
        ++above;
      }
      if (rel) bits |= 1ull << ((tid * RPT + i) & 63);
    }
  }
  if (bits) atomicOr((unsigned long long*)&relmask[(tid * RPT) >> 6], (unsigned long long)bits);
  __syncthreads();
}

// bit i of m as an all-ones / zero word the compiler cannot see through: (x & mk) | (y & ~mk) stays one
// v_bfi_b32 and x & mk one v_and (a known sign-extended bit is canonicalised into a shift, a compare and a
// select per row: 5 VALU where 2 do)
SVOC_DEV uint32_t bit_mask_o(uint64_t m, int i) {
  uint32_t k = bit_mask(m, i);
  asm volatile("" : "+v"(k));
  return k;
}

// sum over the NSEG lanes of a column group (lanes lane ^ t*P)
template <int NSEG, int P, class T>
SVOC_DEV T group_sum(T v) {
#pragma unroll
  for (int t = 1; t < NSEG; t <<= 1) v += __shfl_xor(v, t * P);
  return v;
}

// MODE (launch.hpp ExactParams::mode): 0 whole round; 1 D-sharded first half (c1 + qr partials out);
// 2 D-sharded second half (c1 and the all-reduced qr in).  Instances it cannot take in mode 1 / 2 go
// to the i128 kernel's same mode through p.fallback, as in mode 0.
// CONS = false: unconstrained rounds (contract.cairo:370-434): signed int64 values, pass-2 consensus = the
// reliable mean (no second network), reliabilities W - wsad_div(min(ms, sqrt(mean qr)), ms).  Every column is
// taken relative to its row-0 value B (keys, deviations and z-scores are translation invariant; the two
// truncated quotients -- the smooth median and the mean -- are shifted back exactly by tdiv_rel, and c1 /
// consensus are committed as B + the relative value).  Domain (else the i128 kernel): |B| < 2^52 and every
// value within 2^30 of B (1,073 real units: price-like columns such as 60,000 +- 200 stay here; deviations
// then stay below 2^31, the wide forms' bound, and their 43-bit quotients' high words below 2^11).  Deviations
// below 2^25 take the fast half-offset forms; a wave with any larger one takes the wide forms (double-double
// qdev with 43-bit quotients summed as two 32-bit butterflies, the int64 Newton sqrt) for that slab.
// WINH > 0 (whole constrained rounds, launch_wsad_c): ONE median network per column.  Pass 1 keeps the
// 2 WINH keys around the median (window_group, sortnet.hpp) in the staging buffer; the pass-2 smooth
// median over the reliable rows is then read off that window by ranking the f removed rows' keys
// against it (one lane per column, f + 2 WINH loads):  with G the sorted column, U the sorted removed
// keys (u_f = +inf) and A = G \ U, the r-th smallest of A is  min over j in [0, f] of { g_{r+j} : g_{r+j} <
// u_j }  (multisets, ties included: with Q = #{U <= a_r}, g_{r+Q} = a_r and u_Q > a_r; any qualifying
// g_{r+j} has at least r + 1 elements of A at or below it).  Ranks R/2 - 1 and R/2 (math.cairo:113-126)
// need g at positions R/2 - 1 .. R/2 + f, inside the window when WINH >= max(a + 1, f - a + 1),
// a = N/2 - R/2.  The second network over the reliable rows (~30 % of the kernel's VALU) goes away.
template <int NSEG, int WAVES, bool V32, int MODE, bool CONS, int WINH = 0>
// (2 waves per SIMD where the kernel fits 256 VGPRs without scratch in its loops: the whole / first-half constrained
// rounds and the unconstrained int64 ones; the unconstrained int32 and D-sharded second-half instantiations spill
// a few hundred bytes at that cap and keep one wave with AGPR spill slots)
__global__ __launch_bounds__(WAVES * 64)
__attribute__((amdgpu_waves_per_eu(NSEG <= 4 && !(CONS && MODE == 2) ? 2 : 1)))
void consensus_wsad_kernel(ExactParams p) {
  static_assert(WINH == 0 || (MODE == 0 && CONS), "the window path is for whole constrained rounds");
  constexpr int P = 64 / NSEG;      // columns per wave
  constexpr int NPAD = 64 * NSEG;   // padded oracle rows
  constexpr int W = WAVES * P;      // columns per tile
  constexpr int NT = WAVES * 64;
  constexpr int KEEP = 64 / P;      // qr rows a lane holds after the butterfly
  // WIDE (NSEG 8 .. 64: N up to 512 .. 4096; whole rounds and the constrained D-sharded halves): full cross-lane median networks
  // (median_group_wide), the per-oracle qr summed by LDS atomics instead of the transposing butterfly (a lane
  // holds 64 rows of one column: the butterfly would leave it 64 / P row sums -- 128 VGPRs at P = 1), and
  // 64-bit / fp64 column sums (R values up to 1e6 pass 2^32)
  constexpr bool WIDE = NSEG > 4;
  static_assert(!WIDE || (WINH == 0 && (MODE == 0 || CONS)), "wide groups: two networks; D-sharded halves constrained");
  constexpr int MW = NSEG > 4 ? NSEG : 4;   // 64-bit row-mask words
  constexpr int ESZ = V32 ? 4 : 8;
  // re-reads issued as 64-load batches ordered after the value they need (load_lo / after): +37% at
  // 256 x 4096; the N <= 64 kernel batches the qr and mean re-reads only (+27% at 64 x 1024): batching
  // the fp64 variance / z-power re-reads too costs it a wave per SIMD (-18%)
  constexpr bool BATCH = NSEG >= 2;
  constexpr bool BATCH1 = BATCH || SVOC_WSAD_BATCH_QR;   // the qr and mean re-reads only (no fp64 temporaries)
  __shared__ uint64_t qr_part[WIDE ? 1 : WAVES * NPAD];
  // WIDE: the slab's W columns of every row staged in LDS by 16-byte row loads (a lane owns 64 rows of ONE column,
  // so a direct column load touches a cache line per element: 16x the bytes at D = 64), column-major with one
  // word of padding per 64 rows (row r at r + r / 64: a lane's 64 rows sit in distinct banks across the wave)
  // (TILE: 32 / 64 lanes per column, 1 / 2 columns per wave -- with 8 / 16 lanes per column a wave's direct load
  // still reads 32 / 16 contiguous bytes per row, and the tile's per-slab barriers cost more than they save:
  // 512 x 2048 ran 85 k rounds/s direct, 62 k through the tile)
  constexpr bool TILE = WIDE && NSEG >= 32;
  constexpr int TROW = NPAD + NPAD / 64;
  __shared__ uint32_t tile[TILE ? W * TROW : 1];
  __shared__ uint64_t qr_lds[NPAD];
  __shared__ uint64_t relmask[MW], lowmask[MW];
  __shared__ int64_t rels[2];
  __shared__ int flag;
  __shared__ int early_st;   // a revert decided before the moments (its final status)
  __shared__ int div0;       // a moment stage divides by zero (the round reverts with DIV_BY_ZERO)
  __shared__ int urow[WINH > 0 ? 2 * WINH : 1];   // window path: the removed rows, index order

  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if ((p.active && !p.active[b]) || (MODE == 2 && p.status[b] != ST_OK)) {   // mode 2: a shard failed
    if (tid == 0) p.fallback[b] = 0;
    return;
  }
  if (tid == 0) {
    // (unconstrained, D-sharded second half over int64 values: no pass 1 here to validate the high words)
    flag = (!CONS && MODE == 2 && !V32) ? 1 : 0;
    early_st = ST_OK;
    div0 = 0;
  }
  const int seg = lane / P, cw = lane % P;
  const int N = p.N, D = p.D;
  const int rowb = D * ESZ;
  const __amdgpu_buffer_rsrc_t rs =
      instance_rsrc((const unsigned char*)p.values + (int64_t)b * N * rowb, (uint32_t)(N * rowb));
  // [SROWS][D]: c1, consensus, skewness, kurtosis, then the window keys (WINH > 0) or the columns' base
  // values (unconstrained: low / high words)
  constexpr int SROWS = 4 + 2 * WINH + (CONS ? 0 : 2);
  int32_t* const stg = p.stage + (int64_t)b * SROWS * D;
  auto stage_base = [&](const int32_t* sg, int c) __attribute__((always_inline)) -> int64_t {
    if constexpr (CONS) return 0;
    else return (int64_t)(((uint64_t)(uint32_t)sg[5 * D + c] << 32) | (uint32_t)sg[4 * D + c]);
  };
  const int nslab = (D + W - 1) / W;
  const int lo1 = (NPAD - N + 1) >> 1;   // pass-1 sentinel split (rows >= N): -inf first, then +inf
  const int nv = N - seg * 64;           // this lane's rows < nv are real
  const int nl = N + lo1 - seg * 64;
  const int seg_off = seg * 64 * rowb;
  const uint32_t pol = group_polarity<NSEG>(seg);
  uint32_t badv = 0;                     // a value outside [0, 1e6]

  // WIDE: stage slab s (columns s W .. s W + W - 1, rows < N) into the tile; int64 values' high words must be 0
  auto load_tile = [&](int s) __attribute__((always_inline)) {
    __syncthreads();   // (the previous slab's readers are done)
    constexpr int VPR = W * ESZ / 16;   // 16-byte vectors per row
    const int c0 = s * W;
    for (int v = tid; v < N * VPR; v += NT) {
      const int row = v / VPR, part = v - row * VPR;
      const uint32_t off = (uint32_t)(row * rowb + c0 * ESZ + part * 16);
      const uint4 w = (c0 * ESZ + part * 16 < D * ESZ) ? __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0))
                                                        : make_uint4(0u, 0u, 0u, 0u);
      const int pr = row + (row >> 6);
      if constexpr (V32) {
        tile[(part * 4 + 0) * TROW + pr] = w.x;
        tile[(part * 4 + 1) * TROW + pr] = w.y;
        tile[(part * 4 + 2) * TROW + pr] = w.z;
        tile[(part * 4 + 3) * TROW + pr] = w.w;
      } else {
        tile[(part * 2 + 0) * TROW + pr] = w.x;
        tile[(part * 2 + 1) * TROW + pr] = w.z;
        const int c = c0 + part * 2;
        if constexpr (CONS) {
          badv |= ((c < D && w.y != 0u) || (c + 1 < D && w.w != 0u)) ? 1u : 0u;   // constrained: [0, 1e6]
        } else {
          // unconstrained: the high words are checked here, against the columns' row-0 values (the base B;
          // the same vector of row 0, an L1 hit): x - B must be the sign extension of its low word and
          // within [-2^30, 2^30) -- the tile then holds everything the round reads
          const uint4 b0 = (c0 * ESZ + part * 16 < D * ESZ)
                               ? __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, c0 * ESZ + part * 16, 0, 0))
                               : make_uint4(0u, 0u, 0u, 0u);
          auto bad64 = [](uint32_t l, uint32_t h, uint32_t bl, uint32_t bh) __attribute__((always_inline)) {
            const uint32_t rl = l - bl, rh = h - bh - (l < bl ? 1u : 0u);
            return !(rh == (uint32_t)((int32_t)rl >> 31) && rl + (1u << 30) < (1u << 31));
          };
          badv |= ((c < D && bad64(w.x, w.y, b0.x, b0.y)) || (c + 1 < D && bad64(w.z, w.w, b0.z, b0.w))) ? 1u : 0u;
        }
      }
    }
    __syncthreads();
  };
  // WIDE: row i of this lane's column from the tile
  auto tl = [&](int i) __attribute__((always_inline)) -> uint32_t {
    return tile[(wave * P + cw) * TROW + seg * 65 + i];
  };
  uint64_t acc[WIDE ? 1 : KEEP];
#pragma unroll
  for (int k = 0; k < (WIDE ? 1 : KEEP); ++k) acc[k] = 0;
  if constexpr (WIDE) {
    for (int t = tid; t < NPAD; t += NT) qr_lds[t] = 0;
    __syncthreads();
  }
  // unconstrained: the base B of column c = its row-0 value (low / high words; int32 storage: sign-extended)
  auto base_of = [&](int c, int ord) __attribute__((always_inline)) -> u32x2_t {
    if constexpr (V32) {
      const uint32_t l = bload(rs, after(c * 4, ord), 0);
      return u32x2_t{l, (uint32_t)((int32_t)l >> 31)};
    } else {
      return __builtin_amdgcn_raw_buffer_load_b64(rs, after(c * 8, ord), 0, 0);
    }
  };
  // a stored low word as a number: [0, 1e6] (constrained) or an int32 (unconstrained)
  auto xv = [](uint32_t x) __attribute__((always_inline)) { return CONS ? (double)x : (double)(int32_t)x; };
  constexpr uint32_t kSign = CONS ? 0u : 0x80000000u;   // order-preserving key of an int32

  // ------------------------------------------------------------ pass 1 (contract.cairo:455-463)
  // One slab.  FULL: N = NPAD and every column of the slab < D -- no per-row masks (the general form's 64
  // per-lane row compares were hoisted out of the loop as SGPR masks and, with the 64 row offsets, spilled
  // to VGPR lanes: ~480 v_readlane per slab).  The row offsets are recomputed per slab (opaque stride).
  auto pass1 = [&](auto full_c, int s) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(full_c)::value;
    const int col = s * W + wave * P + cw;
    const bool vc = FULL || col < D;
    const int vo = seg_off + (vc ? col : 0) * ESZ;
    const int nvf = FULL ? 64 : nv, nlf = FULL ? 64 : nl;
    int rowb1 = rowb;
    asm volatile("" : "+s"(rowb1));
    uint32_t c1;
    if constexpr (TILE) load_tile(s);
    // unconstrained: the column's base B = its row-0 value (every lane of the group loads it)
    uint32_t Bl = 0u, Bh = 0u;
    if constexpr (!CONS) Bl = base_of(vc ? col : 0, s)[0];   // (the high word: after the network)
    {
      uint32_t r[64];
      // domain checks as running extremes of the stored words (one v_max3 / v_min3 per two rows; per-row compares
      // became 64 SGPR masks, and the int32 overflow test held the stored words: one wave per SIMD less).  Rows
      // past N read as 0 from the buffer (constrained: inside [0, 1e6]) or are replaced by the base
      uint32_t wmax = 0u;                   // constrained: largest stored word (unsigned: negative -> huge)
      int32_t smax = (int32_t)Bl, smin = (int32_t)Bl;   // unconstrained int32: extremes of the real rows
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        // (the low word only: int64 rows get their high words checked below, 8 rows at a time -- loaded
        // here they held 64 more VGPRs and cost the int64 kernels their second wave per SIMD)
        const uint32_t w = TILE ? tl(i) : bload(rs, vo, i * rowb1);
        const uint32_t x = w - Bl;   // (unconstrained: relative to B)
        const bool real = i < nvf;
        // (rows past N: the non-tiled load reads 0 out of bounds, but the LDS tile's padding rows hold
        // leftover words -- masked, or they would send the instance to the i128 kernel at random)
        if constexpr (CONS) wmax = __builtin_elementwise_max(wmax, (FULL || !TILE) ? w : (w & lt_mask(i, nvf)));
        if constexpr (!CONS && V32) {
          const int32_t ws = FULL ? (int32_t)w : (int32_t)((w & lt_mask(i, nvf)) | (Bl & ~lt_mask(i, nvf)));
          smax = __builtin_elementwise_max(smax, ws);
          smin = __builtin_elementwise_min(smin, ws);
        }
        r[i] = (real ? x ^ kSign : (i < nlf ? 0u : ~0u)) ^ pol;
      }
      if constexpr (CONS) badv |= (vc && wmax > kWsadMax) ? 1u : 0u;   // outside [0, 1e6]
      if constexpr (!CONS && V32) {
        // int32 storage: every x - B within [-2^30, 2^30) as an exact integer (no int32 overflow)
        const int64_t up = (int64_t)smax - (int32_t)Bl, dn = (int64_t)(int32_t)Bl - smin;
        badv |= (vc && (up >= (1ll << 30) || dn > (1ll << 30))) ? 1u : 0u;
      }
      uint32_t lo, hi;
      if constexpr (WINH > 0) {
        // the median pair and the window W[t] = key at padded position NPAD/2 - WINH + t (t < 2 WINH),
        // staged at rows 4 .. 4 + 2 WINH of this instance's stage (true keys = the values)
        constexpr int WN = NSEG == 1 ? 2 * WINH : WINH;
        uint32_t w[WN];
        if constexpr (NSEG == 4 && WINH == 17) {
          // pruned network (sortnet.hpp window_group_pruned: only every lane's middle 32 keys enter the cross-lane
          // merges) with its exactness check; a wave with any failing column reruns the full network from the rows
          bool ok;
          window_group_pruned<P, WINH>(r, seg, lane, w, lo, hi, ok);
          if (__ballot(!ok) != 0) {
#pragma unroll
            for (int i = 0; i < 64; ++i) {
              const uint32_t x = bload(rs, after(vo, lo), i * rowb1) - Bl;
              r[i] = (i < nvf ? x ^ kSign : (i < nlf ? 0u : ~0u)) ^ pol;
            }
            window_group<NSEG, P, WINH>(r, seg, lane, w, lo, hi);
          }
        } else {
          window_group<NSEG, P, WINH>(r, seg, lane, w, lo, hi);
        }
        constexpr int SLO = NSEG == 4 ? 1 : 0;   // the lane holding the lower part (the upper: SLO + 1)
        if (vc) {
#pragma unroll
          for (int m = 0; m < WINH; ++m) {
            if (NSEG == 1) {
              stg[(4 + m) * D + col] = (int32_t)w[m];
              stg[(4 + 2 * WINH - 1 - m) * D + col] = (int32_t)~w[WINH + m];
            } else if (seg == SLO) {
              stg[(4 + m) * D + col] = (int32_t)w[m];
            } else if (seg == SLO + 1) {
              stg[(4 + 2 * WINH - 1 - m) * D + col] = (int32_t)~w[m];
            }
          }
        }
      } else if constexpr (WIDE) {
        median_group_wide<NSEG, P>(r, seg, lane, lo, hi);
      } else {
        median_group<NSEG>(r, lo, hi);   // smooth median: ranks N/2 - 1, N/2 (math.cairo:113-126)
      }
      if constexpr (CONS) {
        c1 = (lo + hi) >> 1;           // idiv_pos64(a + b, 2) of non-negative values
      } else {                         // I128Div(a + b, 2) of the absolute values, relative to B
        const int32_t sum = (int32_t)(lo ^ kSign) + (int32_t)(hi ^ kSign);   // (|sum| < 2^30)
        const u32x2_t bv = base_of(vc ? col : 0, (int)lo);
        Bh = bv[1];
        badv |= (vc && Bh + (1u << 20) >= (1u << 21)) ? 1u : 0u;   // |B| < 2^52
        c1 = (uint32_t)(int32_t)tdiv_rel_fix(sum / 2, (sum & 1) == 0, sum < 0, (int64_t)(((uint64_t)Bh << 32) | Bl));
      }
    }
    if (seg == 0 && vc) {
      stg[col] = (int32_t)c1;
      if constexpr (!CONS) {
        stg[4 * D + col] = (int32_t)Bl;
        stg[5 * D + col] = (int32_t)Bh;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // quadratic risk (math.cairo:225-238): this column's qdev of every row, summed over the columns
    uint32_t q[64];
    const double cd = xv(c1);
    if constexpr (!CONS) {
      // d = x - c1 relative (|d| < 2^30 in the domain); the narrow form unless some |d| >= 2^25 in the wave
      if constexpr (TILE) {
#pragma unroll
        for (int i = 0; i < 64; ++i) q[i] = tl(i);
      } else {
        load_lo(rs, after(vo, c1), rowb, q);
      }
      bool wd = false;
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        q[i] = q[i] - Bl - c1;
        wd = wd || (vc && i < nvf && wide25(q[i]));
      }
      if (__ballot(wd) == 0) {
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          if ((i & 7) == 0) __builtin_amdgcn_sched_barrier(0);
          q[i] = (vc && i < nvf) ? qdev_u((double)(int32_t)q[i]) : 0u;
        }
        if constexpr (!WIDE) qtree64_all<P>(q, lane, acc, std::make_integer_sequence<int, KEEP>{});
      } else if constexpr (WIDE) {
        // 43-bit quotients straight into the per-oracle sums (64-bit LDS atomics); q is cleared for the
        // narrow-path atomics below
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          if ((i & 3) == 0) __builtin_amdgcn_sched_barrier(0);
          const uint64_t qq = (vc && i < nvf) ? (uint64_t)qdev_wide((double)(int32_t)q[i]) : 0ull;
          if (qq) atomicAdd((unsigned long long*)&qr_lds[seg * 64 + i], (unsigned long long)qq);
          q[i] = 0u;
        }
      } else {
        // 43-bit quotients: the low words through the 64-bit butterfly, then (recomputed from a second read)
        // the high words through the 32-bit one, shifted
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          if ((i & 3) == 0) __builtin_amdgcn_sched_barrier(0);   // (4 rows of double-double temporaries)
          q[i] = (vc && i < nvf) ? q_lo(qdev_wide((double)(int32_t)q[i])) : 0u;
        }
        qtree64_all<P>(q, lane, acc, std::make_integer_sequence<int, KEEP>{});
        __builtin_amdgcn_sched_barrier(0);   // (the re-read after the whole butterfly, not beside it)
        load_lo(rs, after(vo, acc[KEEP - 1]), rowb, q);
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          if ((i & 3) == 0) __builtin_amdgcn_sched_barrier(0);
          q[i] = (vc && i < nvf) ? q_hi(qdev_wide((double)(int32_t)(q[i] - Bl - c1))) : 0u;
        }
        qtree_hi_all<P>(q, lane, acc, std::make_integer_sequence<int, KEEP>{});
      }
    } else if constexpr (TILE) {
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        if ((i & 7) == 0) __builtin_amdgcn_sched_barrier(0);
        q[i] = (vc && i < nvf) ? qdev_u((double)tl(i) - cd) : 0u;
      }
    } else if constexpr (BATCH1) {
      load_lo(rs, after(vo, c1), rowb, q);
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        if ((i & 7) == 0) __builtin_amdgcn_sched_barrier(0);   // bound the fp64 temporaries in flight
        q[i] = (vc && i < nvf) ? qdev_u(xv(q[i]) - cd) : 0u;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const uint32_t x = bload(rs, vo, i * rowb1);   // (low word; int64 high words are checked below)
        q[i] = (vc && i < nvf) ? qdev_u(xv(x) - cd) : 0u;
      }
    }
    if constexpr (WIDE) {
      // each lane's 64 rows (one column) into the per-oracle sums: LDS atomics (rows of the same segment meet
      // from the P columns of a wave and from the other waves)
#pragma unroll
      for (int i = 0; i < 64; ++i)
        if (q[i]) atomicAdd((unsigned long long*)&qr_lds[seg * 64 + i], (unsigned long long)q[i]);
    } else if constexpr (CONS) {
      qtree_all<P>(q, lane, acc, std::make_integer_sequence<int, KEEP>{});
    }
    if constexpr (!V32 && !TILE) {
      // int64 storage: the high words, 8 rows in flight -- 0 (constrained: [0, 1e6]); unconstrained: x - B
      // is the sign extension of its low word and within 2^30
#pragma nounroll
      for (int g = 0; g < 64; g += 8) {
        uint32_t hw[8], lw[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          hw[k] = bload(rs, vo + 4, (g + k) * rowb);
          lw[k] = CONS ? 0u : bload(rs, vo, (g + k) * rowb);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if constexpr (CONS) {
            badv |= (vc && g + k < nvf && hw[k] != 0u) ? 1u : 0u;
          } else {
            const uint32_t rl = lw[k] - Bl, rh = hw[k] - Bh - (lw[k] < Bl ? 1u : 0u);
            const bool ok = rh == (uint32_t)((int32_t)rl >> 31) && rl + (1u << 30) < (1u << 31);
            badv |= (vc && g + k < nvf && !ok) ? 1u : 0u;
          }
        }
      }
    }
  };
  if constexpr (MODE != 2) {
    const int nfull = N == NPAD ? min(D / W, nslab) : 0;
    // (a wave that meets a value outside the domain stops: the instance goes to the wide-column / i128 kernels
    // anyway.  Not with the LDS tile, whose loads every wave's barriers share.)
#pragma nounroll
    for (int s = 0; s < nfull; ++s) {
      if (!TILE && __ballot(badv != 0u) != 0) break;
      pass1(std::true_type{}, s);
    }
#pragma nounroll
    for (int s = nfull; s < nslab; ++s) {
      if (!TILE && __ballot(badv != 0u) != 0) break;
      pass1(std::false_type{}, s);
    }
  }
  if constexpr (!WIDE) {
    int base = 0;
#pragma unroll
    for (int h = 32, msk = P / 2; msk >= 1; h >>= 1, msk >>= 1) base += (lane & msk) ? h : 0;
#pragma unroll
    for (int k = 0; k < KEEP; ++k) qr_part[wave * NPAD + seg * 64 + base + k] = acc[k];
  }
  __syncthreads();
  // (WIDE: pass 1 summed the qr into qr_lds by LDS atomics; mode 2 reads the all-reduced qr for every width)
  for (int t = tid; t < ((WIDE && MODE != 2) ? 0 : NPAD); t += NT) {
    uint64_t v = 0;
    if constexpr (MODE == 2) {   // the all-reduced qr (int64; a negative total cannot come from this domain)
      const int64_t q = t < N ? p.qr[(int64_t)b * N + t] : 0;
      if (q < 0) flag = 1;
      v = (uint64_t)q;
    } else {
#pragma unroll
      for (int w = 0; w < WAVES; ++w) v += qr_part[w * NPAD + t];
    }
    qr_lds[t] = v;
  }
  if (MODE != 2 && badv) flag = 1;
  __syncthreads();
  if (MODE == 0 && flag) {   // a value outside the domain: the wide-column / i128 kernels take the round (pass 1
    if (tid == 0) p.fallback[b] = 1;   // stopped at the wave's first such slab; no rank mask / reliabilities here)
    return;
  }
  if (MODE == 1) {   // first half done: c1 and the qr partials out (partials < 2^58: D <= 2^38 columns)
    if (flag) {
      if (tid == 0) p.fallback[b] = 1;
      return;
    }
    for (int c = tid; c < D; c += NT) p.c1[(int64_t)b * D + c] = stg[c] + stage_base(stg, c);
    for (int t = tid; t < N; t += NT) p.qr[(int64_t)b * N + t] = (int64_t)qr_lds[t];
    if (tid == 0) {
      p.status[b] = ST_OK;
      p.fallback[b] = 0;
    }
    return;
  }

  // ------------------------------------------------------------ rank mask (contract.cairo:345-363)
  const int f = p.n_failing;
  const int R = N - f;
  if constexpr (WIDE) {
    __shared__ uint32_t rk_hist[256], rk_wsum[4], rk_sel[2];
    static_assert(NT == 256, "rank_mask_select: 256 threads");
    if (R >= 1 && R <= N) rank_mask_select<NPAD>(qr_lds, N, R, relmask, rk_hist, rk_wsum, rk_sel, tid);
    else
      for (int w = tid; w < MW; w += NT) relmask[w] = 0ull;   // (no reliable row: the stage checks revert)
  }
  // constrained: qr <= D (1e6 + 1) < 2^56 and N <= 256, so (qr asc, idx desc) is the one key qr << 8 | (255 - idx):
  // one 64-bit compare per oracle (rankmask.hpp's form for the exact sums)
  constexpr bool KEY8 = CONS && !WIDE && NPAD <= 256;
  __shared__ uint64_t rk_key[KEY8 ? NPAD : 1];
  if constexpr (KEY8) {
    for (int t = tid; t < N; t += NT) rk_key[t] = (qr_lds[t] << 8) | (uint64_t)(255 - t);
    __syncthreads();
  }
  for (int base = 0; base < (WIDE ? 0 : NPAD); base += NT) {
    const int t = base + tid;
    bool rel = false;
    if (t < N) {
      int rank = 0;
      if constexpr (KEY8) {
        const uint64_t my = rk_key[t];
        for (int j = 0; j < N; ++j) rank += rk_key[j] < my ? 1 : 0;
      } else {
        const uint64_t myq = qr_lds[t];
        for (int j = 0; j < N; ++j) {
          const uint64_t qj = qr_lds[j];
          rank += (qj < myq || (qj == myq && j > t)) ? 1 : 0;   // (qr asc, idx desc)
        }
      }
      rel = rank < R;
    }
    const uint64_t bal = __ballot(rel);
    if (lane == 0 && (t >> 6) < MW) relmask[t >> 6] = bal;
  }
  __syncthreads();
  if (tid == 0) {
    // reliabilities with the wsad.hpp routines (contract.cairo:436-439); any failure -> i128 kernel
    int st = ST_OK;
    i128 s_all = 0, s_rel = 0;
    for (int t = 0; t < N; ++t) {
      const i128 qv = (i128)qr_lds[t];
      s_all = add(s_all, qv, st);
      if ((relmask[t >> 6] >> (t & 63)) & 1) s_rel = add(s_rel, qv, st);
    }
    // D-sharded: the global dimension; the obsolete contracts divide by nothing (contract_nd.cairo:340-442)
    const int64_t rd = p.legacy ? 1 : (p.rel_dim > 0 ? p.rel_dim : D);
    // The reference's stages in order (contract.cairo:442-503; reference_cpu.cpp exact_round_one): rel1 and
    // its interval check, the rank cut, pass 2 (R >= 2 reliable rows, else the i128 kernel names the
    // smooth median's error), rel2 and its interval check, then the moments, whose only failure in this
    // domain is a division by zero (a reliable column of variance 0 or 1, or R <= 3).  A failure before
    // the moments is final here (the round reverts with that code, outputs untouched, no fallback).
    // Unconstrained (contract.cairo:379-433): the pass-2 essence is the reliable mean, whose division by
    // R = 0 is the first failure of an empty reliable set; R = 1 .. 3 fail later, in the moments.
    const i128 rel1 = CONS ? constrained_reliability(idiv(s_all, (i128)N, st), rd, st)
                           : unconstrained_reliability(wsqrt(idiv(s_all, (i128)N, st), st), (i128)p.max_spread, st);
    if (st == ST_OK && !in_unit_interval(rel1)) st = ST_RELIABILITY_INTERVAL;
    if (st == ST_OK && f > N) st = ST_USIZE_UNDERFLOW;
    const bool fb = st == ST_OK && (f < 0 || (CONS ? R < 2 : p.legacy != 0));
    if (!CONS && st == ST_OK && !fb && R == 0) st = ST_DIV_BY_ZERO;
    i128 rel2 = 0;
    if (st == ST_OK && !fb) {
      rel2 = CONS ? constrained_reliability(idiv(s_rel, (i128)R, st), rd, st)
                  : unconstrained_reliability(wsqrt(idiv(s_rel, (i128)R, st), st), (i128)p.max_spread, st);
      if (st == ST_OK && !in_unit_interval(rel2)) st = ST_RELIABILITY_INTERVAL;
    }
    // (the kurtosis divides by (n-2)(n-3), the skewness by (n-1)(n-2); the obsolete contracts stop before)
    if (st == ST_OK && !fb && !p.legacy && R < 4) st = ST_DIV_BY_ZERO;
    rels[0] = (int64_t)rel1;
    rels[1] = (int64_t)rel2;
    early_st = st;
    if (fb) flag = 1;
    // pass-2 sentinel split: the first (NPAD - R + 1) / 2 non-reliable rows (row order) become -inf
    int need = (NPAD - R + 1) >> 1;
    for (int w = 0; w < MW; ++w) {
      uint64_t nr = w < NSEG ? ~relmask[w] : 0ull, lm = 0ull;
      while (need > 0 && nr) {
        const uint64_t bit = nr & (0ull - nr);
        lm |= bit;
        nr ^= bit;
        --need;
      }
      lowmask[w] = lm;
    }
  }
  if (badv) flag = 1;
  __syncthreads();
  if (flag) {
    if (tid == 0) p.fallback[b] = 1;
    return;
  }
  if (early_st != ST_OK) {   // reverted before the moments: final, outputs untouched
    if (tid == 0) {
      p.status[b] = early_st;
      p.fallback[b] = 0;
    }
    return;
  }

  // ------------------------------------------------------------ pass 2 (contract.cairo:476-500)
  if constexpr (WINH > 0) {
    // the pass-2 smooth median from the window (see above): one lane per column
    if (tid == 0) {
      int k = 0;
      for (int t = 0; t < N && k < 2 * WINH; ++t)
        if (!((relmask[t >> 6] >> (t & 63)) & 1)) urow[k++] = t;
    }
    __syncthreads();
    const int a = N / 2 - R / 2;
    const int wb = WINH - a - 1;   // window index of position R/2 - 1 (>= 0: launch_wsad_c checked)
    // f <= 2 WINH - 2 (launch_wsad_c: f - a + 1 <= WINH with a >= f / 2): only the first 2 WINH - 2 slots can
    // hold removed keys, the rest are +inf -- sorted as a 32- (8-) key network instead of the 64-key one with
    // 34 (10) runtime slots
    constexpr int NR = 2 * WINH - 2;
    constexpr int SN = NR <= 8 ? 8 : 32;
    static_assert(WINH == 0 || NR <= SN, "removed-key slots");
    for (int col = tid; col < D; col += NT) {
      uint32_t z[SN];
#pragma unroll
      for (int t = 0; t < SN; ++t) {
        if (t < NR) {
          const int ur = __builtin_amdgcn_readfirstlane(urow[t < f ? t : 0]);
          const uint32_t x = bload(rs, col * ESZ, ur * rowb);
          z[t] = t < f ? x : ~0u;   // u_f.. = +inf
        } else {
          z[t] = ~0u;
        }
      }
      sort_oem<SN>(z);
      uint32_t gw[2 * WINH];
#pragma unroll
      for (int t = 0; t < 2 * WINH; ++t) {
        const int wi = wb + t < 2 * WINH ? wb + t : 2 * WINH - 1;   // (t <= f + 1 < 2 WINH - wb)
        gw[t] = (uint32_t)stg[(4 + wi) * D + col];
      }
      uint32_t lo = ~0u, hi = ~0u;
#pragma unroll
      for (int j = 0; j + 1 < 2 * WINH; ++j) {
        const uint32_t zj = j < SN ? z[j < SN ? j : 0] : ~0u;   // (slot NR = 2 WINH - 2: +inf)
        if (j <= f) {   // (uniform)
          lo = kmin(lo, gw[j] < zj ? gw[j] : ~0u);
          hi = kmin(hi, gw[j + 1] < zj ? gw[j + 1] : ~0u);
        }
      }
      stg[D + col] = (int32_t)((lo + hi) >> 1);
    }
    __syncthreads();   // (the slab loop reads other threads' columns)
  }
  const uint64_t mymask = relmask[seg];
  const uint64_t mylow = lowmask[seg];
  const double Rd = (double)R, invR = recip_lo(Rd);
  const double k3 = (double)((R - 1) * (R - 2)), ik3 = recip_lo(k3);
  bool bad = false;   // a result this kernel cannot represent: the i128 kernel recomputes the round
  bool dz = false;    // the contract divides by zero in the moments: the round reverts
#pragma nounroll
  for (int s = 0; s < nslab; ++s) {
    const int col = s * W + wave * P + cw;
    const bool vc = col < D;
    const int vo = seg_off + (vc ? col : 0) * ESZ;
    uint64_t mm = mymask, ml = mylow;
    asm volatile("" : "+v"(mm), "+v"(ml));   // keep the 64 row masks out of the slab loop's live set
    uint32_t cons = 0;
    if constexpr (TILE) load_tile(s);
    if constexpr (CONS && WINH > 0) {
      cons = (uint32_t)stg[D + (vc ? col : 0)];   // (the window phase above)
    } else if constexpr (CONS) {
      uint32_t r[64];
      if constexpr (BATCH && (MODE != 2 || V32)) {   // values validated in pass 1 (or 32-bit): one batch
        if constexpr (TILE) {
#pragma unroll
          for (int i = 0; i < 64; ++i) r[i] = tl(i);
        } else {
          load_lo(rs, vo, rowb, r);
        }
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          if (MODE == 2) badv |= (vc && i < nv && r[i] > kWsadMax) ? 1u : 0u;   // no pass 1 here
          const uint32_t mk = bit_mask(mm, i), low = bit_mask(ml, i);
          r[i] = ((r[i] & mk) | (~low & ~mk)) ^ pol;   // reliable: key; else -inf (low) / +inf
        }
      } else {
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          uint32_t hw = 0u;
          const uint32_t x = MODE == 2 ? wload<V32>(rs, vo, i * rowb, hw) : bload(rs, vo, i * rowb);
          if (MODE == 2) badv |= (vc && i < nv && (x > kWsadMax || hw != 0)) ? 1u : 0u;   // no pass 1 here
          const uint32_t mk = bit_mask(mm, i), low = bit_mask(ml, i);
          r[i] = ((x & mk) | (~low & ~mk)) ^ pol;   // reliable: key; else -inf (low) / +inf
        }
      }
      uint32_t lo, hi;
      if constexpr (WIDE) median_group_wide<NSEG, P>(r, seg, lane, lo, hi);
      else median_group<NSEG>(r, lo, hi);
      cons = (lo + hi) >> 1;
    }
    __builtin_amdgcn_sched_barrier(0);
    if (CONS && p.legacy) {   // (uniform) obsolete contracts: consensus only, no moments stored
      if (seg == 0 && vc) {
        stg[D + col] = (int32_t)cons;
        stg[2 * D + col] = 0;
        stg[3 * D + col] = 0;
      }
      continue;
    }
    // the column is re-read per statistic (L2-hot) instead of held in 64 more VGPRs: the fp64 work
    // below needs the registers, and occupancy hides the re-read latency
    // mean (math.cairo:240-254): idiv(sum, R) of non-negative values
    uint32_t xr[64];
    double mu;
    using SumT = std::conditional_t<WIDE, uint64_t, uint32_t>;   // (R values of up to 1e6)
    if constexpr (CONS) {
      SumT sx = 0;
      if constexpr (BATCH1) {
        // (window path: no network in this loop, so the column is loaded once and kept for the mean,
        // variance and z-power loops; otherwise re-read per statistic)
        if constexpr (TILE) {
#pragma unroll
          for (int i = 0; i < 64; ++i) xr[i] = tl(i);
        } else {
          load_lo(rs, WINH > 0 ? vo : after(vo, cons), rowb, xr);
        }
#pragma unroll
        for (int i = 0; i < 64; ++i) sx += xr[i] & bit_mask_o(mm, i);
      } else {
#pragma unroll 16
        for (int i = 0; i < 64; ++i) sx += bload(rs, vo, i * rowb) & bit_mask(mm, i);
      }
      sx = group_sum<NSEG, P>(sx);
      mu = floor_div_d((double)sx, Rd, invR);
    } else {   // signed sum of the relative values (|sum| < 2^38: exact), I128Div of the absolute sum toward
               // zero shifted back (tdiv_rel); the mean is the consensus.  The column is loaded once (no network
               // in this loop) and kept for the variance and z-power loops.
      const u32x2_t bv = base_of(vc ? col : 0, (int)mm);
      if constexpr (TILE) {
#pragma unroll
        for (int i = 0; i < 64; ++i) xr[i] = tl(i);
      } else {
        load_lo(rs, after(vo, mm), rowb, xr);
      }
#pragma unroll
      for (int i = 0; i < 64; ++i) xr[i] -= bv[0];
      double sxd = 0.0;
#pragma unroll
      for (int i = 0; i < 64; ++i) sxd += bit_mask(mm, i) ? xv(xr[i]) : 0.0;
      sxd = group_sum<NSEG, P>(sxd);
      const double qd = trunc_div_d(sxd, Rd, invR);
      const int64_t mr = tdiv_rel_fix((int64_t)qd, fma(-qd, Rd, sxd) == 0.0, sxd < 0.0,
                                      (int64_t)(((uint64_t)bv[1] << 32) | bv[0]));
      mu = (double)mr;
      cons = (uint32_t)(int32_t)mr;
    }
    // population variance (math.cairo:208-222): mean of qdev(x, mu) over the reliable rows
    double var;
    if constexpr (CONS) {
      SumT sv = 0;
      if constexpr (BATCH || (WINH > 0 && BATCH1)) {
        if constexpr (TILE) {
#pragma unroll
          for (int i = 0; i < 64; ++i) xr[i] = tl(i);
        } else if constexpr (WINH == 0) {
          load_lo(rs, after(vo, mu), rowb, xr);
        }
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          if ((i & 7) == 0) __builtin_amdgcn_sched_barrier(0);
          sv += bit_mask_o(mm, i) & qdev_u((double)xr[i] - mu);
        }
      } else {
#pragma unroll 16
        for (int i = 0; i < 64; ++i) {
          const uint32_t x = bload(rs, vo, i * rowb);
          sv += bit_mask(mm, i) & qdev_u((double)x - mu);
        }
      }
      sv = group_sum<NSEG, P>(sv);
      var = floor_div_d((double)sv, Rd, invR);
    } else {   // fp64 sums of the relative deviations (exact: terms < 2^43, R <= 256), narrow or wide forms
      const uint32_t mui = (uint32_t)(int32_t)mu;
      // (each loop takes its own opaque copy of the row mask: 64 shared per-row masks, or shared
      // conversions, would stay live across the branch -- one wave per SIMD less)
      bool wd = false;
      {
        uint64_t m0 = mm;
        asm volatile("" : "+v"(m0));
#pragma unroll
        for (int i = 0; i < 64; ++i) wd = wd || (vc && bit_mask(m0, i) != 0u && wide25(xr[i] - mui));
      }
      double svd = 0.0;
      uint64_t m1 = mm;
      asm volatile("" : "+v"(m1));
      if (__ballot(wd) == 0) {
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          if ((i & 7) == 0) __builtin_amdgcn_sched_barrier(0);
          svd += bit_mask(m1, i) ? qdev_h((double)(int32_t)(xr[i] - mui)) : 0.0;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          if ((i & 7) == 0) __builtin_amdgcn_sched_barrier(0);
          svd += bit_mask(m1, i) ? qdev_wide((double)(int32_t)(xr[i] - mui)) : 0.0;
        }
      }
      svd = group_sum<NSEG, P>(svd);
      var = floor_div_d(svd, Rd, invR);
      if (vc && !(var < 8796093022208.0)) bad = true;   // wsqrt_wide's bound (2^43)
      if (bad) var = 0.0;
    }
    // var 0 (sqrt 0 -> wsad_div by zero) and var 1 (sqrt(1) divides by zero) revert the round
    double sd = 1.0;
    bool ok_sd;
    if (CONS || var < 2147483648.0) {
      ok_sd = var >= 2.0 && wsqrt_d(var, sd);
    } else {   // (unconstrained, wide columns)
      int64_t sdi = 1;
      ok_sd = wsqrt_wide((int64_t)var, sdi);
      sd = (double)sdi;
    }
    if (vc && !ok_sd) dz = true;   // sqrt(0) -> wsad_div by 0, sqrt(1) divides by 0: DIV_BY_ZERO
    // z = wsad_div(x - mu, sd) = I128Div((x - mu) 1e6 + floor(sd / 2), sd): A = x 1e6 + C0 (exact integers
    // below 2^51), then the half-offset forms of wsad_fast.hpp -- no remainder tests in the row loop
    const double isd = 1.0 / sd, hisd = 0.5 * isd;
    const double C0 = fma(-mu, kW, floor(sd * 0.5));
    const uint32_t mu_u = (uint32_t)(int32_t)mu;
    // z-score powers (math.cairo:320-363), reliable rows only
    double s3 = 0.0, s4 = 0.0;
    bool outl = false;   // a row with z^2 >= 2^25 (|z| >= 5.79): this column's sums are redone below
    // z-score powers of one row (a masked row reads as mu: z = 0, all powers 0)
    // (1e6 as an opaque SGPR pair: with the literal the fma became v_fmac_f64 on a v_mov_b64 copy of C0)
    double kWs = kW;
    asm volatile("" : "+s"(kWs));
    auto zpow = [&](uint32_t x, uint32_t mk) {
      const uint32_t xm = (x & mk) | (mu_u & ~mk);
      const double z = tdiv_h(fma(xv(xm), kWs, C0), isd, hisd);
      const double z2 = wmul_pos_h(z, z);
      outl = outl || !(z2 < 33554432.0);   // 2^25: keeps z^2 z and z^2 z^2 below the forms' 2.25e9 quotients
      s3 += wmul_t(z2, z);
      s4 += wmul_pos_h(z2, z2);
    };
    if constexpr (BATCH || (WINH > 0 && BATCH1) || !CONS) {
      if constexpr (TILE) {
#pragma unroll
        for (int i = 0; i < 64; ++i) xr[i] = tl(i);
      } else if constexpr (WINH == 0 && CONS) {
        load_lo(rs, after(vo, sd), rowb, xr);
      }
      if constexpr (!CONS) {   // (re-read: the column is not kept across the square root)
        const uint32_t bl = base_of(vc ? col : 0, (int)sd)[0];
        if constexpr (!TILE) load_lo(rs, after(vo, sd), rowb, xr);
#pragma unroll
        for (int i = 0; i < 64; ++i) xr[i] -= bl;
      }
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        if ((i & 7) == 0) __builtin_amdgcn_sched_barrier(0);   // bound the fp64 temporaries in flight
        zpow(xr[i], bit_mask_o(mm, i));
      }
    } else {
#pragma unroll 8
      for (int i = 0; i < 64; ++i) zpow(bload(rs, vo, i * rowb), bit_mask(mm, i));
    }
    // a column with outlier rows (rare; a reliable row far from the mean) is summed again, row by row: the
    // same z and z^2 (exact in fp64), and for the outliers wsad_mul(z^2, z) / wsad_mul(z^2, z^2) in int64
    // -- |z| <= sqrt(R - 1) in real units keeps both products below 2^63 (signed_decimal.cairo:110-112:
    // truncation toward zero, as int64 division).  The fast loop above stays as lean as without outliers.
    if (outl) {
      s3 = 0.0;
      s4 = 0.0;
#pragma nounroll
      for (int g = 0; g < 64; g += 8) {   // 8 rows per step: their loads in flight together
        uint32_t xg[8];
        const uint32_t bl = CONS ? 0u : base_of(vc ? col : 0, g)[0];   // (unconstrained: the base)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xg[k] = (TILE ? tl(g + k) : bload(rs, vo, (g + k) * rowb)) - bl;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t mk = bit_mask(mm, g + k);
          const uint32_t xm = (xg[k] & mk) | (mu_u & ~mk);
          const double z = tdiv_h(fma(xv(xm), kW, C0), isd, hisd);
          const double z2 = wmul_pos_h(z, z);
          if (z2 < 33554432.0) {
            s3 += wmul_t(z2, z);
            s4 += wmul_pos_h(z2, z2);
          } else {
            const int64_t zi = (int64_t)z, z2i = (int64_t)z2;
            if (z2i > (1ll << 40)) bad = true;   // (impossible for |z| <= sqrt(R - 1); kept as a guard)
            s3 += (double)((z2i * zi + 500000ll) / 1000000ll);
            s4 += (double)((z2i * z2i + 500000ll) / 1000000ll);
          }
        }
      }
    }
    s3 = group_sum<NSEG, P>(s3);
    s4 = group_sum<NSEG, P>(s4);
    // skewness = idiv(s3 * n, (n-1)(n-2)); kurtosis = idiv(idiv(s4 n (n+1), n-1) - 3W(n-1)^2, (n-2)(n-3))
    // (wide groups: the int64 / fp64 forms below hold while s3 R < 2^51 and s4 R (R + 1) < 2^63)
    if (vc && !(fabs(s3) * Rd < 2251799813685248.0 && s4 * Rd * (Rd + 1.0) < 9.2e18)) bad = true;
    const double sk = trunc_div_d(s3 * Rd, k3, ik3);
    const int64_t t1 = ((int64_t)s4 * (int64_t)R * (int64_t)(R + 1)) / (int64_t)(R - 1);
    const int64_t t2 = 3ll * 1000000ll * (int64_t)(R - 1) * (int64_t)(R - 1);
    const int64_t ku = (t1 - t2) / ((int64_t)(R - 2) * (int64_t)(R - 3));
    if (vc && (fabs(sk) > 2147483647.0 || ku > INT32_MAX || ku < INT32_MIN)) bad = true;
    if (seg == 0 && vc) {
      stg[D + col] = (int32_t)cons;
      stg[2 * D + col] = (int32_t)sk;
      stg[3 * D + col] = (int32_t)ku;
    }
  }
  if (bad || (MODE == 2 && badv)) flag = 1;
  if (dz) div0 = 1;
  __syncthreads();
  if (flag) {
    if (tid == 0) p.fallback[b] = 1;
    return;
  }
  if (div0) {   // (every moment failure is DIV_BY_ZERO, whichever column comes first: final)
    if (tid == 0) {
      p.status[b] = ST_DIV_BY_ZERO;
      p.fallback[b] = 0;
    }
    return;
  }

  // ------------------------------------------------------------ commit (a successful round)
  const int64_t ob = (int64_t)b * D;
  for (int c = tid; c < D; c += NT) {
    const int64_t bs = stage_base(stg, c);   // (unconstrained: the column's base; else 0)
    if (MODE == 0 && p.c1) p.c1[ob + c] = stg[c] + bs;   // (mode 2: c1 is the input, unchanged)
    p.consensus[ob + c] = stg[D + c] + bs;
    p.skew[ob + c] = stg[2 * D + c];
    p.kurt[ob + c] = stg[3 * D + c];
  }
  for (int t = tid; t < N; t += NT) {
    p.reliable[(int64_t)b * N + t] = (relmask[t >> 6] >> (t & 63)) & 1;
    p.qr[(int64_t)b * N + t] = (int64_t)qr_lds[t];
  }
  if (tid == 0) {
    p.rel[2 * (int64_t)b] = rels[0];
    p.rel[2 * (int64_t)b + 1] = rels[1];
    p.status[b] = ST_OK;
    p.fallback[b] = 0;
  }
}

template <int NSEG, bool CONS>
static int launch_wsad_c(const ExactParams& p, hipStream_t stream) {
  constexpr int WAVES = 4;
  auto k = p.val32 ? consensus_wsad_kernel<NSEG, WAVES, true, 0, CONS> : consensus_wsad_kernel<NSEG, WAVES, false, 0, CONS>;
  if constexpr (CONS) {
    // whole constrained rounds: the one-network window path (exact_win_h: 0 = a second network)
    const int h = p.mode == 0 && !p.legacy ? exact_win_h(p.N, p.n_failing) : 0;
    if (h == 5) k = p.val32 ? consensus_wsad_kernel<NSEG, WAVES, true, 0, true, 5> : consensus_wsad_kernel<NSEG, WAVES, false, 0, true, 5>;
    if (h == 17) k = p.val32 ? consensus_wsad_kernel<NSEG, WAVES, true, 0, true, 17> : consensus_wsad_kernel<NSEG, WAVES, false, 0, true, 17>;
    if (h != p.win_h) return -3;   // (the caller sized the stage for p.win_h)
  }
  if (p.mode == 1)
    k = p.val32 ? consensus_wsad_kernel<NSEG, WAVES, true, 1, CONS> : consensus_wsad_kernel<NSEG, WAVES, false, 1, CONS>;
  if (p.mode == 2)
    k = p.val32 ? consensus_wsad_kernel<NSEG, WAVES, true, 2, CONS> : consensus_wsad_kernel<NSEG, WAVES, false, 2, CONS>;
  hipLaunchKernelGGL(k, dim3(p.B), dim3(WAVES * 64), 0, stream, p);
  return (int)hipGetLastError();
}
// N > 256: whole rounds on the wide lane groups (the binding sized the stage for win_h = 0), and the D-sharded
// halves of constrained rounds (mode 1: c1 + the per-oracle qr partials of this column slice, summed by the LDS
// atomics of pass 1; mode 2: the rank mask from the all-reduced qr, then pass 2 -- svoc.parallel.dshard)
template <int NSEG>
static int launch_wide(const ExactParams& p, hipStream_t stream) {
  constexpr int WAVES = 4;
  if (p.win_h != 0) return -3;
  auto k = p.val32 ? consensus_wsad_kernel<NSEG, WAVES, true, 0, true> : consensus_wsad_kernel<NSEG, WAVES, false, 0, true>;
  if (!p.constrained)
    k = p.val32 ? consensus_wsad_kernel<NSEG, WAVES, true, 0, false> : consensus_wsad_kernel<NSEG, WAVES, false, 0, false>;
  else if (p.mode == 1)
    k = p.val32 ? consensus_wsad_kernel<NSEG, WAVES, true, 1, true> : consensus_wsad_kernel<NSEG, WAVES, false, 1, true>;
  else if (p.mode == 2)
    k = p.val32 ? consensus_wsad_kernel<NSEG, WAVES, true, 2, true> : consensus_wsad_kernel<NSEG, WAVES, false, 2, true>;
  hipLaunchKernelGGL(k, dim3(p.B), dim3(WAVES * 64), 0, stream, p);
  return (int)hipGetLastError();
}
template <int NSEG>
static int launch_wsad(const ExactParams& p, hipStream_t stream) {
  return p.constrained ? launch_wsad_c<NSEG, true>(p, stream) : launch_wsad_c<NSEG, false>(p, stream);
}

}  // namespace svoc

using namespace svoc;

// -2: not applicable (the caller runs the i128 kernel on every instance).
extern "C" int svoc_exact_round_wsad(const ExactParams* p, hipStream_t stream) {
  if (p->B <= 0) return 0;
  // lane = column: with few columns most lanes idle, and for N <= 32 the i128 kernel packs 2-8
  // instances per wave instead (profiles/r2_exact_crossover.json: 7 x 6 140 M vs 10 M rounds/s,
  // 16 x 16 27 M vs 10 M; but 64 x 16 already 8.3 M vs 6.0 M for this kernel)
  if (p->N < 4 || p->N > 4096) return -2;
  if (p->N > 256 && p->mode != 0 && !p->constrained) return -2;   // (wide groups: D-sharded halves constrained)
  if (p->N <= 32 && p->D < p->wsad_min_d) return -2;
  if (!p->stage || !p->fallback) return -2;
  if ((int64_t)p->N * p->D * (p->val32 ? 4 : 8) >= (1ll << 31)) return -2;   // 32-bit buffer offsets
  if (p->N <= 64) return launch_wsad<1>(*p, stream);
  if (p->N <= 128) return launch_wsad<2>(*p, stream);
  if (p->N <= 256) return launch_wsad<4>(*p, stream);
  if (p->N <= 512) return launch_wide<8>(*p, stream);
  if (p->N <= 1024) return launch_wide<16>(*p, stream);
  if (p->N <= 2048) return launch_wide<32>(*p, stream);
  return launch_wide<64>(*p, stream);
}
