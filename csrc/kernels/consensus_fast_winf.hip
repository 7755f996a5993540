// Fused two-pass robust consensus over fp32 STORAGE (reference resolution), "window" variant: ONE
// sorting network and ONE read of the instance per round.
//
// Semantics: contract/src/contract.cairo:442-503 (constrained) / :370-434 (unconstrained), in the fast
// engine's real-unit form (csrc/engine/reference_cpu.cpp fast_round_one, the CPU twin).  Same algorithm
// as the bf16 window kernel (consensus_fast_win.hip:1-26), on 32-bit keys, one column per lane:
//   pass 1 (phase A): per column, the 64*NSEG rows of a lane group (NSEG = ceil(N / 64) lanes x 64
//     rows) go through the in-register median network extended to keep H keys on either side of the
//     median (window_group, sortnet.hpp) -> c1 (math.cairo:113-126) and the window, written to the
//     workspace; the qr loop (math.cairo:225-238) also accumulates the all-row power sums of
//     d = x - c1 (packed over row pairs: v_pk_fma_f32);
//   rank mask: sort by (qr asc, idx desc) (sort.cairo:96-101), the first R = N - f are reliable
//     (contract.cairo:345-363);
//   pass 2 (phase B, one lane per column): only the f removed rows are read.  The pass-2 smooth median
//     over the R reliable rows (contract.cairo:476-480) is an order statistic of the FULL column shifted
//     by at most f ranks, so it is read off the window by ranking the sorted removed keys against it;
//     the reliable rows' power sums are the all-row sums minus the removed rows' (fp64 combination),
//     with an exact two-pass recomputation for columns where that difference would cancel.
// Versus consensus_fast_f32.hip (the two-network kernel): no second 64*NSEG-key network and no second
// read of the instance.  HBM per round: ONE read of the instance (phase A streams it through LDS by
// DMA, double-buffered against the compute through the registers: see SlabDma), the window round trip
// and the f removed rows.
// Valid for f <= 32 with a + 1 <= H and f - a + 1 <= H (a = N/2 - R/2, H = 5 or 17); the dispatcher
// falls back to consensus_fast_f32.hip otherwise.
//
// svoc-hipcc-flags: -fno-slp-vectorize
// (ROCm 7.2's SLP vectorizer turns the 64-key register arrays into <2 x i32> groups whose instruction
// selection crashes clang; the packed math here is written with explicit f32x2 types anyway.)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "svoc/bufload.hpp"
#include "svoc/launch.hpp"
#include "svoc/slabdma.hpp"
#include "svoc/rankmask.hpp"
#include "svoc/sortnet.hpp"
#include "svoc/status.hpp"

namespace svoc {

// Constrained keys: values validated to [0, 1] (sign bit clear, or -0.0: key 0, just below +0.0) ->
// key = bits ^ 0x80000000, one XOR each way.  General keys: f32_key / key_f32.
template <bool CONS>
SVOC_DEV uint32_t fkey(uint32_t raw) {
  if constexpr (CONS) return raw ^ 0x80000000u;
  else return f32_key(raw);
}
template <bool CONS>
SVOC_DEV float fkey_val(uint32_t k) {
  if constexpr (CONS) return __builtin_bit_cast(float, k ^ 0x80000000u);
  else return key_f32(k);
}
SVOC_DEV float u2f(uint32_t w) { return __builtin_bit_cast(float, w); }
SVOC_DEV uint32_t f2u(float v) { return __builtin_bit_cast(uint32_t, v); }

// wt < zt ? wt : ~0
SVOC_DEV uint32_t winf_cand(uint32_t wt, uint32_t zt) {
  const uint32_t d = __builtin_elementwise_sub_sat(zt, wt);
  return wt | (__builtin_elementwise_min(d, 1u) - 1u);
}

// Skewness / sample-adjusted excess kurtosis (math.cairo:320-363) of n values from power sums of
// d = x - shift, combined in fp64; false for zero variance (the contract's sqrt(0) -> div-by-zero).  The
// n-only factors are formed once per instance (MomKd): per column two fp64 divisions and a square root remain
// of the nine divisions of the direct formulas.
struct MomKd {
  double n, in, k3, k4a, k4b, ik4c;
};
SVOC_DEV MomKd mom_kd(double n) {
  return MomKd{n, 1.0 / n, n / ((n - 1.0) * (n - 2.0)), n * (n + 1.0) / (n - 1.0), 3.0 * (n - 1.0) * (n - 1.0),
               1.0 / ((n - 2.0) * (n - 3.0))};
}
SVOC_DEV bool moments_from_sums_d(const MomKd& K, double t1, double t2, double t3, double t4, double& dl, float& sk,
                                  float& ku) {
#pragma clang fp contract(off)   // (as the kernels: every instantiation rounds the same way)
  dl = t1 * K.in;
  const double e2 = t2 * K.in, e3 = t3 * K.in, e4 = t4 * K.in;
  const double mu2 = e2 - dl * dl;
  const double mu3 = e3 - 3.0 * dl * e2 + 2.0 * dl * dl * dl;
  const double mu4 = e4 - 4.0 * dl * e3 + 6.0 * dl * dl * e2 - 3.0 * dl * dl * dl * dl;
  sk = 0.f;
  ku = 0.f;
  if (!(mu2 > 0.0)) return false;
  const double r = 1.0 / mu2;
  sk = (float)(K.n * mu3 * r / sqrt(mu2) * K.k3);
  ku = (float)((K.n * mu4 * (r * r) * K.k4a - K.k4b) * K.ik4c);
  return true;
}

// qr partials: every lane accumulates (x - c1)^2 of its 64 rows (rows 2m, 2m + 1 as one packed pair)
// over all the columns it visits in phase A, with the column's power sums of d = x - c1 on the way
// (v_pk_add / v_pk_fma); the rows' sums across the wave's P column lanes are formed once, after phase
// A, by the transposing butterfly qr_halve (stage MSK exchanges with lane ^ MSK and halves the row set:
// the lane ends with the KEEP = 64 / P row sums its "base" slot names).
// MASKW: slab with columns past D (mw = 0 there: words +0, centre +0); MASKROWS: rows >= N (read as 0)
// masked out of the power sums (their qr partials are never read).
template <int MSK, int H>
SVOC_DEV void qr_halve(float (&part)[64], int lane) {
  if constexpr (MSK >= 1) {
    const bool up = (lane & MSK) != 0;
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const float lo_v = part[i], hi_v = part[i + H];
      const float send = up ? lo_v : hi_v;
      const float keep = up ? hi_v : lo_v;
      part[i] = keep + xor_lane<MSK>(send);
    }
    qr_halve<MSK / 2, H / 2>(part, lane);
  }
}
template <bool MASKW, bool MASKROWS>
SVOC_DEV void qr_moments_regs(const RawRows& xs, int nvl, float c, uint32_t mw, f32x2 (&acc)[32],
                              f32x2& s1, f32x2& s2, f32x2& s3, f32x2& s4) {
#pragma clang fp contract(off)   // (explicit fmas only: the fused and plain instantiations must round alike)
  // (rows 2m, 2m + 1 as one packed pair: the slab copy's ds_read2st64 lands them in adjacent registers, so
  // the pair is a v_pk operand without the v_mov that pairing rows m, m + 32 needed)
#pragma unroll
  for (int m = 0; m < 32; ++m) {
    const uint32_t r0 = xs.at(2 * m), r1 = xs.at(2 * m + 1);
    const uint32_t w0 = MASKW ? r0 & mw : r0, w1 = MASKW ? r1 & mw : r1;
    f32x2 y = f32x2{u2f(w0), u2f(w1)} - f32x2{c, c};
    f32x2 q = y * y;
    acc[m] += q;
    if (MASKROWS) {
      const uint32_t m0 = lt_mask(2 * m, nvl), m1 = lt_mask(2 * m + 1, nvl);
      const float y0 = y.x, y1 = y.y, q0 = q.x, q1 = q.y;
      y = f32x2{fand(y0, m0), fand(y1, m1)};
      q = f32x2{fand(q0, m0), fand(q1, m1)};
    }
    s1 += y;
    s2 += q;
    s3 = __builtin_elementwise_fma(q, y, s3);
    s4 = __builtin_elementwise_fma(q, q, s4);
  }
}

// the lane's KEEP row sums of a packed partial set (qr_halve across the wave's P column lanes)
template <int P>
SVOC_DEV void qr_keep(const f32x2 (&a)[32], int lane, float (&keep)[64 / P], bool add) {
  float part[64];
#pragma unroll
  for (int m = 0; m < 32; ++m) {
    part[2 * m] = a[m].x;
    part[2 * m + 1] = a[m].y;
  }
  qr_halve<P / 2, 32>(part, lane);
#pragma unroll
  for (int i = 0; i < 64 / P; ++i) keep[i] = add ? keep[i] + part[i] : part[i];
}

// window_group_pruned for N = 256 (H = 17, one window part of H keys per lane); `wk` sized by the
// caller's instantiation (the template parameter keeps the call dependent, so other widths compile).
// e0 / e63: the lane's smallest and largest key (the in-lane sort's ends), for the fused interval check.
template <int P, int H, int WN>
SVOC_DEV bool try_pruned(uint32_t (&r)[64], int seg, int lane, uint32_t (&w)[WN], uint32_t& lo, uint32_t& hi,
                         uint32_t& e0, uint32_t& e63) {
  if constexpr (WN == H && H == 17) {
    bool ok;
    sort_oem<64>(r);
    e0 = r[0];
    e63 = r[63];
    window_group_pruned_sorted<P, H>(r, seg, lane, w, lo, hi, ok);
    return ok;
  } else {
    return false;
  }
}

// One workgroup per instance.  Phase A streams the instance through LDS one WAVES * P-column slab at a
// time: wait for the slab's DMA + barrier, every lane copies its column's 64 rows (its lane-group
// segment) into registers (raw values and sort keys), barrier, the next slab's DMA is issued, and the
// network, window, c1 and qr pass run on the registers while it lands.  2 waves per SIMD (<= 256
// VGPRs: 64 keys + 64 raw rows + the window), LDS = WAVES x 16 KiB.

template <int NSEG, int WAVES, int H, bool CONS, int MODE, bool FUSED = false>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(2))) void consensus_fast_winf_kernel(FastParams p) {
  // (no implicit fma contraction: the fused-streaming and plain instantiations compile their arithmetic in
  // different contexts and must still round alike -- tests/test_fast_transactional.py compares them bit for bit)
#pragma clang fp contract(off)
  constexpr int P = 64 / NSEG;          // columns per wave (phase A)
  constexpr int NPAD = 64 * NSEG;
  constexpr int W = WAVES * P;          // columns per workgroup step (phase A)
  constexpr int NT = WAVES * 64;
  constexpr int KEEP = 64 / P;
  constexpr bool PASS1 = MODE != 2;
  __shared__ uint32_t slab[PASS1 ? WAVES * 64 * 64 : 1];   // one 16-KiB DMA region per wave
  __shared__ __attribute__((aligned(16))) float qr_part[WAVES * NPAD];   // (then the rank keys: 2 NPAD words)
  __shared__ float qr_lds[NPAD];
  __shared__ uint64_t relmask[4];
  __shared__ int urow[32];      // removed rows, index order
  __shared__ float misc_f[2];
  __shared__ int misc_i[3];     // status, zero-variance flag, cleanup list length
  __shared__ uint32_t redo[128];   // constrained, D <= 4096: the cleanup columns as a bit mask
  // fused transactional streaming (FastParams.upd_rows): row -> its update's slot in this instance's batch
  // (-1: the state row), and the slots whose row failed the interval check
  __shared__ int smap[FUSED ? NPAD : 1];
  __shared__ uint32_t badu[8];

  const int b = blockIdx.x;
  static_assert(!FUSED || (MODE == 0 && CONS), "fused streaming: whole constrained rounds");
  constexpr bool fused = FUSED;
  const int U = fused ? p.upd_per_inst : 0;
  if (p.active && !p.active[b]) {
    // (the fused path runs only when every instance is active; an inactive one would not commit)
    for (int t = threadIdx.x; t < U; t += WAVES * 64) p.upd_status[(int64_t)b * U + t] = ST_NOT_ACTIVE;
    return;
  }
  // (wave made explicitly uniform: it feeds the DMA's M0 and SGPR row offsets)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < 32) urow[tid] = 0;  // f < 32: unused slots still name a valid row
  if (tid == 0) misc_i[2] = 0;
  if (tid < 128) redo[tid] = 0u;
  const int seg = lane / P, cw = lane % P;
  const int N = p.N, D = p.D;
  const int rowb = p.ld * 4;
  const float* inst = (const float*)p.values + (int64_t)b * p.inst_stride;
  const __amdgpu_buffer_rsrc_t rs = instance_rsrc(inst, (uint32_t)(N * rowb));
  const BufDesc rsd = buf_desc(inst, (uint32_t)(N * rowb));   // the same descriptor, for the DMA asm
  const int nslab = (D + W - 1) / W;
  const int Dc = 2 * p.work_pairs;      // workspace columns (launch.hpp: fast_work_words)
  // this instance's workspace: [H][2][Dc] window keys, at byte MOM the [4][Dc] all-row power sums, at
  // LST the [Dc] cleanup column list, at STG the [3][Dc] staged pass-2 outputs (unconstrained)
  const __amdgpu_buffer_rsrc_t ws = instance_rsrc(p.work + (int64_t)b * p.work_stride, (uint32_t)(p.work_stride * 4));
  const int MOM = 2 * H * Dc * 4;
  const int LST = MOM + 4 * Dc * 4;
  const int STG = Dc * kWinfStageCols * 4;
  // the batch rows of this instance's updates ([U, D], pitch D): rows being updated this round are read
  // from here, the state keeps the committed rows until svoc_commit_updates copies the accepted ones
  const float* urows = fused ? p.upd_rows + (int64_t)b * U * D : inst;
  const uint32_t ubytes = fused ? (uint32_t)(U * D * 4) : 0u;
  const __amdgpu_buffer_rsrc_t rb = instance_rsrc(urows, ubytes);
  const BufDesc rbd = buf_desc(urows, ubytes);
  if constexpr (FUSED) {
    for (int t = tid; t < NPAD; t += NT) smap[t] = -1;
  }
  if (tid < 8) badu[tid] = 0u;
  __syncthreads();
  if (fused)
    for (int t = tid; t < U; t += NT) {
      const int64_t o = p.upd_oracle[(int64_t)b * U + t];
      if (o >= 0 && o < N) smap[o] = t;
    }
  __syncthreads();
  // one value of row `row` (wave-uniform) at byte offset `cb` of the row: batch or state
  auto row_load = [&](int row, int cb) __attribute__((always_inline)) -> uint32_t {
    int u = -1;
    if constexpr (FUSED) u = __builtin_amdgcn_readfirstlane(smap[row]);
    return u >= 0 ? bload(rb, cb, u * D * 4) : bload(rs, cb, row * rowb);
  };
  auto bad_slot = [&](int u) __attribute__((always_inline)) { return (badu[u >> 5] >> (u & 31)) & 1u; };
  // every update's transaction status once the round's outcome is known (contract.cairo:588-603)
  auto upd_out = [&](int st) __attribute__((always_inline)) {
    if (fused)
      for (int t = tid; t < U; t += NT) {
        int s = bad_slot(t) ? ST_INTERVAL_INPUT : st;
        const int64_t o = p.upd_oracle[(int64_t)b * U + t];
        if (o < 0 || o >= N) {
          // never mapped to a row (so never interval-checked by the round): the contract's order, the
          // prediction's interval check, then the caller's oracle lookup (contract.cairo:588-596)
          s = ST_NOT_ORACLE;
          for (int d = 0; d < D; ++d) {
            const float v = urows[(int64_t)t * D + d];
            if (!(v >= 0.f && v <= 1.f)) {
              s = ST_INTERVAL_INPUT;
              break;
            }
          }
        }
        p.upd_status[(int64_t)b * U + t] = s;
      }
  };
  const int lo1 = (NPAD - N + 1) >> 1;
  const int nv = N - seg * 64;
  const int nl = N + lo1 - seg * 64;
  const uint32_t pol = group_polarity<NSEG>(seg);
  const uint32_t kp = 0x80000000u ^ pol;   // constrained key = raw ^ kp

  // qr partials of rows (m, m + 32) summed over the lane's phase-A columns, reduced across the column
  // lanes once after phase A (ACC64); the unconstrained kernels (more live registers: general key
  // mapping, two-median network) reduce them every slab into KEEP row sums instead
  constexpr bool ACC64 = CONS;
  f32x2 acc[ACC64 ? 32 : 1];
#pragma unroll
  for (int i = 0; i < (ACC64 ? 32 : 1); ++i) acc[i] = f32x2{0.f, 0.f};
  float keep[KEEP];
#pragma unroll
  for (int i = 0; i < KEEP; ++i) keep[i] = 0.f;
  int net_fallbacks = 0;   // slabs whose pruned network failed its check (wave-uniform)

  // ------------------------------------------------------------ phase A: pass 1 (contract.cairo:455-463)
  const int pass1_slabs = PASS1 ? nslab : 0;
  const SlabDma<NSEG> dma(lane, rowb);
  uint32_t* const region = slab + (PASS1 ? wave * 64 * 64 : 0);
  // this lane's words: global row seg * 64 + i at LDS row NSEG * i + seg, i.e. word 64 i + seg P + cw
  const uint32_t* const mine = region + (PASS1 ? seg * P + cw : 0);
  // fused: per-piece row sources of this lane's DMA, packed 4 per register (byte k % 4 of pmap[k / 4] =
  // batch slot + 1 of the piece's row, 0 = the state row); offsets formed at issue
  uint32_t pmap[FUSED ? 4 : 1] = {};
  auto map_pieces = [&]() __attribute__((always_inline)) {
    if constexpr (FUSED) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int row = dma.row_of(k);
        const int u = row < N ? smap[row] : -1;
        if (k % 4 == 0) pmap[k / 4] = 0u;
        pmap[k / 4] |= (uint32_t)(u + 1) << (8 * (k % 4));
      }
    }
  };
  auto issue_slab = [&](int s) __attribute__((always_inline)) {
    if constexpr (FUSED) {
      // (opaque per slab: the masks and offsets derived from the map are loop-invariant, and hoisted out of
      // the slab loop they take 32+ SGPRs / VGPRs for the whole phase -- spills)
      uint32_t pm[4] = {pmap[0], pmap[1], pmap[2], pmap[3]};
      asm volatile("" : "+v"(pm[0]), "+v"(pm[1]), "+v"(pm[2]), "+v"(pm[3]));
      int rowb_o = rowb, d4 = D * 4;
      asm volatile("" : "+s"(rowb_o), "+s"(d4));
      uint32_t* reg_o = region;
      asm volatile("" : "+s"(reg_o));
      // batch piece: slot byte u + 1 of the map -> byte offset u * D * 4 + the lane's column offset.  (24-bit
      // multiplies: a 32-bit integer product is a quarter-rate v_mad_u64_u32 here; the dispatcher keeps rows
      // and D * 4 below 2^24 bytes on this path.  A state piece's batch offset wraps below zero and is never
      // used: exec-masked.)  Per piece: the byte extract, the multiply-add and the mask compare.
      int cbm = (s * W + wave * P) * 4 + dma.colb - d4;
      asm volatile("" : "+v"(cbm));   // (one v_mad_u32_u24 per piece, not a multiply and two adds)
      dma.issue_mapped(
          rsd, rbd, reg_o, rowb_o, s * W + wave * P,
          [&](int k) { return (pm[k / 4] >> (8 * (k % 4))) & 0xffu; },
          [&](int, uint32_t fb) { return (int)__umul24(fb, (unsigned)d4) + cbm; });
    } else {
      dma.issue(rsd, region, rowb, s * W + wave * P);
    }
  };
  for (int attempt = 0; attempt < 2; ++attempt) {   // (a second pass only when a fused update was invalid)
  if (fused) map_pieces();
  if (pass1_slabs > 0) issue_slab(0);
  // One slab of phase A.  FULL: every column of the slab is < D and N = NPAD, so no masks at all; the
  // masked form serves the tail slab and padded N.  (One body per loop: reading the raw rows in two
  // branches of one loop makes the compiler demote them to scratch.)
  auto slab_body = [&](auto full_c, int s) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(full_c)::value;
    const int col = s * W + wave * P + cw;
    const bool vc = FULL || col < D;
    int nvl = nv, nll = nl;
    asm volatile("" : "+v"(nvl), "+v"(nll));
    float c1v;
    const uint32_t mW = vc ? 0xffffffffu : 0u;
    RawRows xs;        // the lane's raw rows, kept for the qr pass
    __builtin_amdgcn_s_waitcnt(0x0F70);      // vmcnt(0): this wave's pieces of slab s have landed
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      xs.lo[i] = mine[i * 64];
      xs.hi[i] = mine[(i + 32) * 64];
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);      // lgkmcnt(0): the region is read, the next slab may land
    if (s + 1 < pass1_slabs) issue_slab(s + 1);
    // interval check of the batch rows (contract.cairo:591-593, math.cairo:298-310): the lane's rows against
    // [+0, 1.0f] (state rows were checked when stored); past it (or -0.0 somewhere) the batch rows are checked one
    // by one and a failing slot is marked.  On the pruned-network path the lane's extremes come from its sorted
    // keys (after the network); elsewhere from the maximum raw word here.
    constexpr bool IV_LATE = FUSED && FULL && CONS && NSEG == 4 && H == 17;
    auto mark_bad_rows = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const int row = seg * 64 + i;
        const uint32_t raw = xs.at(i);
        if (vc && row < N && !(raw <= 0x3f800000u || raw == 0x80000000u)) {
          int u = -1;
          if constexpr (FUSED) u = smap[row];
          if (u >= 0) atomicOr(&badu[u >> 5], 1u << (u & 31));
        }
      }
    };
    if (fused && !IV_LATE) {
      uint32_t mx = 0u;
#pragma unroll
      for (int i = 0; i < 64; i += 2) mx = __builtin_elementwise_max(mx, __builtin_elementwise_max(xs.at(i), xs.at(i + 1)));
      if (__ballot(mx > 0x3f800000u) != 0) mark_bad_rows();
    }
    {
      uint32_t r[64];
      auto build_keys = [&](uint32_t kpx) __attribute__((always_inline)) {
        if (FULL || N == NPAD) {
#pragma unroll
          for (int i = 0; i < 64; ++i) r[i] = CONS ? xs.at(i) ^ kpx : fkey<CONS>(xs.at(i)) ^ pol;
        } else {
#pragma unroll
          for (int i = 0; i < 64; ++i) {
            // real rows -> key; rows >= N (read as 0) -> 0 (the first lo1) / ~0 sentinels, so the middle of
            // the padded sort is the middle of the real rows
            const uint32_t hi_m = ~lt_mask(i, nll);
            r[i] = ((fkey<CONS>(xs.at(i)) & (lt_mask(i, nvl) | hi_m)) | hi_m) ^ pol;
          }
        }
      };
      build_keys(kp);
      uint32_t klo, khi;
      if constexpr (CONS) {
        uint32_t wk[NSEG == 1 ? 2 * H : H];
        auto pruned_net = [&](auto full_c2) __attribute__((always_inline)) {
          if constexpr (NSEG == 4 && H == 17 && decltype(full_c2)::value) {
            // N = 256: the pruned network (middle 32 keys of every lane) + its exact check; a wave with any
            // failing column reruns the full network from the raw rows (sortnet.hpp window_group_pruned)
            uint32_t e0, e63;
            const bool ok = try_pruned<P, H>(r, seg, lane, wk, klo, khi, e0, e63);
            if constexpr (IV_LATE) {
              // keys = (raw ^ 0x80000000) ^ pol: the lane's raw words all in [+0, 1.0f] <=> its true keys (e0 / e63
              // XOR pol, in either order) within [0x80000000, 0xbf800000]
              const uint32_t a = e0 ^ pol, bk = e63 ^ pol;
              const uint32_t tmin = __builtin_elementwise_min(a, bk), tmax = __builtin_elementwise_max(a, bk);
              if (__ballot(tmin < 0x80000000u || tmax > 0xbf800000u) != 0) mark_bad_rows();
            }
            if (__ballot(!ok) != 0) {
              ++net_fallbacks;
              // an opaque copy of the key XOR: otherwise CSE keeps the first 64 keys alive across the
              // pruned network to reuse them here (+64 VGPRs: spills)
              uint32_t kpo = kp;
              asm volatile("" : "+v"(kpo));
              build_keys(kpo);
              window_group<NSEG, P, H>(r, seg, lane, wk, klo, khi);
            }
          } else {
            window_group<NSEG, P, H>(r, seg, lane, wk, klo, khi);
          }
        };
        pruned_net(full_c);
        if constexpr (NSEG == 1) {
#pragma unroll
          for (int m = 0; m < H; ++m) {
            bstore(ws, wk[m], col * 4, 2 * m * Dc * 4);
            bstore(ws, wk[H + m], (Dc + col) * 4, 2 * m * Dc * 4);
          }
        } else {
          constexpr int slo = NSEG == 2 ? 0 : 1;
          if (seg == slo || seg == slo + 1) {
            const int part = seg - slo;
#pragma unroll
            for (int m = 0; m < H; ++m) bstore(ws, wk[m], (part * Dc + col) * 4, 2 * m * Dc * 4);
          }
        }
      } else {
        median_group<NSEG>(r, klo, khi);
      }
      c1v = 0.5f * (fkey_val<CONS>(klo) + fkey_val<CONS>(khi));
    }
    if (seg == 0 && vc) p.c1[(int64_t)b * D + col] = c1v;
    const float cq = vc ? c1v : 0.f;
    f32x2 s1 = {0.f, 0.f}, s2 = s1, s3 = s1, s4 = s1;
    if constexpr (ACC64) {
      qr_moments_regs<!FULL, !FULL>(xs, nvl, cq, mW, acc, s1, s2, s3, s4);
    } else {
      f32x2 slab_acc[32];
#pragma unroll
      for (int i = 0; i < 32; ++i) slab_acc[i] = f32x2{0.f, 0.f};
      qr_moments_regs<!FULL, !FULL>(xs, nvl, cq, mW, slab_acc, s1, s2, s3, s4);
      qr_keep<P>(slab_acc, lane, keep, true);
    }
    float t1 = s1.x + s1.y, t2 = s2.x + s2.y, t3 = s3.x + s3.y, t4 = s4.x + s4.y;
    if constexpr (NSEG == 4) {
      t1 += xor_lane<16>(t1); t2 += xor_lane<16>(t2); t3 += xor_lane<16>(t3); t4 += xor_lane<16>(t4);
    }
    if constexpr (NSEG >= 2) {
      t1 += xor_lane<32>(t1); t2 += xor_lane<32>(t2); t3 += xor_lane<32>(t3); t4 += xor_lane<32>(t4);
    }
    if (seg == 0) {
      bstore(ws, f2u(t1), col * 4, MOM);
      bstore(ws, f2u(t2), col * 4, MOM + Dc * 4);
      bstore(ws, f2u(t3), col * 4, MOM + 2 * Dc * 4);
      bstore(ws, f2u(t4), col * 4, MOM + 3 * Dc * 4);
    }
  };
  if constexpr (PASS1) {
    const int nfull = N == NPAD ? min(D / W, pass1_slabs) : 0;
#pragma nounroll
    for (int s = 0; s < nfull; ++s) slab_body(std::true_type{}, s);
#pragma nounroll
    for (int s = nfull; s < pass1_slabs; ++s) slab_body(std::false_type{}, s);
  }
  if (!fused) break;
  __syncthreads();
  uint32_t anybad = 0u;
#pragma unroll
  for (int w = 0; w < 8; ++w) anybad |= badu[w];
  if (anybad == 0u || attempt == 1) break;
  // an update row failed the interval check: its transaction reverts alone (INTERVAL_INPUT) and the round
  // is recomputed on the state row instead (the other updates of the batch stand)
  if constexpr (FUSED) {
    for (int t = tid; t < NPAD; t += NT)
      if (smap[t] >= 0 && bad_slot(smap[t])) smap[t] = -1;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < (ACC64 ? 32 : 1); ++i) acc[i] = f32x2{0.f, 0.f};
#pragma unroll
  for (int i = 0; i < KEEP; ++i) keep[i] = 0.f;
  }   // attempts

  if (net_fallbacks && lane == 0 && p.net_fallbacks) atomicAdd(p.net_fallbacks, (unsigned)net_fallbacks);
  // ------------------------------------------------------------ qr reduction
  {
    if constexpr (ACC64) qr_keep<P>(acc, lane, keep, false);
    int base = 0;
#pragma unroll
    for (int h = 32, msk = P / 2; msk >= 1; h >>= 1, msk >>= 1) base += (lane & msk) ? h : 0;
#pragma unroll
    for (int i = 0; i < KEEP; ++i) qr_part[wave * NPAD + seg * 64 + base + i] = keep[i];
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
    // reliabilities (contract.cairo:365-368,436-439) from fp64 sums of the fp32 qr
    double s_all = 0.0, s_rel = 0.0;
    for (int t = tid; t < N; t += 64) {
      const double q = (double)qr_lds[t];
      s_all += q;
      s_rel += ((relmask[t >> 6] >> (t & 63)) & 1) ? q : 0.0;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      s_all += __shfl_xor(s_all, o);
      s_rel += __shfl_xor(s_rel, o);
    }
    if (tid == 0) {
      int st = ST_OK;
      const double rd = p.legacy ? 1.0 : (double)(p.rel_dim > 0 ? p.rel_dim : D);
      const double ms = (double)p.max_spread;
      auto rel_of = [&](double mean_qr) -> float {
        return CONS ? (float)(1.0 - 2.0 * sqrt(mean_qr / rd)) : (float)(1.0 - fmin(ms, sqrt(mean_qr)) / ms);
      };
      const float rel1 = rel_of(s_all / (double)N);
      float rel2 = 0.f;
      if (!(rel1 >= 0.f && rel1 <= 1.f)) st = ST_RELIABILITY_INTERVAL;
      else if (R < 2) st = R <= 0 ? ST_USIZE_UNDERFLOW : ST_INDEX_OOB;
      else {
        rel2 = rel_of(s_rel / (double)R);
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
    if (tid == 0) p.status[b] = misc_i[0];
    upd_out(misc_i[0]);
    return;
  }

  // ------------------------------------------------------------ zero-variance pre-check (constrained)
  // A reliable column of zero variance reverts the round (math.cairo:322,331; contract.cairo:588-603).
  // The R equal values would form a sorted run covering positions [f, N - f - 1]; when f + H <= N/2 that
  // run contains the whole window, so only columns whose window is constant qualify and only those are
  // compared against the reliable rows (as consensus_fast_win.hip).  Decided before any output is written.
  if (CONS && !p.legacy) {
    const bool inwin = f + H <= N / 2;
    int fr = 0;   // first reliable row
    for (int w = 0; w < 4; ++w)
      if (relmask[w]) { fr = 64 * w + __builtin_ctzll(relmask[w]); break; }
    bool zv = false;
#pragma nounroll
    for (int base = wave * 64; base < D; base += WAVES * 64) {
      const int col = base + lane;
      const int pc = col < D ? col : D - 1;
      bool cand = col < D;
      if (inwin) {
        // compared as values: a run of +0.0 and -0.0 is constant, but its keys differ
        const uint32_t lo = bload(ws, pc * 4, 0), hi = ~bload(ws, (Dc + pc) * 4, 0);
        cand = cand && fkey_val<true>(lo) == fkey_val<true>(hi);
      }
      if (__ballot(cand)) {   // rare: compare the reliable rows with the first one
        const float r0 = u2f(row_load(fr, pc * 4));
        for (int i = fr + 1; i < N; ++i) {
          if (!((relmask[i >> 6] >> (i & 63)) & 1)) continue;   // uniform
          cand = cand && u2f(row_load(i, pc * 4)) == r0;
        }
        zv = zv || cand;
      }
    }
    if (zv) misc_i[1] = 1;
    __syncthreads();
    if (misc_i[1]) {
      if (tid == 0) p.status[b] = ST_ZERO_VARIANCE;
      upd_out(ST_ZERO_VARIANCE);
      return;
    }
  }
  if (CONS) {
    for (int t = tid; t < N; t += NT) {
      p.reliable[(int64_t)b * N + t] = (relmask[t >> 6] >> (t & 63)) & 1;
      p.qr[(int64_t)b * N + t] = qr_lds[t];
    }
  }

  // ------------------------------------------------------------ phase B: pass 2 (contract.cairo:476-500)
  // one lane per column: the removed keys are sorted once and ranked against the window.
  // Constrained rounds with D <= 4096 (LDSO): the outputs are staged in the idle slab region and the
  // cleanup columns in an LDS bit mask, so the loop issues no global store -- and with loads only in
  // flight, the next column's words (removed rows, window, power sums, c1) are loaded while this one is
  // computed (in-order vmcnt waits).  Otherwise one column per iteration, outputs stored directly.
  const double n = (double)R;
  const MomKd mk = mom_kd(n);
  const int sh = H - 1 - (N / 2 - R / 2);   // -inf sentinels in front of the removed keys
  const int64_t ob = (int64_t)b * D;
  bool zv = false;
  constexpr int NS = CONS ? 2 * H : 32;
  constexpr int NW = CONS ? H : 1;
  struct PBWords {
    uint32_t uw[NS];          // removed rows (constrained: the 2H network slots)
    uint32_t wl[NW], wu[NW];  // window halves (constrained)
    uint32_t am[4];           // all-row power sums (phase A)
    float c1c;
  };
  auto pb_load = [&](int base, PBWords& q) __attribute__((always_inline)) {
    const int col = base + lane;
    const int pc = col < D ? col : D - 1;
    const int vo = pc * 4;
    // opaque per-iteration copies: otherwise LICM hoists the 2H slot offsets / masks out of the loop
    int shl = sh, fl = f;
    asm volatile("" : "+s"(shl), "+s"(fl));
    const int s0 = CONS ? shl : 0;
    const uint64_t realm = ((fl >= 64 ? ~0ull : (1ull << fl) - 1)) << s0;
    q.c1c = p.c1[ob + pc];
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      const int row = t - s0;
      const bool real = (realm >> t) & 1;
      q.uw[t] = 0u;
      if (CONS || real) q.uw[t] = row_load(__builtin_amdgcn_readfirstlane(urow[real ? row : 0]), vo);
    }
    if constexpr (CONS) {
#pragma unroll
      for (int m = 0; m < H; ++m) {
        q.wl[m] = bload(ws, pc * 4, 2 * m * Dc * 4);
        q.wu[m] = ~bload(ws, (Dc + pc) * 4, 2 * m * Dc * 4);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) q.am[k] = bload(ws, pc * 4, MOM + k * Dc * 4);
  };
  float* const o_lds = reinterpret_cast<float*>(slab);   // [consensus | skew | kurt | c1] x D
  const bool ldso = CONS && PASS1 && D <= 4096;         // (4 D floats fit the WAVES x 16 KiB region)
  auto pb_col = [&](auto ldso_c, int base, const PBWords& cur) __attribute__((always_inline)) {
    constexpr bool LDSO = decltype(ldso_c)::value;
    const int col = base + lane;
    const float c1c = cur.c1c;
    int shl = sh, fl = f;
    asm volatile("" : "+s"(shl), "+s"(fl));
    const int s0 = CONS ? shl : 0;
    const uint64_t realm = ((fl >= 64 ? ~0ull : (1ull << fl) - 1)) << s0;
    const uint64_t lowm = (1ull << s0) - 1;
    // removed rows' power sums of d = x - c1
    float u1 = 0.f, u2 = 0.f, u3 = 0.f, u4 = 0.f;
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      if ((realm >> t) & 1) {   // uniform
        const float y = u2f(cur.uw[t]) - c1c;
        const float q = y * y;
        u1 += y;
        u2 += q;
        u3 = __builtin_fmaf(q, y, u3);
        u4 = __builtin_fmaf(q, q, u4);
      }
    }
    float cons_v = 0.f;
    if constexpr (CONS) {
      // lower window half: position c - H + m pairs with U'[m] (lo) / U'[m - 1] (hi); upper half
      // (stored complemented, position c + H - 1 - m): U'[2H - 1 - m] (lo) / U'[2H - 2 - m] (hi)
      auto cands = [&](const auto& z) __attribute__((always_inline)) {
        uint32_t clo = ~0u, chi = ~0u;
#pragma unroll
        for (int m = 0; m < H; ++m) {
          const uint32_t wl = cur.wl[m], wu = cur.wu[m];
          clo = kmin(clo, winf_cand(wl, z(m)));
          if (m) chi = kmin(chi, winf_cand(wl, z(m - 1)));
          clo = kmin(clo, winf_cand(wu, z(2 * H - 1 - m)));
          chi = kmin(chi, winf_cand(wu, z(2 * H - 2 - m)));
        }
        cons_v = 0.5f * (fkey_val<true>(clo) + fkey_val<true>(chi));
      };
      constexpr int NF = H == 17 ? 32 : 8;   // f at the sentinel-free shape (c3: N = 256, f = 32; N = 64, f = 8)
      if (s0 == 0 && fl == NF) {   // (uniform) U' = the f sorted removed keys, then +inf: an NF-key network
        uint32_t z[NF];
#pragma unroll
        for (int t = 0; t < NF; ++t) z[t] = cur.uw[t] ^ 0x80000000u;
        sort_oem<NF>(z);
        cands([&](int t) __attribute__((always_inline)) { return t < NF ? z[t < NF ? t : 0] : ~0u; });
      } else {
        // removed keys + sentinels: U'[t], t < 2H, ascending keys
        uint32_t z[64];
#pragma unroll
        for (int t = 0; t < 64; ++t) {
          if (t < 2 * H) {
            const uint32_t mreal = 0u - (uint32_t)((realm >> t) & 1);
            const uint32_t kx = (0x80000000u & mreal) | (~mreal & (0u - (uint32_t)(((~lowm) >> t) & 1)));
            z[t] = (cur.uw[t] & mreal) ^ kx;
          } else {
            z[t] = ~0u;
          }
        }
        sort_oem<64>(z);
        cands([&](int t) __attribute__((always_inline)) { return z[t]; });
      }
    }
    // reliable rows' power sums = all-row sums (phase A) - removed rows' sums
    const double a1 = (double)u2f(cur.am[0]), a2 = (double)u2f(cur.am[1]);
    const double a3 = (double)u2f(cur.am[2]), a4 = (double)u2f(cur.am[3]);
    const double r1 = a1 - (double)u1, r2 = a2 - (double)u2, r3 = a3 - (double)u3, r4 = a4 - (double)u4;
    if (col < D) {
      // trusted: no deep cancellation in the all-minus-removed difference, and the reliable mean within
      // 2 sigma of the shift c1 (moments about a far shift cancel like (dl^2 / mu2)^2)
      const double rdl = r1 * mk.in, rmu2 = r2 * mk.in - rdl * rdl;
      const double wc = (double)p.win_cancel;
      const bool good = r2 > 0.0 && a2 <= wc * r2 && a4 <= wc * r4 && rdl * rdl <= 4.0 * rmu2;
      if constexpr (LDSO) {
        o_lds[col] = cons_v;
        o_lds[3 * D + col] = c1c;
      } else if (CONS) {
        p.consensus[ob + col] = cons_v;
        if (MODE == 0 && p.c1_out) p.c1_out[ob + col] = c1c;   // (no revert after the pre-check)
      }
      if (good) {
        double dl;
        float sk, ku;
        const bool nz = moments_from_sums_d(mk, r1, r2, r3, r4, dl, sk, ku);
        if constexpr (LDSO) {
          o_lds[D + col] = p.legacy ? 0.f : sk;
          o_lds[2 * D + col] = p.legacy ? 0.f : ku;
        } else if (CONS) {
          p.skew[ob + col] = p.legacy ? 0.f : sk;
          p.kurt[ob + col] = p.legacy ? 0.f : ku;
        } else {
          stage_out(ws, STG, Dc, 0, col, (float)((double)c1c + dl));
          stage_out(ws, STG, Dc, 1, col, p.legacy ? 0.f : sk);
          stage_out(ws, STG, Dc, 2, col, p.legacy ? 0.f : ku);
          zv |= !nz;
        }
      } else if constexpr (LDSO) {
        atomicOr(&redo[col >> 5], 1u << (col & 31));   // exact recomputation below
      } else {
        // exact recomputation over the reliable rows below (each column listed once)
        const int k = atomicAdd(&misc_i[2], 1);
        bstore(ws, (uint32_t)col, k * 4, LST);
      }
    }
  };
  if (ldso) {
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): no store in flight into the load-only loop
    PBWords cur;
    pb_load(wave * 64, cur);
#pragma nounroll
    for (int base = wave * 64; base < D; base += WAVES * 64) {
      PBWords nxt;
      if (base + WAVES * 64 < D) pb_load(base + WAVES * 64, nxt);   // uniform
      // compiler barrier: the next column's loads are issued here, not sunk to their first use after the
      // compute (the scheduler moves loads down to shorten live ranges)
      asm volatile("" ::: "memory");
      pb_col(std::true_type{}, base, cur);
      cur = nxt;
    }
  } else {
#pragma nounroll
    for (int base = wave * 64; base < D; base += WAVES * 64) {
      PBWords cur;
      pb_load(base, cur);
      pb_col(std::false_type{}, base, cur);
    }
  }
  if (!CONS && zv && !p.legacy) misc_i[1] = 1;
  __syncthreads();
  // cleanup: one wave per listed column, lanes stride the rows, two-pass wave reductions
  // (math.cairo:320-363): the reliable mean first, then the power sums about it (no cancellation)
  // (ldso: the columns of the LDS bit mask in index order, dealt round-robin to the waves)
  auto cleanup_col = [&](int col) __attribute__((always_inline)) {
      const float cc = p.c1[ob + col];
      const float* xc = inst + col;
      float y[NSEG];
      float t1 = 0.f;
#pragma unroll
      for (int g = 0; g < NSEG; ++g) {
        const int i = g * 64 + lane;
        const bool use = i < N && ((relmask[g] >> lane) & 1);
        float xv = 0.f;
        if (use) {
          int u = -1;
          if constexpr (FUSED) u = smap[i];
          xv = u >= 0 ? urows[(int64_t)u * D + col] : xc[(int64_t)i * p.ld];
        }
        y[g] = use ? xv - cc : 0.f;
        t1 += y[g];
      }
      t1 += xor_lane<1>(t1); t1 += xor_lane<2>(t1); t1 += xor_lane<4>(t1);
      t1 += xor_lane<8>(t1); t1 += xor_lane<16>(t1); t1 += xor_lane<32>(t1);
      const float mu = t1 / (float)R;   // reliable mean - c1
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
        double dl;
        float sk, ku;
        const bool nz = moments_from_sums_d(mk, c1s, t2, t3, t4, dl, sk, ku);
        if (CONS && ldso) {
          o_lds[D + col] = p.legacy ? 0.f : sk;
          o_lds[2 * D + col] = p.legacy ? 0.f : ku;
        } else if (CONS) {
          p.skew[ob + col] = p.legacy ? 0.f : sk;
          p.kurt[ob + col] = p.legacy ? 0.f : ku;
        } else {
          stage_out(ws, STG, Dc, 0, col, (float)((double)cc + (double)mu + dl));
          stage_out(ws, STG, Dc, 1, col, p.legacy ? 0.f : sk);
          stage_out(ws, STG, Dc, 2, col, p.legacy ? 0.f : ku);
          if (!nz && !p.legacy) misc_i[1] = 1;
        }
      }
  };
  if (ldso) {
    int k = 0;
    for (int w32 = 0; w32 < (D + 31) / 32; ++w32) {
      uint32_t bits = redo[w32];   // uniform
      while (bits) {
        const int c = __builtin_ctz(bits);
        bits &= bits - 1;
        if (k % WAVES == wave) cleanup_col(w32 * 32 + c);
        ++k;
      }
    }
    __syncthreads();
    // staged outputs -> global (16-B vectors when the rows allow it)
    const bool c1o = MODE == 0 && p.c1_out;
    if ((D & 3) == 0) {
      for (int i = tid; i < D / 4; i += NT) {
        const float4* o4 = reinterpret_cast<const float4*>(o_lds);
        reinterpret_cast<float4*>(p.consensus + ob)[i] = o4[i];
        reinterpret_cast<float4*>(p.skew + ob)[i] = o4[D / 4 + i];
        reinterpret_cast<float4*>(p.kurt + ob)[i] = o4[2 * (D / 4) + i];
        if (c1o) reinterpret_cast<float4*>(p.c1_out + ob)[i] = o4[3 * (D / 4) + i];
      }
    } else {
      for (int i = tid; i < D; i += NT) {
        p.consensus[ob + i] = o_lds[i];
        p.skew[ob + i] = o_lds[D + i];
        p.kurt[ob + i] = o_lds[2 * D + i];
        if (c1o) p.c1_out[ob + i] = o_lds[3 * D + i];
      }
    }
  } else {
    const int nredo = misc_i[2];
    if (nredo) {
      for (int k = wave; k < nredo; k += WAVES) {
        // (sc0: read through the vL1D -- the entry was written by another wave of this workgroup)
        cleanup_col((int)__builtin_amdgcn_readfirstlane(__builtin_amdgcn_raw_buffer_load_b32(ws, 0, LST + k * 4, 1)));
      }
      __syncthreads();
    }
  }
  // ------------------------------------------------------------ commit
  // (constrained: written in place -- the pre-check ruled out every revert; unconstrained: copied from
  // the staging area, only when the round succeeded)
  if (!CONS) {
    if (misc_i[1]) {
      if (tid == 0) p.status[b] = ST_ZERO_VARIANCE;
      return;
    }
    commit_staged<NT>(ws, STG, Dc, D, tid, p.consensus + ob, p.skew + ob, p.kurt + ob);
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
  upd_out(ST_OK);
}

template <int NSEG, int WAVES, int H, bool CONS>
static void launch_winf_w(const FastParams& p, hipStream_t stream) {
  if constexpr (CONS) {
    if (p.upd_rows) {   // fused transactional streaming (mode 0)
      hipLaunchKernelGGL((consensus_fast_winf_kernel<NSEG, WAVES, H, CONS, 0, true>), dim3(p.B), dim3(WAVES * 64), 0,
                         stream, p);
      return;
    }
  }
  if (p.mode == 1) hipLaunchKernelGGL((consensus_fast_winf_kernel<NSEG, WAVES, H, CONS, 1>), dim3(p.B), dim3(WAVES * 64), 0, stream, p);
  else if (p.mode == 2) hipLaunchKernelGGL((consensus_fast_winf_kernel<NSEG, WAVES, H, CONS, 2>), dim3(p.B), dim3(WAVES * 64), 0, stream, p);
  else hipLaunchKernelGGL((consensus_fast_winf_kernel<NSEG, WAVES, H, CONS, 0>), dim3(p.B), dim3(WAVES * 64), 0, stream, p);
}

// 4-wave workgroups: 64 KiB of LDS slab each, two workgroups per CU (2 waves per SIMD) -- one's
// barriers and slab-0 load overlap the other's compute.  (A 2-wave form with two DMA regions per wave,
// one wave per SIMD, measured slower: c3 fp32 rounds 1944 vs 1796 us per 1024 instances, c2 fp32
// 8.1 M vs 10.1 M rounds/s -- profiles/r4_winf_dbuf_ab.txt.)
template <int NSEG, int H, bool CONS>
static void launch_winf_c(const FastParams& p, hipStream_t stream) {
  launch_winf_w<NSEG, 4, H, CONS>(p, stream);
}

template <int NSEG>
static void launch_winf(const FastParams& p, int H, hipStream_t stream) {
  if (!p.constrained) launch_winf_c<NSEG, 5, false>(p, stream);   // no window: H = 5 keeps the layout
  else if (H == 5) launch_winf_c<NSEG, 5, true>(p, stream);
  else launch_winf_c<NSEG, 17, true>(p, stream);
}

}  // namespace svoc

using namespace svoc;

// Returns -2 when the window kernel does not apply (no workspace, f > 32, N > 256, ...): the caller
// falls back to the two-network fp32 kernel.
extern "C" int svoc_fast_round_f32_win(const FastParams* p, hipStream_t stream) {
  if (p->B <= 0) return 0;
  if (!p->work || p->N < 2 || p->N > 256 || p->D > p->ld) return -2;
  if ((int64_t)p->N * p->ld * 4 >= (1ll << 31)) return -2;
  if (p->mode == 2 && p->work_fresh) return -2;   // pass 1 ran elsewhere: no windows to read
  if (p->upd_rows && (p->mode != 0 || !p->constrained || p->upd_per_inst <= 0 || p->upd_per_inst > 256 ||
                      (int64_t)p->upd_per_inst * p->D * 4 >= (1ll << 31) || (int64_t)p->ld * 4 >= (1ll << 24)))
    return -3;
  if (p->n_failing < 0 || p->n_failing > 32 || p->n_failing > p->N - 2) return -2;
  const int H = fast_win_h(p->N, p->n_failing);
  if (H == 0) return -2;
  if (p->work_pairs < fast_work_pairs(p->D) || p->work_pairs % 256 != 0 || p->work_stride < fast_work_words(p->D))
    return -1;
  if (p->N <= 64) launch_winf<1>(*p, H, stream);
  else if (p->N <= 128) launch_winf<2>(*p, H, stream);
  else launch_winf<4>(*p, H, stream);
  return (int)hipGetLastError();
}
