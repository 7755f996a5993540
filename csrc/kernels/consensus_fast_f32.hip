// Fast-mode consensus round over fp32 STORAGE (reference resolution): one workgroup per instance,
// one lane per column.
//
// Why a separate kernel: the bf16 kernels (consensus_fast_win / _reg / _small) sort two 16-bit keys
// per VGPR (v_pk_min_u16); bf16 quantises [0, 1] values to 2^-9..2^-8, three orders of magnitude
// coarser than the contract's 1e-6 wsad grid (signed_decimal.cairo:82-83).  fp32 keeps 24 bits
// (<= 6e-8 absolute on [0, 1]: every wsad value keeps its own rounding interval), so this path
// selects the same oracles as the exact engine on data the fp32 grid separates
// (tests/test_f32_gpu.py pins fast-fp32 against the exact wsad kernel).
//
// Semantics: contract/src/contract.cairo:442-503 (constrained) and :370-434 (unconstrained), in the
// fast engine's real-unit form (csrc/engine/reference_cpu.cpp:fast_round_one, its CPU twin):
//   pass 1: c1 = smooth median per column (ranks N/2 - 1, N/2; math.cairo:113-126), qr_i =
//           sum_d (x_id - c1_d)^2 (math.cairo:225-238), rel1 from mean(qr) (contract.cairo:436-439);
//   rank mask (qr asc, idx desc; sort.cairo:96-101) keeps N - f rows;
//   pass 2: consensus = smooth median (constrained) / mean (unconstrained) of the reliable rows, rel2
//           from their qr, population variance, sample-adjusted skewness / excess kurtosis
//           (math.cairo:320-398).
//
// MI355X mapping (the column-parallel layout of consensus_wsad.hip with float math):
//   * lane = column; NSEG = ceil(N / 64) lanes share a column for N > 64 (64 rows per lane; N <= 1024);
//     row offsets ride in SGPR soffsets of one buffer resource per instance (no address VGPRs);
//   * fp32 -> order-preserving u32 key (sign-magnitude flip); median_group (sortnet.hpp) finds the
//     two middle order statistics; rows >= N (and unreliable rows in pass 2) become 0 / ~0
//     sentinels split so the middle pair lands on the real middle ranks -- no per-row masks in the
//     network;
//   * qr partials: a transposing butterfly over the wave's columns (DPP / ds_swizzle / permlane32),
//     per-oracle sums in LDS, deterministic (no atomics);
//   * pass 2 reads each column ONCE: the sort keys and, from the same registers, the reliable rows'
//     power sums shifted by the pass-1 median plus their min / max key (a constant column -- zero
//     variance -- is decided exactly, as by the CPU twin); a column whose mean sits far from c1
//     relative to its spread is re-read once with the shift at its mean (cancellation guard);
//     moments combined in fp64;
//   * outputs are staged in the workspace and committed only when the round's status is OK
//     (contract.cairo:588-603: a failed assert reverts the whole transaction).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "svoc/bufload.hpp"
#include "svoc/launch.hpp"
#include "svoc/sortnet.hpp"
#include "svoc/status.hpp"


namespace svoc {

// Transposing butterfly over the wave's P columns: stage L exchanges with lane ^ (P >> L); the lane
// ends with rows I + base(lane) summed over all P columns.
template <int L, int I, int P>
SVOC_DEV float qtree_f(const float (&q)[64], int lane) {
  if constexpr (L == 0) {
    return q[I];
  } else {
    constexpr int msk = P >> L;
    const float lo_v = qtree_f<L - 1, I, P>(q, lane);
    const float hi_v = qtree_f<L - 1, I + (64 >> L), P>(q, lane);
    const bool up = (lane & msk) != 0;
    const float send = up ? lo_v : hi_v;
    const float keep = up ? hi_v : lo_v;
    return keep + xor_lane<msk>(send);
  }
}
template <int P, int... Is>
SVOC_DEV void qtree_f_all(const float (&q)[64], int lane, float* acc, std::integer_sequence<int, Is...>) {
  ((acc[Is] += qtree_f<__builtin_ctz(P), Is, P>(q, lane)), ...);
}

// The lane's 64 rows of one column, every load issued before any is consumed (64 in flight: the
// compiler otherwise interleaves each load with its consumer and keeps ~4 outstanding).
SVOC_DEV void load_col(__amdgpu_buffer_rsrc_t rs, int vo, int rowb, uint32_t (&x)[64]) {
  // opaque: the 64 row soffsets are recomputed here (s_mul), not hoisted out of the slab loops into 64
  // live SGPRs (spilled to VGPRs), and a re-read stays a re-read (not CSE'd with an earlier load of the
  // same words, which would keep 64 more VGPRs live across the sort)
  asm volatile("" : "+s"(rowb));
#pragma unroll
  for (int i = 0; i < 64; ++i) x[i] = bload(rs, vo, i * rowb);
  __builtin_amdgcn_sched_barrier(0);
}

// The two middle order statistics of the column group's 64*NSEG keys: median_group (NSEG <= 4,
// keys XOR group_polarity) or the full cross-lane bitonic sort for N up to 512 / 1024 (NSEG 8 / 16).
template <int NSEG, int P>
SVOC_DEV void col_median(uint32_t (&r)[64], int lane, uint32_t& lo, uint32_t& hi) {
  if constexpr (NSEG >= 8) median_group_wide<NSEG, P>(r, lane / P, lane, lo, hi);
  else median_group<NSEG>(r, lo, hi);
}

// 0, computed from v: a re-read whose offset adds after(v) cannot be issued before v exists.  Keeps the
// re-read loads below the sort network that produces v (LLVM otherwise hoists them above it and holds
// 64 more VGPRs across the network).  v is a median of real rows (never NaN) on every lane that
// commits; elsewhere the +4 only shifts a discarded read.
SVOC_DEV int after(float v) { return v != v ? 4 : 0; }

template <int NSEG, int P, class T>
SVOC_DEV T seg_sum(T v) {
#pragma unroll
  for (int t = 1; t < NSEG; t <<= 1) v += __shfl_xor(v, t * P);
  return v;
}

// MODE: 0 whole round; 1 pass 1 only (c1 + this shard's qr partials); 2 from the all-reduced qr
// (D-sharding, svoc/parallel/dshard.py).
template <int NSEG, int WAVES, bool CONS, int MODE>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(1))) void consensus_fast_f32_kernel(FastParams p) {
  constexpr int P = 64 / NSEG;      // columns per wave
  constexpr int NPAD = 64 * NSEG;   // padded oracle rows
  constexpr int W = WAVES * P;      // columns per slab
  constexpr int NT = WAVES * 64;
  constexpr int KEEP = 64 / P;      // qr rows a lane holds after the butterfly
  // the raw column stays in registers across the pass-1 network (no re-read), at the waves per SIMD
  // that register budget allows (capping at 128 VGPRs spilled and lost: profiles/r2_f32_wpe_ab.txt,
  // r2_f32_keep_raw_ab.txt, r2_f32_raw_nseg_ab.txt)
  constexpr bool KEEP_RAW = true;
  __shared__ float qr_part[WAVES * NPAD];
  __shared__ float qr_lds[NPAD];
  constexpr int NM = NSEG < 4 ? 4 : NSEG;   // 64-row mask words
  __shared__ uint64_t relmask[NM], lowmask[NM];
  __shared__ float rels[2];
  __shared__ int st_sh, zv_sh;

  const int b = blockIdx.x;
  if (p.active && !p.active[b]) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = p.N, D = p.D;
  if (p.n_failing > N) {   // reference_cpu.cpp fast_round_one: checked before anything is computed
    if (tid == 0) p.status[b] = ST_USIZE_UNDERFLOW;
    return;
  }
  if (tid == 0) zv_sh = 0;
  const int seg = lane / P, cw = lane % P;
  const int rowb = p.ld * 4;
  const __amdgpu_buffer_rsrc_t rs =
      instance_rsrc((const float*)p.values + (int64_t)b * p.inst_stride, (uint32_t)(N * rowb));
  const int nslab = (D + W - 1) / W;
  const int lo1 = (NPAD - N + 1) >> 1;   // pass-1 sentinel split (rows >= N): low keys first, then high
  const int nv = N - seg * 64;           // this lane's rows < nv are real
  const int nl = N + lo1 - seg * 64;
  const int seg_off = seg * 64 * rowb;
  const uint32_t pol = group_polarity<NSEG>(seg);

  float acc[KEEP];
#pragma unroll
  for (int k = 0; k < KEEP; ++k) acc[k] = 0.f;

  // ------------------------------------------------------------ pass 1 (contract.cairo:455-463)
#pragma nounroll
  for (int s = 0; s < (MODE == 2 ? 0 : nslab); ++s) {
    const int col = s * W + wave * P + cw;
    const bool vc = col < D;
    const int vo = seg_off + (vc ? col : 0) * 4;
    int nvl = nv, nll = nl;
    asm volatile("" : "+v"(nvl), "+v"(nll));   // opaque per slab: stop LICM from hoisting 64 row masks
    float c1;
    float q[64];
    const uint32_t vcm = vc ? 0xffffffffu : 0u;
    if constexpr (KEEP_RAW) {
      // the raw column stays in registers across the sort: no re-read for the quadratic risk
      uint32_t xs[64], r[64];
      load_col(rs, vo, rowb, xs);
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const uint32_t mr = lt_mask(i, nvl), ml1 = lt_mask(i, nll);
        r[i] = ((f32_key(xs[i]) & mr) | (~mr & ~ml1)) ^ pol;
      }
      uint32_t lo, hi;
      col_median<NSEG, P>(r, lane, lo, hi);
      c1 = 0.5f * (key_f32(lo) + key_f32(hi));
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const float y = __builtin_bit_cast(float, xs[i]) - c1;
        q[i] = fand(y * y, vcm & lt_mask(i, nvl));
      }
      if (seg == 0 && vc) p.c1[(int64_t)b * D + col] = c1;
    } else {
      {
        uint32_t r[64];
        load_col(rs, vo, rowb, r);
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          // arithmetic masks, no per-row branches: real -> key, rows >= N -> 0 (first lo1) / ~0
          const uint32_t mr = lt_mask(i, nvl), ml1 = lt_mask(i, nll);
          r[i] = ((f32_key(r[i]) & mr) | (~mr & ~ml1)) ^ pol;
        }
        uint32_t lo, hi;
        col_median<NSEG, P>(r, lane, lo, hi);
        c1 = 0.5f * (key_f32(lo) + key_f32(hi));
      }
      if (seg == 0 && vc) p.c1[(int64_t)b * D + col] = c1;
      __builtin_amdgcn_sched_barrier(0);
      // quadratic risk partials of this column (math.cairo:225-238), summed over the wave's columns
      uint32_t xr[64];
      load_col(rs, vo + after(c1), rowb, xr);
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const float y = __builtin_bit_cast(float, xr[i]) - c1;
        q[i] = fand(y * y, vcm & lt_mask(i, nvl));   // a mask, not a multiply: columns past D may hold anything
      }
    }
    qtree_f_all<P>(q, lane, acc, std::make_integer_sequence<int, KEEP>{});
  }
  {
    int base = 0;
#pragma unroll
    for (int h = 32, msk = P / 2; msk >= 1; h >>= 1, msk >>= 1) base += (lane & msk) ? h : 0;
#pragma unroll
    for (int k = 0; k < KEEP; ++k) qr_part[wave * NPAD + seg * 64 + base + k] = acc[k];
  }
  __syncthreads();
  for (int t = tid; t < NPAD; t += NT) {
    float v = 0.f;
    if (MODE == 2) {
      v = t < N ? p.qr[(int64_t)b * N + t] : 0.f;
    } else {
#pragma unroll
      for (int w = 0; w < WAVES; ++w) v += qr_part[w * NPAD + t];
    }
    qr_lds[t] = v;
  }
  __syncthreads();
  if (MODE == 1) {   // D-sharding, first half: this shard's qr partials out (c1 already written)
    for (int t = tid; t < N; t += NT) p.qr[(int64_t)b * N + t] = qr_lds[t];
    if (tid == 0) p.status[b] = ST_OK;
    return;
  }

  // ------------------------------------------------------------ rank mask (contract.cairo:345-363)
  const int R = N - p.n_failing;
  for (int base = 0; base < NPAD; base += NT) {
    const int t = base + tid;
    bool rel = false;
    if (t < N) {
      const float myq = qr_lds[t];
      int rank = 0;
      for (int j = 0; j < N; ++j) {
        const float qj = qr_lds[j];
        rank += (qj < myq || (qj == myq && j > t)) ? 1 : 0;   // (qr asc, idx desc)
      }
      rel = rank < R;
    }
    const uint64_t bal = __ballot(rel);
    if (lane == 0 && (t >> 6) < NM) relmask[t >> 6] = bal;
  }
  __syncthreads();
  if (tid == 0) {
    // reliabilities in fp64 over the fp32 qr, in the CPU twin's order (reference_cpu.cpp:224-243)
    double s_all = 0.0, s_rel = 0.0;
    for (int t = 0; t < N; ++t) {
      s_all += (double)qr_lds[t];
      if ((relmask[t >> 6] >> (t & 63)) & 1) s_rel += (double)qr_lds[t];
    }
    const double rd = p.legacy ? 1.0 : (double)(p.rel_dim > 0 ? p.rel_dim : D);
    const double ms = (double)p.max_spread;
    auto rel_of = [&](double mean_qr) -> float {
      return CONS ? (float)(1.0 - 2.0 * sqrt(mean_qr / rd)) : (float)(1.0 - fmin(ms, sqrt(mean_qr)) / ms);
    };
    int st = ST_OK;
    const float rel1 = rel_of(s_all / (double)N);
    float rel2 = 0.f;
    if (!(rel1 >= 0.f && rel1 <= 1.f)) st = ST_RELIABILITY_INTERVAL;
    else if (R < 2) st = R == 0 ? ST_USIZE_UNDERFLOW : ST_INDEX_OOB;
    else {
      rel2 = rel_of(s_rel / (double)R);
      if (!(rel2 >= 0.f && rel2 <= 1.f)) st = ST_RELIABILITY_INTERVAL;
      else if (R < 4 && !p.legacy) st = ST_TOO_FEW_RELIABLE;
    }
    rels[0] = rel1;
    rels[1] = rel2;
    st_sh = st;
    // pass-2 sentinel split: the first (NPAD - R + 1) / 2 non-reliable rows (row order) sort low
    int need = (NPAD - R + 1) >> 1;
    for (int w = 0; w < NM; ++w) {
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
  __syncthreads();
  if (st_sh != ST_OK) {
    if (tid == 0) p.status[b] = st_sh;
    return;   // revert: outputs untouched
  }

  // ------------------------------------------------------------ pass 2 (contract.cairo:476-500)
  const int Dp = p.work_pairs, D2 = 2 * Dp;
  const int STG = Dp * (2 * 17 + 8 + 2) * 4;   // launch.hpp: fast_work_stage_word
  const __amdgpu_buffer_rsrc_t ws = instance_rsrc(p.work + (int64_t)b * p.work_stride, (uint32_t)(p.work_stride * 4));
  const uint64_t mymask = relmask[seg];
  const uint64_t mylow = lowmask[seg];
  int first_rel = 0;   // N <= 64 unconstrained: the power sums are shifted by the first reliable row
  if (!CONS && NSEG == 1) {
    if (relmask[0]) first_rel = __builtin_ctzll(relmask[0]);
    first_rel = __builtin_amdgcn_readfirstlane(first_rel);
  }
  const double n = (double)R, inv_n = 1.0 / n;
  const double k3 = n / ((n - 1.0) * (n - 2.0));
  const double k4a = n * (n + 1.0) / (n - 1.0), k4b = 3.0 * (n - 1.0) * (n - 1.0), k4c = (n - 2.0) * (n - 3.0);
  bool zv = false;
#pragma nounroll
  for (int s = 0; s < nslab; ++s) {
    const int col = s * W + wave * P + cw;
    const bool vc = col < D;
    const int vo = seg_off + (vc ? col : 0) * 4;
    uint64_t mm = mymask, ml = mylow;
    asm volatile("" : "+v"(mm), "+v"(ml));   // keep the 64 row masks out of the slab loop's live set
    float sh = 0.f;       // constrained: the pass-2 smooth median (the consensus)
    bool constant;        // every reliable value equal (zero variance, decided exactly)
    double shift, s1, s2, s3, s4;   // power sums of the reliable rows about `shift`
    if constexpr (NSEG == 1) {
      // N <= 64: median first, then one re-read for the moments (the one-read form below costs this
      // instantiation ~250 VGPRs: the pruned 64-key network does not stream)
      // shift of the power sums: the pass-2 median (constrained) or the first reliable row's value --
      // inside the reliable cluster, and equal to every value of a constant column (zero variance exact)
      float s1f = 0.f, s2f = 0.f, s3f = 0.f, s4f = 0.f;
      if constexpr (CONS && KEEP_RAW) {
        // the raw column stays in registers across the median network: no re-read for the moments
        uint32_t xs[64], r[64];
        load_col(rs, vo, rowb, xs);
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          const uint32_t mk = bit_mask(mm, i), low = bit_mask(ml, i);
          r[i] = ((f32_key(xs[i]) & mk) | (~low & ~mk)) ^ pol;
        }
        uint32_t lo, hi;
        col_median<NSEG, P>(r, lane, lo, hi);
        sh = 0.5f * (key_f32(lo) + key_f32(hi));
        uint64_t mm2 = mymask;
        asm volatile("" : "+v"(mm2));
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          const float y = fand(__builtin_bit_cast(float, xs[i]) - sh, bit_mask(mm2, i));
          const float y2 = y * y;
          s1f += y;
          s2f += y2;
          s3f = __builtin_fmaf(y2, y, s3f);
          s4f = __builtin_fmaf(y2, y2, s4f);
        }
      } else {
        if constexpr (CONS) {
          uint32_t r[64];
          load_col(rs, vo, rowb, r);
#pragma unroll
          for (int i = 0; i < 64; ++i) {
            const uint32_t mk = bit_mask(mm, i), low = bit_mask(ml, i);
            r[i] = ((f32_key(r[i]) & mk) | (~low & ~mk)) ^ pol;   // reliable: key; else low (0) / high (~0)
          }
          uint32_t lo, hi;
          col_median<NSEG, P>(r, lane, lo, hi);
          sh = 0.5f * (key_f32(lo) + key_f32(hi));
        } else {
          sh = __builtin_bit_cast(float, bload(rs, (vc ? col : 0) * 4, first_rel * rowb));
        }
        uint64_t mm2 = mymask;
        asm volatile("" : "+v"(mm2));   // a fresh copy: no row mask CSE'd across the sort (64 live VGPRs)
        __builtin_amdgcn_sched_barrier(0);
        // shifted power sums of the reliable rows (one re-read of the column, L2-resident); y = x - sh is
        // 0 exactly for every row of a constant column, so its variance is exactly 0, as the CPU twin's
        uint32_t xr[64];
        load_col(rs, vo + after(sh), rowb, xr);
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          const float y = fand(__builtin_bit_cast(float, xr[i]) - sh, bit_mask(mm2, i));
          const float y2 = y * y;
          s1f += y;
          s2f += y2;
          s3f = __builtin_fmaf(y2, y, s3f);
          s4f = __builtin_fmaf(y2, y2, s4f);
        }
      }
      s1 = seg_sum<NSEG, P>((double)s1f); s2 = seg_sum<NSEG, P>((double)s2f);
      s3 = seg_sum<NSEG, P>((double)s3f); s4 = seg_sum<NSEG, P>((double)s4f);
      constant = false;
      shift = (double)sh;
    } else {
      // ONE read of the column: the sort keys of pass 2 and, from the same registers, the reliable rows'
      // power sums shifted by the pass-1 median c1 (known here: written by pass 1 / the caller in mode 2)
      // plus their min / max key (a constant column is decided exactly: zero variance, as the CPU twin)
      const float c1c = vc ? p.c1[(int64_t)b * D + col] : 0.f;
      float s1f = 0.f, s2f = 0.f, s3f = 0.f, s4f = 0.f;
      uint32_t kmn = ~0u, kmx = 0u;
      {
        uint32_t r[64];
        load_col(rs, vo, rowb, r);
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          if ((i & 7) == 0) __builtin_amdgcn_sched_barrier(0);   // stream the rows: raw value -> key in place
          const uint32_t mk = bit_mask(mm, i);
          const float y = fand(__builtin_bit_cast(float, r[i]) - c1c, mk);
          const float y2 = y * y;
          s1f += y;
          s2f += y2;
          s3f = __builtin_fmaf(y2, y, s3f);
          s4f = __builtin_fmaf(y2, y2, s4f);
          const uint32_t key = f32_key(r[i]);
          kmn = min(kmn, key | ~mk);
          kmx = max(kmx, key & mk);
          if constexpr (CONS) {
            const uint32_t low = bit_mask(ml, i);
            r[i] = ((key & mk) | (~low & ~mk)) ^ pol;   // reliable: key; else low (0) / high (~0)
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (CONS) {
          uint32_t lo, hi;
          col_median<NSEG, P>(r, lane, lo, hi);
          sh = 0.5f * (key_f32(lo) + key_f32(hi));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 1; t < NSEG; t <<= 1) {
        kmn = min(kmn, (uint32_t)__shfl_xor((int)kmn, t * P));
        kmx = max(kmx, (uint32_t)__shfl_xor((int)kmx, t * P));
      }
      constant = kmn == kmx;
      s1 = seg_sum<NSEG, P>((double)s1f); s2 = seg_sum<NSEG, P>((double)s2f);
      s3 = seg_sum<NSEG, P>((double)s3f); s4 = seg_sum<NSEG, P>((double)s4f);
      shift = (double)c1c;
      // cancellation guard: when the reliable rows' mean sits far from c1 relative to their spread
      // (mean offset^2 > 16 x variance), re-read the column once with the shift at the mean
      {
        const double dl = s1 * inv_n, mu2 = s2 * inv_n - dl * dl;
        if (!constant && dl * dl > 16.0 * mu2) {
          uint64_t mm2 = mymask;
          asm volatile("" : "+v"(mm2));
          const float sh2 = (float)((double)c1c + dl);
          float t1 = 0.f, t2 = 0.f, t3 = 0.f, t4 = 0.f;
          uint32_t xr[64];
          load_col(rs, vo, rowb, xr);
#pragma unroll
          for (int i = 0; i < 64; ++i) {
            const float y = fand(__builtin_bit_cast(float, xr[i]) - sh2, bit_mask(mm2, i));
            const float y2 = y * y;
            t1 += y;
            t2 += y2;
            t3 = __builtin_fmaf(y2, y, t3);
            t4 = __builtin_fmaf(y2, y2, t4);
          }
          s1 = seg_sum<NSEG, P>((double)t1); s2 = seg_sum<NSEG, P>((double)t2);
          s3 = seg_sum<NSEG, P>((double)t3); s4 = seg_sum<NSEG, P>((double)t4);
          shift = (double)sh2;
        }
      }
    }
    // central moments from the shifted sums
    const double dl = s1 * inv_n, e2 = s2 * inv_n, e3 = s3 * inv_n, e4 = s4 * inv_n;
    const double mu2 = e2 - dl * dl;
    const double mu3 = e3 - 3.0 * dl * e2 + 2.0 * dl * dl * dl;
    const double mu4 = e4 - 4.0 * dl * e3 + 6.0 * dl * dl * e2 - 3.0 * dl * dl * dl * dl;
    if (seg == 0 && vc) {
      float sk = 0.f, ku = 0.f;
      if (!p.legacy) {
        if (constant || mu2 <= 0.0) {
          zv = true;
        } else {
          const double sd = sqrt(mu2);
          const double z3 = n * mu3 / (mu2 * sd), z4 = n * mu4 / (mu2 * mu2);
          sk = (float)(z3 * k3);
          ku = (float)((z4 * k4a - k4b) / k4c);
        }
      }
      stage_out(ws, STG, D2, 0, col, CONS ? sh : (float)(shift + dl));
      stage_out(ws, STG, D2, 1, col, sk);
      stage_out(ws, STG, D2, 2, col, ku);
    }
  }
  if (zv) zv_sh = 1;
  __syncthreads();
  // ------------------------------------------------------------ commit (a successful round only)
  if (zv_sh) {
    if (tid == 0) p.status[b] = ST_ZERO_VARIANCE;
    return;
  }
  const int64_t ob = (int64_t)b * D;
  commit_staged<NT>(ws, STG, D2, D, tid, p.consensus + ob, p.skew + ob, p.kurt + ob);
  for (int t = tid; t < N; t += NT) {
    p.reliable[(int64_t)b * N + t] = (relmask[t >> 6] >> (t & 63)) & 1;
    p.qr[(int64_t)b * N + t] = qr_lds[t];
  }
  if (tid == 0) {
    p.rel[2 * (int64_t)b] = rels[0];
    p.rel[2 * (int64_t)b + 1] = rels[1];
    p.status[b] = ST_OK;
  }
}

template <int NSEG, bool CONS>
static int launch_f32_cons(const FastParams& p, hipStream_t stream) {
  constexpr int WAVES = 4;
  auto k = consensus_fast_f32_kernel<NSEG, WAVES, CONS, 0>;
  if (p.mode == 1) k = consensus_fast_f32_kernel<NSEG, WAVES, CONS, 1>;
  if (p.mode == 2) k = consensus_fast_f32_kernel<NSEG, WAVES, CONS, 2>;
  hipLaunchKernelGGL(k, dim3(p.B), dim3(WAVES * 64), 0, stream, p);
  return (int)hipGetLastError();
}
template <int NSEG>
static int launch_f32(const FastParams& p, hipStream_t stream) {
  return p.constrained ? launch_f32_cons<NSEG, true>(p, stream) : launch_f32_cons<NSEG, false>(p, stream);
}

}  // namespace svoc

using namespace svoc;

// -1: shape / workspace outside what the kernel supports (the binding checks these first).
extern "C" int svoc_fast_round_f32(const FastParams* p, hipStream_t stream) {
  if (p->B <= 0) return 0;
  if (p->N < 2 || p->N > 4096 || p->D > p->ld || p->mode < 0 || p->mode > 2) return -1;
  if ((int64_t)p->N * p->ld * 4 >= (1ll << 31)) return -1;   // 32-bit buffer offsets
  if (p->mode != 1 && (!p->work || p->work_pairs < fast_work_pairs(p->D) || p->work_stride < fast_work_words(p->D)))
    return -1;   // pass 2 stages its outputs in the workspace
  // default: the one-network window kernel (consensus_fast_winf.hip) where it applies; wave_hint -7
  // forces this two-network kernel (tests cross-check the two)
  if (p->wave_hint != -7) {
    const int rc = svoc_fast_round_f32_win(p, stream);
    if (rc != -2) return rc;
  }
  if (p->upd_rows) return -3;   // fused transactional streaming exists in the window kernel only
  if (p->rst_saved) return -3;  // in-kernel rollback: the bf16 window kernel only
  int rc;
  if (p->N <= 64) rc = launch_f32<1>(*p, stream);
  else if (p->N <= 128) rc = launch_f32<2>(*p, stream);
  else if (p->N <= 256) rc = launch_f32<4>(*p, stream);
  else if (p->N <= 512) rc = launch_f32<8>(*p, stream);
  else if (p->N <= 1024) rc = launch_f32<16>(*p, stream);
  // N > 1024: 32 / 64 lanes per column (two / one column per wave), the same cross-lane bitonic sort
  else if (p->N <= 2048) rc = launch_f32<32>(*p, stream);
  else rc = launch_f32<64>(*p, stream);
  // c1 (mode 0 with c1_out): the window kernel commits it itself, this kernel stages it
  if (rc == 0 && p->mode == 0 && p->c1_out)
    rc = svoc_commit_rows(p->c1, p->c1_out, p->status, p->active, p->B, p->D, stream);
  return rc;
}
