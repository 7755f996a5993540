// Register-resident sorting networks for per-column order statistics on CDNA4 (wave64).
//
// Layout ("lane groups"): a column pair (two adjacent bf16 columns packed in one 32-bit VGPR as
// u16x2 sort keys) is owned by NSEG lanes; lane `seg` of the group holds rows [64*seg, 64*seg+64)
// of both columns in 64 VGPRs.  Intra-lane stages are pure VALU (v_pk_min_u16 / v_pk_max_u16 sort
// two columns per instruction); cross-lane stages exchange whole registers with the partner lane
// (lane ^ m*P, where P = 64/NSEG is the number of column pairs per wave).
//
// The network is the "flip + half-cleaner" form of bitonic sort, so every run stays ascending:
//   sort64 (21 stages) inside each lane, then for run size s = 2..NSEG segments:
//   flip across lanes seg ^ (s-1) with index reversal, half-cleaners across lanes for strides
//   s/4..1 segments, then the 6 intra-lane half-cleaner stages.
// Replaces the reference's per-column MergeSort (math.cairo:113-126 via alexandria MergeSort):
// only the order statistics' VALUES matter for the smooth median, so a data-oblivious network is
// exact.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace svoc {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

#define SVOC_DEV __device__ __forceinline__

SVOC_DEV u16x2 kmin(u16x2 a, u16x2 b) { return __builtin_elementwise_min(a, b); }
SVOC_DEV u16x2 kmax(u16x2 a, u16x2 b) { return __builtin_elementwise_max(a, b); }
SVOC_DEV uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
SVOC_DEV u16x2 as_k(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
// 32-bit keys (one column per lane: the wsad kernel's int32 values) share the networks below
SVOC_DEV uint32_t kmin(uint32_t a, uint32_t b) { return a < b ? a : b; }
SVOC_DEV uint32_t kmax(uint32_t a, uint32_t b) { return a < b ? b : a; }
SVOC_DEV uint32_t as_u32(uint32_t v) { return v; }
template <class K>
SVOC_DEV K key_from(uint32_t v) { return __builtin_bit_cast(K, v); }

// bf16 bit pattern -> order-preserving unsigned key (and back), two lanes-halves at a time.
SVOC_DEV u16x2 bf16x2_to_key(uint32_t raw) {
  u16x2 r = as_k(raw);
  u16x2 s = __builtin_bit_cast(u16x2, __builtin_bit_cast(s16x2, r) >> (short)15);
  return r ^ (s | (unsigned short)0x8000);
}
SVOC_DEV uint32_t key_to_bf16x2(u16x2 k) {
  u16x2 nk = ~k;
  u16x2 s = __builtin_bit_cast(u16x2, __builtin_bit_cast(s16x2, nk) >> (short)15);
  return as_u32(k ^ (s | (unsigned short)0x8000));
}
// Constrained inputs are validated to [0, 1] (math.cairo:298-310), i.e. sign bit clear (or -0.0):
// on that domain x ^ 0x8000 is an order-preserving bijection both ways (-0.0 -> key 0, below +0.0,
// and back to -0.0) -- one v_xor_b32 instead of the general sign-magnitude mapping.
SVOC_DEV u16x2 pos_to_key(uint32_t raw) { return as_k(raw ^ 0x80008000u); }
SVOC_DEV uint32_t key_to_pos(u16x2 k) { return as_u32(k) ^ 0x80008000u; }

// fp32 bits <-> monotone u32 key (negative values: all bits flipped; positive: sign bit set)
SVOC_DEV uint32_t f32_key(uint32_t u) { return u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u); }
SVOC_DEV float key_f32(uint32_t k) {
  return __builtin_bit_cast(float, k ^ ((uint32_t)((int32_t)~k >> 31) | 0x80000000u));
}

SVOC_DEV float bf16_lo(uint32_t w) { return __builtin_bit_cast(float, w << 16); }
SVOC_DEV float bf16_hi(uint32_t w) { return __builtin_bit_cast(float, w & 0xffff0000u); }
SVOC_DEV float fand(float x, uint32_t m) { return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, x) & m); }
typedef float f32x2 __attribute__((ext_vector_type(2)));  // packed-FP32 (v_pk_*_f32) operand
SVOC_DEV f32x2 bf16x2_to_f32x2(uint32_t w) { return f32x2{bf16_lo(w), bf16_hi(w)}; }
// (element copies first: clang 20 mis-lowers __builtin_bit_cast applied directly to x.y -- the
// second lane comes out as poison)
SVOC_DEV f32x2 fand2(f32x2 x, uint32_t m) {
  const float a = x.x, b = x.y;
  return f32x2{fand(a, m), fand(b, m)};
}

// All-ones / zero lane masks built arithmetically (no v_cmp): a compare writes a VCC/SGPR pair, and
// 64 unrolled rows of them exhaust the SGPR file (spills) and get hoisted out of loops.
// (v_bfe_i32 keeps LLVM from canonicalising the arithmetic back into icmp + select.)
SVOC_DEV uint32_t lt_mask(int i, int n) { return (uint32_t)__builtin_amdgcn_sbfe(i - n, 31, 1); }  // i < n
SVOC_DEV uint32_t bit_mask(uint64_t m, int i) {  // bit i set
  const uint32_t w = i < 32 ? (uint32_t)m : (uint32_t)(m >> 32);
  return (uint32_t)__builtin_amdgcn_sbfe((int)w, i & 31, 1);
}

SVOC_DEV u16x2 shfl_xor_k(u16x2 v, int m) { return as_k((uint32_t)__shfl_xor((int)as_u32(v), m)); }
SVOC_DEV uint32_t shfl_xor_k(uint32_t v, int m) { return (uint32_t)__shfl_xor((int)v, m); }

// Value of lane ^ M (compile-time M) without __shfl_xor's per-call lane-index arithmetic:
// DPP quad_perm for M = 1, 2 (VALU, foldable into the consumer), ds_swizzle xor-mode for 4..16,
// v_permlane32_swap for 32.
template <int M>
SVOC_DEV uint32_t xor_lane_u32(uint32_t v) {
  static_assert(M == 1 || M == 2 || M == 4 || M == 8 || M == 16 || M == 32, "xor distance");
  if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
  else if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
  else if constexpr (M <= 16) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (M << 10));
  else {
    const auto t = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (__lane_id() & 32) ? t[0] : t[1];
  }
}
template <int M>
SVOC_DEV float xor_lane(float v) { return __builtin_bit_cast(float, xor_lane_u32<M>(__builtin_bit_cast(uint32_t, v))); }
SVOC_DEV u16x2 shfl_k(u16x2 v, int src) { return as_k((uint32_t)__shfl((int)as_u32(v), src)); }
SVOC_DEV uint32_t shfl_k(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src); }

// Full ascending bitonic sort of the 64 registers of one lane (each half independently).
SVOC_DEV void sort64(u16x2 (&r)[64]) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const int l = i ^ j;
        if (l > i) {
          const u16x2 a = r[i], b = r[l];
          if ((i & k) == 0) {
            r[i] = kmin(a, b);
            r[l] = kmax(a, b);
          } else {
            r[i] = kmax(a, b);
            r[l] = kmin(a, b);
          }
        }
      }
    }
  }
}

// Batcher's odd-even merge sort of the 64 registers of one lane: 543 compare-exchanges instead of
// bitonic's 672, and when only a few outputs are consumed (the two middle order statistics) dead
// code elimination prunes it to ~414 (bitonic: 543).  The comparator list is a compile-time table;
// the fully unrolled loop indexes registers with constants only.
template <int NN>
struct CmpNet {
  static constexpr int kMax = NN * 16;  // >= comparators of Batcher's network for NN <= 64
  unsigned char a[kMax], b[kMax];
  int n;
};
template <int NN>
constexpr CmpNet<NN> make_oem() {
  CmpNet<NN> t{};
  int c = 0;
  for (int p = 1; p < NN; p <<= 1)
    for (int k = p; k >= 1; k >>= 1)
      for (int j = k % p; j + k < NN; j += 2 * k)
        for (int i = 0; i < k && i + j + k < NN; ++i)
          if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) {
            t.a[c] = (unsigned char)(i + j);
            t.b[c] = (unsigned char)(i + j + k);
            ++c;
          }
  t.n = c;
  return t;
}
// In-register odd-even merge sort of NN keys (NN a power of two <= 64).
template <int NN, class K>
SVOC_DEV void sort_oem(K (&r)[NN]) {
  constexpr CmpNet<NN> T = make_oem<NN>();
#pragma unroll
  for (int c = 0; c < T.n; ++c) {
    const K x = r[T.a[c]], y = r[T.b[c]];
    r[T.a[c]] = kmin(x, y);
    r[T.b[c]] = kmax(x, y);
  }
}
SVOC_DEV void sort64_oem(u16x2 (&r)[64]) {
  static_assert(make_oem<64>().n == 543, "odd-even merge sort of 64");
  sort_oem<64>(r);
}

// Ascending half-cleaner cascade (strides 32..1): sorts a bitonic lane-local sequence.
template <class K>
SVOC_DEV void merge64(K (&r)[64]) {
#pragma unroll
  for (int j = 32; j > 0; j >>= 1) {
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      const int l = i ^ j;
      if (l > i) {
        const K a = r[i], b = r[l];
        r[i] = kmin(a, b);
        r[l] = kmax(a, b);
      }
    }
  }
}

// Cross-lane flip: position i meets the partner's position 63-i; lower lane keeps the minima.
// (K: u16x2 = two bf16 columns per register, uint32_t = one 32-bit key)
template <class K>
SVOC_DEV void xlane_flip(K (&r)[64], int xmask, bool upper) {
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const K a = r[i], b = r[63 - i];
    const K pa = shfl_xor_k(b, xmask);  // partner's r[63-i]
    const K pb = shfl_xor_k(a, xmask);  // partner's r[i]
    r[i] = upper ? kmax(a, pa) : kmin(a, pa);
    r[63 - i] = upper ? kmax(b, pb) : kmin(b, pb);
  }
}

// Cross-lane half-cleaner: position i meets the partner's position i.
template <class K>
SVOC_DEV void xlane_hc(K (&r)[64], int xmask, bool upper) {
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const K a = r[i];
    const K p = shfl_xor_k(a, xmask);
    r[i] = upper ? kmax(a, p) : kmin(a, p);
  }
}

// Sort 64*NSEG keys (x2 columns) spread over the NSEG lanes of a group. P = pairs per wave.
template <int NSEG, int P, class K>
SVOC_DEV void sort_group(K (&r)[64], int seg) {
  sort_oem<64>(r);
#pragma unroll
  for (int s = 2; s <= NSEG; s <<= 1) {
    xlane_flip(r, (s - 1) * P, (seg & (s >> 1)) != 0);
#pragma unroll
    for (int t = s >> 2; t >= 1; t >>= 1) xlane_hc(r, t * P, (seg & t) != 0);
    merge64(r);
  }
}

// Register k (runtime, 0..63) of a lane: a 63-step v_bfi_b32 blend tree.  Written with bit
// blends, not `?:` -- LLVM folds a select between two array elements into a dynamically indexed
// load, which demotes the whole register array to scratch.
SVOC_DEV uint32_t blend(uint32_t a, uint32_t b, uint32_t m) { return (a & ~m) | (b & m); }

SVOC_DEV u16x2 reg_select(const u16x2 (&r)[64], int k) {
  uint32_t a[32];
  uint32_t m = 0u - (uint32_t)(k & 1);
#pragma unroll
  for (int j = 0; j < 32; ++j) a[j] = blend(as_u32(r[2 * j]), as_u32(r[2 * j + 1]), m);
  m = 0u - (uint32_t)((k >> 1) & 1);
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = blend(a[2 * j], a[2 * j + 1], m);
  m = 0u - (uint32_t)((k >> 2) & 1);
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = blend(a[2 * j], a[2 * j + 1], m);
  m = 0u - (uint32_t)((k >> 3) & 1);
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = blend(a[2 * j], a[2 * j + 1], m);
  m = 0u - (uint32_t)((k >> 4) & 1);
#pragma unroll
  for (int j = 0; j < 2; ++j) a[j] = blend(a[2 * j], a[2 * j + 1], m);
  m = 0u - (uint32_t)((k >> 5) & 1);
  return as_k(blend(a[0], a[1], m));
}

// Rank `rank` (0-based, runtime) of the group's sorted sequence, broadcast to every group lane.
template <int NSEG, int P>
SVOC_DEV u16x2 group_select(const u16x2 (&r)[64], int rank, int lane) {
  const u16x2 v = reg_select(r, rank & 63);
  if constexpr (NSEG == 1) {
    return v;
  } else {
    const int owner = (rank >> 6) * P + (lane % P);
    return shfl_k(v, owner);
  }
}

// The two middle order statistics of the group's sorted 64*NSEG keys when the sentinel padding has
// been split so that they sit at the fixed positions NPAD/2 - 1 and NPAD/2: no runtime register
// indexing, at most one cross-lane read per value.
template <int NSEG, int P, class K>
SVOC_DEV void middle_pair(const K (&r)[64], int seg, int lane, K& lo, K& hi) {
  if constexpr (NSEG == 1) {
    lo = r[31];
    hi = r[32];
  } else {
    constexpr int h = NSEG / 2;
    const int pw = lane % P;
    lo = shfl_k(r[63], (h - 1) * P + pw);
    hi = shfl_k(r[0], h * P + pw);
  }
}

// ---------------------------------------------------------------------------------------------
// Median selection over a lane group (the fast kernels' hot path).
//
// Cross-lane stages use the gfx950 half-exchange instructions instead of ds_bpermute: one
// v_permlane{16,32}_swap moves register x of the upper lanes and register y of the lower lanes in
// a single VALU op.  Applied to a register pair (r[2k], r[2k+1]) it leaves every lane holding the
// lower lane's value in x and the upper lane's value in y, so the compare-exchange is a plain
// min + max in every lane (no lane-dependent select), and a second swap puts the results back.
//
// Bitonic direction without selects ("polarity"): lanes whose run must be descending store their
// keys complemented (~key), so the one ascending in-lane network serves both directions.  A
// cross-lane half-cleaner meets a lower lane of polarity d and an upper lane of polarity ~d: the
// upper value is complemented after the swap (one v_not per pair), and both results leave in
// polarity d -- exactly the direction the next in-lane merge needs.
template <int XM>
SVOC_DEV void xswap(uint32_t& x, uint32_t& y) {
  static_assert(XM == 16 || XM == 32, "lane-half exchange distance");
  if constexpr (XM == 32) {
    const auto t = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    x = t[0];
    y = t[1];
  } else {
    const auto t = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    x = t[0];
    y = t[1];
  }
}

// Half-cleaner between lanes l and l ^ XM (lower lane keeps the minima); the upper lane's keys are
// in the opposite polarity.  Afterwards both lanes hold keys in the lower lane's polarity.
template <int XM, class K>
SVOC_DEV void xhc_swap(K (&r)[64]) {
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    uint32_t x = as_u32(r[2 * k]), y = as_u32(r[2 * k + 1]);
    xswap<XM>(x, y);               // x: lower lane's key, y: upper lane's key (complemented)
    y = ~y;
    const K lo = kmin(key_from<K>(x), key_from<K>(y)), hi = kmax(key_from<K>(x), key_from<K>(y));
    x = as_u32(lo);
    y = as_u32(hi);
    xswap<XM>(x, y);               // lower lanes get the minima, upper lanes the maxima
    r[2 * k] = key_from<K>(x);
    r[2 * k + 1] = key_from<K>(y);
  }
}

// Final half-cleaner of a bitonic sequence whose lower half ends at the median: the two middle
// order statistics are max(lower half) and min(upper half), so the compare-exchange results are
// folded into a running max / min instead of being written back (no swap back, no merge).
template <int XM, class K>
SVOC_DEV void xhc_middle(const K (&r)[64], K& mx, K& mn) {
  mx = key_from<K>(0u);
  mn = key_from<K>(0xffffffffu);
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    uint32_t x = as_u32(r[2 * k]), y = as_u32(r[2 * k + 1]);
    xswap<XM>(x, y);
    y = ~y;
    mx = kmax(mx, kmin(key_from<K>(x), key_from<K>(y)));
    mn = kmin(mn, kmax(key_from<K>(x), key_from<K>(y)));
  }
}

// Load-time polarity of lane-group segment `seg` (XOR it into the keys before median_group).
template <int NSEG>
SVOC_DEV uint32_t group_polarity(int seg) {
  if constexpr (NSEG == 2) return seg == 1 ? 0xffffffffu : 0u;
  else if constexpr (NSEG == 4) return (seg == 1 || seg == 2) ? 0xffffffffu : 0u;
  else return 0u;
}

// The two middle order statistics (positions NPAD/2 - 1 and NPAD/2) of the group's 64*NSEG keys,
// returned in every lane of the group.  r must hold keys XOR group_polarity<NSEG>(seg).
//   NSEG 1: odd-even merge sort, pruned by DCE to the two outputs (~414 compare-exchanges).
//   NSEG 2: full in-lane sort, final cross-lane half-cleaner folded into max / min.
//   NSEG 4: in-lane sort, stage-2 exchange (lane ^ 16) + bitonic merge, final stage folded.
template <int NSEG, class K>
SVOC_DEV void median_group(K (&r)[64], K& lo, K& hi) {
  sort_oem<64>(r);
  if constexpr (NSEG == 1) {
    lo = r[31];
    hi = r[32];
  } else {
    if constexpr (NSEG == 4) {
      xhc_swap<16>(r);
      merge64(r);
    }
    K mx, mn;
    xhc_middle<32>(r, mx, mn);               // final stage: lower half = lanes with bit 5 clear
#pragma unroll
    for (int m = 16; m <= 32; m <<= 1) {   // lanes of the group: ^16 (NSEG 4), ^32
      if (NSEG == 2 && m == 16) continue;
      mx = kmax(mx, shfl_xor_k(mx, m));
      mn = kmin(mn, shfl_xor_k(mn, m));
    }
    lo = mx;
    hi = mn;
  }
}

// The two middle order statistics for wide groups (NSEG = 8 .. 64: N up to 512 .. 4096 oracles): a
// full cross-lane bitonic sort of the 64*NSEG keys (sort_group: in-lane odd-even merge sort, then
// per merge level a cross-lane flip, cross-lane half-cleaners and an in-lane merge), then the keys
// at sorted positions NPAD/2 - 1 and NPAD/2 read from their owner lanes (middle_pair).  Keys in true
// polarity (group_polarity<NSEG> = 0 for these widths).
template <int NSEG, int P, class K>
SVOC_DEV void median_group_wide(K (&r)[64], int seg, int lane, K& lo, K& hi) {
  static_assert(NSEG == 8 || NSEG == 16 || NSEG == 32 || NSEG == 64, "wide groups");
  sort_group<NSEG, P>(r, seg);
  middle_pair<NSEG, P>(r, seg, lane, lo, hi);
}

// ---------------------------------------------------------------------------------------------
// Order-statistic windows (consensus_fast_win.hip).  Pass 2's smooth median over the reliable rows
// is an order statistic of the FULL column shifted by at most f ranks, so pass 1 keeps the H keys on
// either side of the median instead of just the middle pair, and pass 2 only ranks the f removed
// keys against that window (no second sorting network over N rows).

// Half-cleaner between lanes l and l ^ XM with XOR hooks: `iy` is XORed into the upper lane's keys
// on the way in (~0 when the upper lane is in the opposite polarity), `ox` / `oy` into the minima /
// maxima on the way out (the output polarity of the lower / upper lane).  xhc_swap<XM> is
// xhc_pol<XM>(r, ~0u, 0, 0).
template <int XM, class K>
SVOC_DEV void xhc_pol(K (&r)[64], uint32_t iy, uint32_t ox, uint32_t oy) {
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    uint32_t x = as_u32(r[2 * k]), y = as_u32(r[2 * k + 1]);
    xswap<XM>(x, y);
    y ^= iy;
    const K lo = kmin(key_from<K>(x), key_from<K>(y)), hi = kmax(key_from<K>(x), key_from<K>(y));
    x = as_u32(lo) ^ ox;
    y = as_u32(hi) ^ oy;
    xswap<XM>(x, y);
    r[2 * k] = key_from<K>(x);
    r[2 * k + 1] = key_from<K>(y);
  }
}

// The top H = 2^k + 1 keys of a bitonic in-lane sequence of 64, ascending: out[0] is the H-th
// largest, out[H-1] the maximum.  Max-only half-cleaners down to 2K = 2(H-1) keys, one split into
// the top K (sorted by a half-cleaner cascade) and the rest (whose maximum is the H-th largest).
template <int H, class K>
SVOC_DEV void bitonic_top(const K (&r)[64], K (&out)[H]) {
  constexpr int KT = H - 1;
  static_assert(KT >= 2 && KT <= 32 && (KT & (KT - 1)) == 0, "H = 2^k + 1, at most 33");
  K t[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) t[i] = r[i];
#pragma unroll
  for (int n = 64; n > 2 * KT; n >>= 1) {
#pragma unroll
    for (int i = 0; i < n / 2; ++i) t[i] = kmax(t[i], t[i + n / 2]);
  }
  K mx = kmin(t[0], t[KT]);
#pragma unroll
  for (int i = 0; i < KT; ++i) {
    const K a = t[i], b = t[i + KT];
    if (i) mx = kmax(mx, kmin(a, b));
    t[i] = kmax(a, b);
  }
#pragma unroll
  for (int j = KT / 2; j > 0; j >>= 1) {
#pragma unroll
    for (int i = 0; i < KT; ++i) {
      const int l = i ^ j;
      if (l > i) {
        const K a = t[i], b = t[l];
        t[i] = kmin(a, b);
        t[l] = kmax(a, b);
      }
    }
  }
  out[0] = mx;
#pragma unroll
  for (int i = 0; i < KT; ++i) out[i + 1] = t[i];
}

// Sorted-position window around the middle of the group's 64*NSEG keys (r holds keys XOR
// group_polarity<NSEG>(seg), sentinel-split as for median_group).  With c = NPAD/2:
//   part 0 ("lower"): w0[m] = key at sorted position c - H + m      (ascending, true keys)
//   part 1 ("upper"): w1[m] = ~(key at sorted position c + H - 1 - m) (ascending complemented keys)
// NSEG 1: both parts in the lane (w holds w0 then w1, 2H keys).  NSEG 2: part 0 in seg 0, part 1 in
// seg 1.  NSEG 4: part 0 in seg 1, part 1 in seg 2 (segs 0 and 3 compute discarded keys).  lo / hi
// (the middle pair, positions c - 1 and c, true keys) are returned in every lane of the group.
// (K: u16x2 = two bf16 columns per register, uint32_t = one fp32 column: consensus_fast_winf.hip)
template <int NSEG, int P, int H, class K>
SVOC_DEV void window_group(K (&r)[64], int seg, int lane, K (&w)[NSEG == 1 ? 2 * H : H], K& lo, K& hi) {
  sort_oem<64>(r);
  if constexpr (NSEG == 1) {
#pragma unroll
    for (int m = 0; m < H; ++m) {
      w[m] = r[32 - H + m];
      w[H + m] = ~r[32 + H - 1 - m];
    }
    lo = r[31];
    hi = r[32];
  } else {
    if constexpr (NSEG == 2) {
      xhc_pol<32>(r, ~0u, 0u, ~0u);         // seg 0: lower half (true), seg 1: upper half complemented
    } else {
      xhc_swap<16>(r);
      merge64(r);
      xhc_pol<32>(r, ~0u, 0u, 0u);          // segs 0-1: lower 128, segs 2-3: upper 128 (true keys)
      const uint32_t xm = seg >= 2 ? ~0u : 0u;
      xhc_pol<16>(r, 0u, xm, xm);           // seg 1: top of the lower half, seg 2: bottom of upper (~)
    }
    bitonic_top<H>(r, w);
    constexpr int slo = NSEG == 2 ? 0 : 1;
    const int pw = lane % P;
    lo = shfl_k(w[H - 1], slo * P + pw);
    hi = ~shfl_k(w[H - 1], (slo + 1) * P + pw);
  }
}


// ---------------------------------------------------------------------------------------------
// Pruned window network for N = 256 (NSEG = 4), with an exact verification (the c3 hot path).
//
// The window (sorted positions c - H .. c + H - 1 of the 256 keys, c = 128) lies in the middle of the
// column, so after each lane has sorted its 64 keys only its middle 32 (in-lane positions 16..47) take
// part in the cross-lane merges: the four lanes' 16 lowest keys (64 in all) and 16 highest are set
// aside, and the window is read at positions 47 .. 80 of the 128 kept keys.  That is exact whenever
// every set-aside low key is <= the kept window's lowest key and every set-aside high key >= its highest:
// then exactly 64 keys precede the kept set's position j in the full order for every window position
// (G[64 + j] = K[j]; ties included).  The caller checks `ok` and reruns the full network
// (window_group) for the wave when any column fails; on exchangeable rows a column fails with
// probability ~1e-3 (SURVEY A.3 data: Beta(20,20) honest + U(0,1) failing, f = 32: 8.6e-4).
// Versus window_group<4>: the in-lane sort is pruned to the outputs 15..48 (988 of 1086 min / max)
// and every cross-lane stage works on 32 registers instead of 64 (~620 instead of ~1240 VALU).

template <int XM, int L, class K>
SVOC_DEV void xhc_swap_n(K (&r)[L]) {
#pragma unroll
  for (int k = 0; k < L / 2; ++k) {
    uint32_t x = as_u32(r[2 * k]), y = as_u32(r[2 * k + 1]);
    xswap<XM>(x, y);
    y = ~y;
    const K lo = kmin(key_from<K>(x), key_from<K>(y)), hi = kmax(key_from<K>(x), key_from<K>(y));
    x = as_u32(lo);
    y = as_u32(hi);
    xswap<XM>(x, y);
    r[2 * k] = key_from<K>(x);
    r[2 * k + 1] = key_from<K>(y);
  }
}
template <int XM, int L, class K>
SVOC_DEV void xhc_pol_n(K (&r)[L], uint32_t iy, uint32_t ox, uint32_t oy) {
#pragma unroll
  for (int k = 0; k < L / 2; ++k) {
    uint32_t x = as_u32(r[2 * k]), y = as_u32(r[2 * k + 1]);
    xswap<XM>(x, y);
    y ^= iy;
    const K lo = kmin(key_from<K>(x), key_from<K>(y)), hi = kmax(key_from<K>(x), key_from<K>(y));
    x = as_u32(lo) ^ ox;
    y = as_u32(hi) ^ oy;
    xswap<XM>(x, y);
    r[2 * k] = key_from<K>(x);
    r[2 * k + 1] = key_from<K>(y);
  }
}
template <int L, class K>
SVOC_DEV void merge_n(K (&r)[L]) {
#pragma unroll
  for (int j = L / 2; j > 0; j >>= 1) {
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int l = i ^ j;
      if (l > i) {
        const K a = r[i], b = r[l];
        r[i] = kmin(a, b);
        r[l] = kmax(a, b);
      }
    }
  }
}
// top H = KT + 1 keys (KT = L / 2) of a bitonic in-lane sequence of L, ascending (bitonic_top for L = 2 KT)
template <int H, int L, class K>
SVOC_DEV void bitonic_top_n(const K (&r)[L], K (&out)[H]) {
  constexpr int KT = H - 1;
  static_assert(2 * KT == L, "bitonic_top_n: L = 2 (H - 1)");
  K t[KT];
  K mx = kmin(r[0], r[KT]);
#pragma unroll
  for (int i = 0; i < KT; ++i) {
    const K a = r[i], b = r[i + KT];
    if (i) mx = kmax(mx, kmin(a, b));
    t[i] = kmax(a, b);
  }
#pragma unroll
  for (int j = KT / 2; j > 0; j >>= 1) {
#pragma unroll
    for (int i = 0; i < KT; ++i) {
      const int l = i ^ j;
      if (l > i) {
        const K a = t[i], b = t[l];
        t[i] = kmin(a, b);
        t[l] = kmax(a, b);
      }
    }
  }
  out[0] = mx;
#pragma unroll
  for (int i = 0; i < KT; ++i) out[i + 1] = t[i];
}

// window_group<4, P, 17> on the middle 32 keys of every lane + the verification (see above).  r: the
// lane's 64 keys XOR group_polarity<4>(seg) (consumed).  Outputs as window_group; `ok` is the same in the
// four lanes of a group (K = u16x2: both columns of the pair must pass).
// (window_group_pruned_sorted: the same from r already sorted in-lane -- a caller that also wants the lane's
// extremes r[0] / r[63] reads them in between)
template <int P, int H, class K>
SVOC_DEV void window_group_pruned_sorted(K (&r)[64], int seg, int lane, K (&w)[H], K& lo, K& hi, bool& ok) {
  static_assert(H == 17, "pruned window: H = 17 (f <= 32 at N = 256)");
  const bool pol = seg == 1 || seg == 2;   // complemented lanes: stored ascending = true descending
  // the set-aside keys' extremes in true keys: highest of the low side, lowest of the high side
  K dl = pol ? key_from<K>(~as_u32(r[48])) : r[15];
  K dh = pol ? key_from<K>(~as_u32(r[15])) : r[48];
  K k[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) k[i] = r[16 + i];
  xhc_swap_n<16, 32>(k);
  merge_n<32>(k);
  xhc_pol_n<32, 32>(k, ~0u, 0u, 0u);
  const uint32_t xm = seg >= 2 ? ~0u : 0u;
  xhc_pol_n<16, 32>(k, 0u, xm, xm);
  bitonic_top_n<H, 32>(k, w);
  const int pw = lane % P;
  lo = shfl_k(w[H - 1], 1 * P + pw);
  hi = key_from<K>(~as_u32(shfl_k(w[H - 1], 2 * P + pw)));
  const K wlo = shfl_k(w[0], 1 * P + pw);                              // window's lowest key (true), seg 1
  const K whi = key_from<K>(~as_u32(shfl_k(w[0], 2 * P + pw)));       // window's highest key (true), seg 2
  dl = kmax(dl, key_from<K>(xor_lane_u32<16>(as_u32(dl))));
  dl = kmax(dl, key_from<K>(xor_lane_u32<32>(as_u32(dl))));
  dh = kmin(dh, key_from<K>(xor_lane_u32<16>(as_u32(dh))));
  dh = kmin(dh, key_from<K>(xor_lane_u32<32>(as_u32(dh))));
  ok = as_u32(kmax(dl, wlo)) == as_u32(wlo) && as_u32(kmin(dh, whi)) == as_u32(whi);
}
template <int P, int H, class K>
SVOC_DEV void window_group_pruned(K (&r)[64], int seg, int lane, K (&w)[H], K& lo, K& hi, bool& ok) {
  sort_oem<64>(r);
  window_group_pruned_sorted<P, H>(r, seg, lane, w, lo, hi, ok);
}

}  // namespace svoc
