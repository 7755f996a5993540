// Fused two-pass robust consensus, fast mode (bf16 storage, fp32 math), one workgroup per instance.
//
// Semantics: contract/src/contract.cairo:442-503 (constrained) and :370-434 (unconstrained):
//   pass 1: c1 = per-column smooth median over all N oracles (math.cairo:113-126, the odd branch is
//           dead so ranks N/2-1 and N/2 are always averaged); qr_i = sum_d (x_id - c1_d)^2
//           (math.cairo:225-238); rel1 from mean(qr); rank-mask by (qr asc, idx desc) keeps the
//           N - f best (sort.cairo:96-101, contract.cairo:345-363);
//   pass 2: consensus = smooth median (constrained) or mean (unconstrained) of the reliable rows;
//           rel2 from the reliable rows' qr *against c1* (contract.cairo:484); per-column
//           population variance, sample-adjusted skewness and excess kurtosis (math.cairo:320-398).
//
// MI355X mapping:
//   * the instance is streamed in column slabs [Npad x W] bf16 into LDS with global_load_lds_dwordx4
//     (16 B/lane, lane-linear LDS image; the 16-B chunks of a row are XOR-swizzled by the row's
//     64-row segment through the SOURCE address so the lane-group reads below are conflict-free);
//   * each column pair is sorted in registers by a lane group (csrc/include/svoc/sortnet.hpp):
//     v_pk_min_u16/v_pk_max_u16 sort two columns per instruction, 64 rows per lane;
//   * per-row qr partials stay in 64 fp32 VGPRs per lane across all slabs and are reduce-scattered
//     across lanes once at the end (no atomics, deterministic);
//   * the rank mask is one LDS pass (thread = oracle), the reliable set becomes 64-bit ballots;
//   * pass 2 re-sorts each column with unreliable rows forced to the max key and reads moments as
//     shifted power sums (one LDS pass).  When the whole instance fits in one slab the LDS tile is
//     reused and the instance is read from HBM exactly once.
// Reverts (rel outside [0,1], too few reliable rows, a zero-variance reliable column) leave every
// output of the instance untouched and only set status[b]: pass 2 stages its outputs in the
// workspace and copies them out once the status is final (contract.cairo:588-603).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svoc/bufload.hpp"
#include "svoc/launch.hpp"
#include "svoc/sortnet.hpp"
#include "svoc/status.hpp"

namespace svoc {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

template <int NSEG, int WAVES>
struct FastGeom {
  static constexpr int NT = WAVES * 64;          // threads per workgroup
  static constexpr int P = 64 / NSEG;            // column pairs per wave
  static constexpr int NPAD = 64 * NSEG;         // padded oracle rows
  static constexpr int W = WAVES * P * 2;        // columns per slab
  static constexpr int ROWB = W * 2;             // bytes per slab row
  static constexpr int CPR = ROWB / 16;          // 16-B chunks per row
  static constexpr int TILE = NPAD * ROWB;       // slab bytes
  static constexpr int OFF_QRP = TILE;                         // [WAVES][NPAD] f32
  static constexpr int OFF_QR = OFF_QRP + WAVES * NPAD * 4;    // [NPAD] f32
  static constexpr int OFF_MISC = OFF_QR + NPAD * 4;           // 4 x u64 masks + 4 x f32 + 4 x i32
  static constexpr int LDS = OFF_MISC + 64;
  static_assert(CPR >= 4 * NSEG || NSEG == 1, "swizzle needs 4*NSEG chunks per row");
};

// chunk swizzle: rows of segment s store chunk c at c ^ (4 s)
template <int NSEG, int CPR>
SVOC_DEV int swz(int row) {
  if constexpr (NSEG == 1) return 0;
  else return ((row >> 6) * 4) & (CPR - 1);
}

// Stage one [NPAD x W] column slab into LDS with global_load_lds_dwordx4.  Rows that do not take
// part (row >= N, or unreliable rows in pass 2 when rel_only) are not read from HBM: their 16-B
// chunks are filled with the bf16 pattern 0x7FFF, whose sort key is 0xFFFF (the maximum), so they
// sort behind every real value without any per-row mask in the sort.
template <int NSEG, int WAVES>
SVOC_DEV void load_slab(const uint16_t* __restrict__ inst, int N, int ld, int col0, unsigned char* smem,
                        int tid, const uint64_t* relmask, bool rel_only) {
  using G = FastGeom<NSEG, WAVES>;
  const int lane = tid & 63;
#pragma unroll 4
  for (int off = tid * 16; off < G::TILE; off += G::NT * 16) {
    const int row = off / G::ROWB;
    const int c = (off % G::ROWB) >> 4;
    const int sc = c ^ swz<NSEG, G::CPR>(row);
    const int col = col0 + sc * 8;
    const int base = __builtin_amdgcn_readfirstlane(off - lane * 16);
    bool take = row < N;
    if (rel_only) take = take && ((relmask[row >> 6] >> (row & 63)) & 1);
    if (take && col < ld) {
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(inst + (int64_t)row * ld + col),
                                       (lds_ptr_t)(smem + base), 16, 0, 0);
    } else if (!take) {
      *(uint4*)(smem + off) = make_uint4(0x7fff7fffu, 0x7fff7fffu, 0x7fff7fffu, 0x7fff7fffu);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// Single-slab instances keep their tile for pass 2: overwrite the unreliable rows in place.
template <int NSEG, int WAVES>
SVOC_DEV void mask_unreliable(int N, unsigned char* smem, int tid, const uint64_t* relmask) {
  using G = FastGeom<NSEG, WAVES>;
  for (int off = tid * 16; off < N * G::ROWB; off += G::NT * 16) {
    const int row = off / G::ROWB;
    if (!((relmask[row >> 6] >> (row & 63)) & 1))
      *(uint4*)(smem + off) = make_uint4(0x7fff7fffu, 0x7fff7fffu, 0x7fff7fffu, 0x7fff7fffu);
  }
  __syncthreads();
}

// LDS byte address of (row, pair cp) inside the slab
template <int NSEG, int WAVES>
SVOC_DEV int pair_addr(int row, int cp) {
  using G = FastGeom<NSEG, WAVES>;
  const int c = (cp >> 2) ^ swz<NSEG, G::CPR>(row);
  return row * G::ROWB + c * 16 + (cp & 3) * 4;
}

template <int NSEG, int WAVES, bool CONS>
__global__ __launch_bounds__(WAVES * 64) void consensus_fast_bf16_kernel(FastParams p) {
  using G = FastGeom<NSEG, WAVES>;
  constexpr int P = G::P;
  constexpr int KEEP = 64 / P;  // row sums a lane keeps after the qr reduce-scatter
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* qr_part = (float*)(smem + G::OFF_QRP);
  float* qr_lds = (float*)(smem + G::OFF_QR);
  uint64_t* relmask = (uint64_t*)(smem + G::OFF_MISC);
  float* misc_f = (float*)(smem + G::OFF_MISC + 32);
  int* misc_i = (int*)(smem + G::OFF_MISC + 48);

  const int b = blockIdx.x;
  if (p.active && !p.active[b]) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int seg = lane / P, pair_w = lane % P;
  const int cp = wave * P + pair_w;  // pair index inside the slab
  const int N = p.N, D = p.D, ld = p.ld;
  const uint16_t* inst = (const uint16_t*)p.values + (int64_t)b * p.inst_stride;
  const int nslab = (D + G::W - 1) / G::W;
  const int m = N >> 1;  // smooth-median ranks m-1, m (math.cairo:118-119)
  const int a0 = pair_addr<NSEG, WAVES>(seg * 64, cp);

  float acc[KEEP];
#pragma unroll
  for (int i = 0; i < KEEP; ++i) acc[i] = 0.f;

  // ------------------------------------------------------------ pass 1
  const int pass1_slabs = p.mode == 2 ? 0 : nslab;  // mode 2: qr comes all-reduced from the caller
#pragma nounroll
  for (int s = 0; s < pass1_slabs; ++s) {
    const int col0 = s * G::W;
    if (s > 0) __syncthreads();  // previous slab fully consumed before it is overwritten
    load_slab<NSEG, WAVES>(inst, N, ld, col0, smem, tid, relmask, false);
    const int colA = col0 + 2 * cp;
    const bool vA = colA < D, vB = colA + 1 < D;
    float cA, cB;
    {
      u16x2 r[64];
#pragma unroll
      for (int i = 0; i < 64; ++i) r[i] = bf16x2_to_key(*(const uint32_t*)(smem + a0 + i * G::ROWB));
      sort_group<NSEG, P>(r, seg);
      const uint32_t lo = key_to_bf16x2(group_select<NSEG, P>(r, m - 1, lane));
      const uint32_t hi = key_to_bf16x2(group_select<NSEG, P>(r, m, lane));
      cA = 0.5f * (bf16_lo(lo) + bf16_lo(hi));
      cB = 0.5f * (bf16_hi(lo) + bf16_hi(hi));
    }
    if (seg == 0) {
      if (vA) p.c1[(int64_t)b * D + colA] = cA;
      if (vB) p.c1[(int64_t)b * D + colA + 1] = cB;
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the qr loads below the sort (register pressure)
    // per-row partials of qr; rows >= N hold NaN sentinels and are never read back
    float part[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      const uint32_t w = *(const uint32_t*)(smem + a0 + i * G::ROWB);
      // selects, not multiplies: columns past D hold stale bytes (maybe NaN)
      const float yA = vA ? bf16_lo(w) - cA : 0.f;
      const float yB = vB ? bf16_hi(w) - cB : 0.f;
      part[i] = __builtin_fmaf(yA, yA, yB * yB);
    }
    // reduce-scatter over the pair bits of the lane: lanes sharing a segment sum their partials
#pragma unroll
    for (int h = 32, msk = P / 2; msk >= 1; h >>= 1, msk >>= 1) {
      const bool up = (lane & msk) != 0;
#pragma unroll
      for (int i = 0; i < h; ++i) {
        const float lo_v = part[i], hi_v = part[i + h];
        const float send = up ? lo_v : hi_v;
        const float keep = up ? hi_v : lo_v;
        part[i] = keep + __shfl_xor(send, msk);
      }
    }
#pragma unroll
    for (int i = 0; i < KEEP; ++i) acc[i] += part[i];
  }

  // ------------------------------------------------------------ qr: lane holds rows seg*64+base+[0,KEEP)
  {
    int base = 0;
#pragma unroll
    for (int h = 32, msk = P / 2; msk >= 1; h >>= 1, msk >>= 1) base += (lane & msk) ? h : 0;
#pragma unroll
    for (int i = 0; i < KEEP; ++i) qr_part[wave * G::NPAD + seg * 64 + base + i] = acc[i];
  }
  __syncthreads();
  for (int t = tid; t < G::NPAD; t += G::NT) {
    float q = 0.f;
    if (p.mode == 2) {
      q = t < N ? p.qr[(int64_t)b * N + t] : 0.f;
    } else {
#pragma unroll
      for (int w = 0; w < WAVES; ++w) q += qr_part[w * G::NPAD + t];
    }
    qr_lds[t] = q;
  }
  __syncthreads();
  if (p.mode == 1) {  // D-sharding, pass 1: publish this shard's qr partials (c1 already written)
    for (int t = tid; t < N; t += G::NT) p.qr[(int64_t)b * N + t] = qr_lds[t];
    if (tid == 0) p.status[b] = ST_OK;
    return;
  }

  // ------------------------------------------------------------ rank mask (contract.cairo:345-363)
  const int R = N - p.n_failing;
  {
    bool rel = false;
    float myq = 0.f;
    if (tid < N) {
      myq = qr_lds[tid];
      // rank = #{j : (qr_j, -j) < (qr_me, -me)}; 4 rows per ds_read_b128, independent loads
      int rank = 0;
      const int n4 = N & ~3;
      for (int j = 0; j < n4; j += 4) {
        const float4 q4 = *(const float4*)(qr_lds + j);
        rank += (q4.x < myq || (q4.x == myq && j > tid)) ? 1 : 0;
        rank += (q4.y < myq || (q4.y == myq && j + 1 > tid)) ? 1 : 0;
        rank += (q4.z < myq || (q4.z == myq && j + 2 > tid)) ? 1 : 0;
        rank += (q4.w < myq || (q4.w == myq && j + 3 > tid)) ? 1 : 0;
      }
      for (int j = n4; j < N; ++j) {
        const float qj = qr_lds[j];
        rank += (qj < myq || (qj == myq && j > tid)) ? 1 : 0;  // (qr asc, idx desc)
      }
      rel = rank < R;
    }
    const uint64_t bal = __ballot(rel);
    if (lane == 0 && wave < 4) relmask[wave] = bal;
    float s_all = myq, s_rel = rel ? myq : 0.f;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      s_all += __shfl_xor(s_all, o);
      s_rel += __shfl_xor(s_rel, o);
    }
    __syncthreads();  // qr_part is reused below
    if (lane == 0) {
      qr_part[wave] = s_all;
      qr_part[WAVES + wave] = s_rel;
    }
  }
  __syncthreads();
  if (tid == 0) {
    float sa = 0.f, sr = 0.f;
    for (int w = 0; w < WAVES; ++w) {
      sa += qr_part[w];
      sr += qr_part[WAVES + w];
    }
    int st = ST_OK;
    float rel1, rel2 = 0.f;
    const float rd = p.legacy ? 1.f : (float)(p.rel_dim > 0 ? p.rel_dim : D);
    if (CONS) rel1 = 1.f - 2.f * sqrtf(sa / (float)N / rd);                  // contract.cairo:436-439
    else rel1 = 1.f - fminf(p.max_spread, sqrtf(sa / (float)N)) / p.max_spread;  // :365-368
    if (!(rel1 >= 0.f && rel1 <= 1.f)) st = ST_RELIABILITY_INTERVAL;
    else if (R < 2) st = R <= 0 ? ST_USIZE_UNDERFLOW : ST_INDEX_OOB;
    else {
      if (CONS) rel2 = 1.f - 2.f * sqrtf(sr / (float)R / rd);
      else rel2 = 1.f - fminf(p.max_spread, sqrtf(sr / (float)R)) / p.max_spread;
      if (!(rel2 >= 0.f && rel2 <= 1.f)) st = ST_RELIABILITY_INTERVAL;
      else if (R < 4 && !p.legacy) st = ST_TOO_FEW_RELIABLE;
    }
    misc_f[0] = rel1;
    misc_f[1] = rel2;
    misc_i[0] = st;
    misc_i[1] = 0;  // zero-variance flag
  }
  __syncthreads();
  if (misc_i[0] != ST_OK) {
    if (tid == 0) p.status[b] = misc_i[0];
    return;  // revert: outputs untouched
  }
  // pass-2 outputs are staged in the workspace and committed at the end once the status is final
  const int Dp = p.work_pairs, D2 = 2 * Dp;
  const int STG = Dp * (2 * 17 + 8 + 2) * 4;   // launch.hpp: fast_work_stage_word
  const __amdgpu_buffer_rsrc_t ws = instance_rsrc(p.work + (int64_t)b * p.work_stride, (uint32_t)(p.work_stride * 4));
  const float n = (float)R;
  const int m2 = R >> 1;
  // reliable rows held by this lane after the masked sort: sorted positions [0, cnt)
  const int cnt = min(64, max(0, R - seg * 64));
  // unconstrained: power sums are shifted by the first reliable row (inside the reliable cluster)
  int first_rel = 0;
  if (!CONS) {
    for (int w = 0; w < 4; ++w)
      if (relmask[w]) { first_rel = 64 * w + __builtin_ctzll(relmask[w]); break; }
  }
  const uint64_t mymask = relmask[seg];

  // ------------------------------------------------------------ pass 2 (contract.cairo:476-500)
  // slabs walked backwards: the slab resident from pass 1 is reused without a reload
#pragma nounroll
  for (int s = nslab - 1; s >= 0; --s) {
    const int col0 = s * G::W;
    if (s != nslab - 1 || p.mode == 2) {
      __syncthreads();
      load_slab<NSEG, WAVES>(inst, N, ld, col0, smem, tid, relmask, true);
    } else if (CONS) {
      mask_unreliable<NSEG, WAVES>(N, smem, tid, relmask);
    }
    const int colA = col0 + 2 * cp;
    const bool vA = colA < D, vB = colA + 1 < D;
    const uint32_t mA = vA ? 0xffffffffu : 0u, mB = vB ? 0xffffffffu : 0u;
    uint64_t mm = mymask;  // opaque per-iteration copies: stop LICM from hoisting 64 row masks
    int cntl = cnt;
    asm volatile("" : "+v"(mm), "+v"(cntl));
    float shA, shB;
    float s1A = 0.f, s2A = 0.f, s3A = 0.f, s4A = 0.f, s1B = 0.f, s2B = 0.f, s3B = 0.f, s4B = 0.f;
    if (CONS) {
      u16x2 r[64];
#pragma unroll
      for (int i = 0; i < 64; ++i) r[i] = bf16x2_to_key(*(const uint32_t*)(smem + a0 + i * G::ROWB));
      sort_group<NSEG, P>(r, seg);
      const uint32_t lo = key_to_bf16x2(group_select<NSEG, P>(r, m2 - 1, lane));
      const uint32_t hi = key_to_bf16x2(group_select<NSEG, P>(r, m2, lane));
      shA = 0.5f * (bf16_lo(lo) + bf16_lo(hi));
      shB = 0.5f * (bf16_hi(lo) + bf16_hi(hi));
      __builtin_amdgcn_sched_barrier(0);
      // moments straight from the sorted registers: positions < cnt are the reliable values
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        // sched_barrier every 8 rows: otherwise hipcc converts all 64 keys up front (+100 VGPRs)
        if ((i & 7) == 0) __builtin_amdgcn_sched_barrier(0);
        const uint32_t w = key_to_bf16x2(r[i]);
        const uint32_t mk = lt_mask(i, cntl);  // sorted positions >= cnt hold NaN sentinels
        const float yA = fand(bf16_lo(w) - shA, mk), yB = fand(bf16_hi(w) - shB, mk);
        const float qA = yA * yA, qB = yB * yB;
        s1A += yA; s2A += qA; s3A = __builtin_fmaf(qA, yA, s3A); s4A = __builtin_fmaf(qA, qA, s4A);
        s1B += yB; s2B += qB; s3B = __builtin_fmaf(qB, yB, s3B); s4B = __builtin_fmaf(qB, qB, s4B);
      }
    } else {
      const uint32_t w0 = *(const uint32_t*)(smem + pair_addr<NSEG, WAVES>(first_rel, cp));
      shA = bf16_lo(w0);
      shB = bf16_hi(w0);
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const uint32_t w = *(const uint32_t*)(smem + a0 + i * G::ROWB);
        const bool mk = (mm >> i) & 1;
        const float yA = mk ? bf16_lo(w) - shA : 0.f, yB = mk ? bf16_hi(w) - shB : 0.f;
        const float qA = yA * yA, qB = yB * yB;
        s1A += yA; s2A += qA; s3A = __builtin_fmaf(qA, yA, s3A); s4A = __builtin_fmaf(qA, qA, s4A);
        s1B += yB; s2B += qB; s3B = __builtin_fmaf(qB, yB, s3B); s4B = __builtin_fmaf(qB, qB, s4B);
      }
    }
#pragma unroll
    for (int t = 1; t < NSEG; t <<= 1) {
      s1A += __shfl_xor(s1A, t * P); s2A += __shfl_xor(s2A, t * P);
      s3A += __shfl_xor(s3A, t * P); s4A += __shfl_xor(s4A, t * P);
      s1B += __shfl_xor(s1B, t * P); s2B += __shfl_xor(s2B, t * P);
      s3B += __shfl_xor(s3B, t * P); s4B += __shfl_xor(s4B, t * P);
    }
    if (seg == 0) {
      // central moments from shifted power sums; skew / kurt as math.cairo:320-363
      const float k3 = n / ((n - 1.f) * (n - 2.f));
      const float k4a = n * (n + 1.f) / (n - 1.f), k4b = 3.f * (n - 1.f) * (n - 1.f), k4c = (n - 2.f) * (n - 3.f);
      bool zv = false;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool v = h ? vB : vA;
        if (!v) continue;
        const float s1 = h ? s1B : s1A, s2 = h ? s2B : s2A, s3 = h ? s3B : s3A, s4 = h ? s4B : s4A;
        const float sh = h ? shB : shA;
        const float dl = s1 / n, e2 = s2 / n, e3 = s3 / n, e4 = s4 / n;
        const float mu2 = e2 - dl * dl;
        const float mu3 = e3 - 3.f * dl * e2 + 2.f * dl * dl * dl;
        const float mu4 = e4 - 4.f * dl * e3 + 6.f * dl * dl * e2 - 3.f * dl * dl * dl * dl;
        float sk = 0.f, ku = 0.f;
        if (mu2 > 0.f) {
          const float sd = sqrtf(mu2);
          const float z3 = n * mu3 / (mu2 * sd), z4 = n * mu4 / (mu2 * mu2);
          sk = z3 * k3;
          ku = (z4 * k4a - k4b) / k4c;
        } else {
          zv = true;
        }
        stage_out(ws, STG, D2, 0, colA + h, CONS ? sh : sh + dl);
        stage_out(ws, STG, D2, 1, colA + h, p.legacy ? 0.f : sk);
        stage_out(ws, STG, D2, 2, colA + h, p.legacy ? 0.f : ku);
      }
      if (zv && !p.legacy) misc_i[1] = 1;
    }
  }
  __syncthreads();
  // ------------------------------------------------------------ commit (only a successful round)
  if (misc_i[1]) {
    if (tid == 0) p.status[b] = ST_ZERO_VARIANCE;
    return;
  }
  const int64_t ob = (int64_t)b * D;
  commit_staged<G::NT>(ws, STG, D2, D, tid, p.consensus + ob, p.skew + ob, p.kurt + ob);
  if (tid < N) {
    p.reliable[(int64_t)b * N + tid] = (relmask[tid >> 6] >> (tid & 63)) & 1;
    p.qr[(int64_t)b * N + tid] = qr_lds[tid];
  }
  if (tid == 0) {
    p.rel[2 * (int64_t)b] = misc_f[0];
    p.rel[2 * (int64_t)b + 1] = misc_f[1];
    p.status[b] = ST_OK;
  }
}

template <int NSEG, int WAVES>
static int launch_fast(const FastParams& p, hipStream_t stream) {
  using G = FastGeom<NSEG, WAVES>;
  auto k = p.constrained ? consensus_fast_bf16_kernel<NSEG, WAVES, true>
                         : consensus_fast_bf16_kernel<NSEG, WAVES, false>;
  hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k, dim3(p.B), dim3(G::NT), G::LDS, stream, p);
  return (int)hipGetLastError();
}

}  // namespace svoc

using namespace svoc;

// Picks the lane-group geometry from N (rows) and D (columns):
//   N <= 64  -> 1 lane per column pair; 8 waves when the whole instance fits one 128-KiB slab.
//   N <= 128 -> 2 lanes; N <= 256 -> 4 lanes (4 waves, 64-KiB slabs, 2 workgroups per CU).
extern "C" int svoc_fast_round_bf16_reg(const FastParams* p, hipStream_t stream);
extern "C" int svoc_fast_round_bf16_small(const FastParams* p, hipStream_t stream);
extern "C" int svoc_fast_round_bf16_win(const FastParams* p, hipStream_t stream);

extern "C" int svoc_fast_round_bf16(const FastParams* p, hipStream_t stream) {
  if (p->B <= 0) return 0;
  // default (0) and negative hints: register-streaming kernel (consensus_fast_reg.hip).  Positive
  // hints select this LDS-tiled kernel (1 = its default geometry).
  // small instances (N <= 16, D <= 128, full round): several instances per wave, registers only
  if (p->wave_hint == 0 && p->mode == 0 && p->N <= 16 && p->D <= 128) return svoc_fast_round_bf16_small(p, stream);
  // default: one-network window kernel (consensus_fast_win.hip) when it applies (workspace given,
  // f <= 32); -7 forces the two-network register kernel
  if (p->wave_hint == 0) {
    const int rc = svoc_fast_round_bf16_win(p, stream);
    if (rc != -2) return rc;
  }
  if (p->wave_hint == -7) {
    FastParams q = *p;
    q.wave_hint = 0;
    return svoc_fast_round_bf16_reg(&q, stream);
  }
  if (p->wave_hint <= 0) return svoc_fast_round_bf16_reg(p, stream);
  if (p->N < 2 || p->N > 256 || p->ld % 8 != 0 || p->D > p->ld) return -1;
  if (p->mode != 1 && (!p->work || p->work_pairs < fast_work_pairs(p->D) || p->work_stride < fast_work_words(p->D)))
    return -1;   // pass 2 stages its outputs in the workspace
  if (p->N <= 64) {
    // wave_hint: 2 / 4 / 8 waves per workgroup = 256 / 512 / 1024-column slabs (32/64/128 KiB LDS)
    if (p->wave_hint == 2) return launch_fast<1, 2>(*p, stream);
    if (p->wave_hint == 4) return launch_fast<1, 4>(*p, stream);
    if (p->wave_hint == 8) return launch_fast<1, 8>(*p, stream);
    return launch_fast<1, 4>(*p, stream);  // measured best for 64 x 1024 (2 workgroups / CU)
  }
  if (p->N <= 128) return launch_fast<2, 4>(*p, stream);
  return launch_fast<4, 4>(*p, stream);
}
