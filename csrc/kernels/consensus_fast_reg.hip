// Fused two-pass robust consensus, fast mode, "register-streaming" variant: no LDS tile.
//
// Semantics: contract/src/contract.cairo:442-503 (constrained) / :370-434 (unconstrained).  The
// two-network fallback of the bf16 window kernel (consensus_fast_win.hip: f > 32, N > 256, or no
// pass-1 windows in D-sharded mode 2) and the cross-check the tests compare it with (wave_hint -7).
// Every lane loads its column-pair segment (64 rows x 2 bf16 = one dword per row) straight from
// HBM/L2 into VGPRs: no LDS tile and no slab barrier, so occupancy is set by VGPRs only and waves
// drift freely (one wave's loads overlap another's sorting network).  The qr pass re-reads the same dwords (L2/MALL-hot, just touched); pass 2 reads
// the instance again, with unreliable rows turned into max-key sentinels by a register OR.
// LDS holds only the per-wave qr partials, the reduced qr, the reliable bitmask and the status.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svoc/bufload.hpp"
#include "svoc/launch.hpp"
#include "svoc/sortnet.hpp"
#include "svoc/status.hpp"

namespace svoc {

// MODE 0: fused round; 1: pass 1 only (c1 + qr -> global); 2: rank + pass 2 from the global qr
// (D-sharding: the caller all-reduces the qr partials in between).
template <int NSEG, int WAVES, bool CONS, int MODE>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(NSEG >= 64 ? 1 : NSEG >= 32 ? 2 : 4))) void consensus_fast_reg_kernel(FastParams p) {
  constexpr int P = 64 / NSEG;          // column pairs per wave
  constexpr int NPAD = 64 * NSEG;       // padded oracle rows
  constexpr int W = WAVES * P * 2;      // columns per workgroup step
  constexpr int NT = WAVES * 64;
  constexpr int KEEP = 64 / P;
  __shared__ float qr_part[WAVES * NPAD];
  __shared__ float qr_lds[NPAD];
  constexpr int MW = NSEG < 4 ? 4 : NSEG;   // 64-row mask words
  __shared__ uint64_t relmask[MW];
  __shared__ uint64_t lowmask[MW];  // non-reliable rows turned into -inf sentinels (pass 2)
  __shared__ float misc_f[2];
  __shared__ int misc_i[2];

  const int b = blockIdx.x;
  if (p.active && !p.active[b]) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int seg = lane / P, pair_w = lane % P;
  const int cp = wave * P + pair_w;
  const int N = p.N, D = p.D;
  const int rowb = p.ld * 2;  // row stride in bytes
  const uint16_t* inst = (const uint16_t*)p.values + (int64_t)b * p.inst_stride;
  const __amdgpu_buffer_rsrc_t rs = instance_rsrc(inst, (uint32_t)(N * rowb));
  const int nslab = (D + W - 1) / W;
  // sentinel split (pass 1): rows >= N are padding; the first lo1 = ceil((NPAD-N)/2) of them become
  // -inf (key 0), the rest +inf (key 0xFFFF), so the smooth-median ranks N/2-1, N/2 (math.cairo:
  // 118-119, floor division for odd N too) always land on positions NPAD/2-1, NPAD/2 of the sorted
  // sequence: only those two network outputs are consumed, and dead-code elimination prunes the
  // sorting network down to a median selection network
  const int lo1 = (NPAD - N + 1) >> 1;
  const int nv = N - seg * 64;          // rows < nv are real
  const int nl = N + lo1 - seg * 64;    // rows in [nv, nl) are -inf, rows >= nl are +inf
  const int seg_off = seg * 64 * rowb;  // this lane's first row (bytes)
  const uint32_t pol = group_polarity<NSEG>(seg);  // complemented keys for descending runs

  float acc[KEEP];
#pragma unroll
  for (int i = 0; i < KEEP; ++i) acc[i] = 0.f;

  // ------------------------------------------------------------ pass 1
  const int pass1_slabs = MODE == 2 ? 0 : nslab;
#pragma nounroll
  for (int s = 0; s < pass1_slabs; ++s) {
    const int colA = s * W + 2 * cp;
    const bool vA = colA < D, vB = colA + 1 < D;
    const int vo = seg_off + (vA ? colA * 2 : 0);
    // opaque per-iteration copy: otherwise LICM hoists the 64 row masks out of the slab loop and
    // keeps them live in 64 VGPRs (+ their SGPR twins), doubling the register footprint
    int nvl = nv, nll = nl;
    asm volatile("" : "+v"(nvl), "+v"(nll));
    float cA, cB;
    // columns past D contribute 0 to qr: their bf16 halves are masked to +0 and their centre is +0
    const uint32_t mW = vA ? (vB ? 0xffffffffu : 0x0000ffffu) : 0u;
    {
      u16x2 r[64];
      if (N == NPAD) {  // uniform: no padding rows
        if (CONS) {  // key and run polarity in one XOR: raw ^ (0x80008000 ^ pol)
          const uint32_t kp = 0x80008000u ^ pol;
#pragma unroll
          for (int i = 0; i < 64; ++i) r[i] = as_k(bload(rs, vo, i * rowb) ^ kp);
        } else {
#pragma unroll
          for (int i = 0; i < 64; ++i) r[i] = as_k(as_u32(to_key<CONS>(bload(rs, vo, i * rowb))) ^ pol);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 64; ++i) {
          const uint32_t hi_m = ~lt_mask(i, nll);
          r[i] = as_k((as_u32(to_key<CONS>(bload(rs, vo, i * rowb))) & (lt_mask(i, nvl) | hi_m)) | hi_m);
        }
      }
      if (N != NPAD) {
#pragma unroll
        for (int i = 0; i < 64; ++i) r[i] = as_k(as_u32(r[i]) ^ pol);
      }
      u16x2 klo, khi;
      if constexpr (NSEG >= 8) median_group_wide<NSEG, P>(r, seg, lane, klo, khi);
      else median_group<NSEG>(r, klo, khi);
      const uint32_t lo = from_key<CONS>(klo), hi = from_key<CONS>(khi);
      cA = 0.5f * (bf16_lo(lo) + bf16_lo(hi));
      cB = 0.5f * (bf16_hi(lo) + bf16_hi(hi));
    }
    if (seg == 0) {
      if (vA) p.c1[(int64_t)b * D + colA] = cA;
      if (vB) p.c1[(int64_t)b * D + colA + 1] = cB;
    }
    __builtin_amdgcn_sched_barrier(0);
    float part[64];
    const f32x2 c2 = {vA ? cA : 0.f, vB ? cB : 0.f};
    if ((s + 1) * W > D) {  // slab with columns past D (uniform): masked words
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const uint32_t w = bload(rs, vo, i * rowb) & mW;  // L2/MALL-hot re-read
        const f32x2 y = bf16x2_to_f32x2(w) - c2;          // v_pk_add_f32
        const f32x2 q = y * y;                              // v_pk_mul_f32
        part[i] = q.x + q.y;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const f32x2 y = bf16x2_to_f32x2(bload(rs, vo, i * rowb)) - c2;
        const f32x2 q = y * y;
        part[i] = q.x + q.y;
      }
    }
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
  const int R = N - p.n_failing;
  for (int base = 0; base < NPAD; base += NT) {  // NT >= 64: one ballot word per wave-chunk
    const int t = base + tid;
    bool rel = false;
    float myq = 0.f;
    if (t < N) {
      myq = qr_lds[t];
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
    if (lane == 0 && (t >> 6) < MW) relmask[t >> 6] = bal;
  }
  __syncthreads();
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
      // pass-2 sentinel split: the first (NPAD - R) / 2 non-reliable rows become -inf
      int need = (NPAD - (N - p.n_failing) + 1) >> 1;
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
        else if (R < 4 && !p.legacy) st = ST_TOO_FEW_RELIABLE;  // legacy: no moments
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
    return;
  }
  // pass-2 outputs are staged in the workspace and committed at the end once the status is final
  const int Dp = p.work_pairs, D2 = 2 * Dp;
  const int STG = Dp * (2 * 17 + 8 + 2) * 4;   // launch.hpp: fast_work_stage_word
  const __amdgpu_buffer_rsrc_t ws = instance_rsrc(p.work + (int64_t)b * p.work_stride, (uint32_t)(p.work_stride * 4));
  const float n = (float)R;
  const uint64_t mymask = relmask[seg];
  const uint64_t mylow = lowmask[seg];
  int first_rel = 0;
  for (int w = 0; w < MW; ++w)
    if (relmask[w]) { first_rel = 64 * w + __builtin_ctzll(relmask[w]); break; }

  // ------------------------------------------------------------ pass 2 (contract.cairo:476-500)
#pragma nounroll
  for (int s = 0; s < nslab; ++s) {
    const int colA = s * W + 2 * cp;
    const bool vA = colA < D, vB = colA + 1 < D;
    const int vo = seg_off + (vA ? colA * 2 : 0);
    // sentinel bits with the run polarity folded in: row bit set -> key 0xFFFF (after ^pol), i.e.
    // mlp = ~(lowmask ^ polarity): a low (-inf) row gives 0 ^ pol, a high (+inf) row ~0 ^ pol
    uint64_t mm = mymask, mlp = ~(mylow ^ (pol ? ~0ull : 0ull));
    asm volatile("" : "+v"(mm), "+v"(mlp));
    const uint32_t kp2 = 0x80008000u ^ pol;
    // shifted power sums (shift = the first reliable row: no cancellation for clustered columns)
    const uint32_t w0 = bload(rs, vA ? colA * 2 : 0, first_rel * rowb);
    const f32x2 sh = {bf16_lo(w0), bf16_hi(w0)};
    f32x2 s1 = {0.f, 0.f}, s2 = s1, s3 = s1, s4 = s1;   // packed (column A, column B) power sums
    uint32_t wv[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) wv[i] = bload(rs, vo, i * rowb);
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      uint32_t w = wv[i];
      uint32_t mk = bit_mask(mm, i);
      // reliable rows keep their key; non-reliable rows become -inf (lowmask) / +inf sentinels
      // reliable rows: key ^ polarity; others: the -inf / +inf sentinel ^ polarity, read straight
      // from the pre-combined mask mlp (v_bfi: 4 ops per row for key + sentinel + polarity)
      uint32_t key = CONS ? ((w ^ kp2) & mk) | (bit_mask(mlp, i) & ~mk) : 0u;
      // row-ordered accumulation: keeps LLVM from front-loading all 64 rows (VGPRs)
      asm volatile("" : "+v"(w), "+v"(mk), "+v"(key), "+v"(s1), "+v"(s2), "+v"(s3), "+v"(s4));
      if (CONS) wv[i] = key;
      f32x2 y = bf16x2_to_f32x2(w) - sh;
      y = fand2(y, mk);
      const f32x2 q = y * y;
      s1 += y;
      s2 += q;
      s3 = __builtin_elementwise_fma(q, y, s3);
      s4 = __builtin_elementwise_fma(q, q, s4);
    }
    float s1A = s1.x, s2A = s2.x, s3A = s3.x, s4A = s4.x, s1B = s1.y, s2B = s2.y, s3B = s3.y, s4B = s4.y;
    const float shA = sh.x, shB = sh.y;
    float cA = 0.f, cB = 0.f;  // pass-2 smooth median (constrained consensus)
    if (CONS) {
      u16x2 r[64];
#pragma unroll
      for (int i = 0; i < 64; ++i) r[i] = as_k(wv[i]);
      u16x2 klo, khi;
      if constexpr (NSEG >= 8) median_group_wide<NSEG, P>(r, seg, lane, klo, khi);
      else median_group<NSEG>(r, klo, khi);
      const uint32_t lo = key_to_pos(klo), hi = key_to_pos(khi);
      cA = 0.5f * (bf16_lo(lo) + bf16_lo(hi));
      cB = 0.5f * (bf16_hi(lo) + bf16_hi(hi));
    }
#pragma unroll
    for (int t = 1; t < NSEG; t <<= 1) {
      s1A += __shfl_xor(s1A, t * P); s2A += __shfl_xor(s2A, t * P);
      s3A += __shfl_xor(s3A, t * P); s4A += __shfl_xor(s4A, t * P);
      s1B += __shfl_xor(s1B, t * P); s2B += __shfl_xor(s2B, t * P);
      s3B += __shfl_xor(s3B, t * P); s4B += __shfl_xor(s4B, t * P);
    }
    if (seg == 0) {
      // (the n-only factors once per slab, one division and one v_rsq per column: as consensus_fast_win.hip)
      const float in = 1.f / n, k3 = n / ((n - 1.f) * (n - 2.f));
      const float k4a = n * (n + 1.f) / (n - 1.f), k4b = 3.f * (n - 1.f) * (n - 1.f), ik4c = 1.f / ((n - 2.f) * (n - 3.f));
      bool zv = false;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool v = h ? vB : vA;
        if (!v) continue;
        const float s1 = h ? s1B : s1A, s2 = h ? s2B : s2A, s3 = h ? s3B : s3A, s4 = h ? s4B : s4A;
        const float sh = h ? shB : shA, med = h ? cB : cA;
        const float dl = s1 * in, e2 = s2 * in, e3 = s3 * in, e4 = s4 * in;
        const float mu2 = e2 - dl * dl;
        const float mu3 = e3 - 3.f * dl * e2 + 2.f * dl * dl * dl;
        const float mu4 = e4 - 4.f * dl * e3 + 6.f * dl * dl * e2 - 3.f * dl * dl * dl * dl;
        float sk = 0.f, ku = 0.f;
        if (mu2 > 0.f) {
          const float r = 1.f / mu2;
          const float z3 = n * mu3 * r * __builtin_amdgcn_rsqf(mu2), z4 = n * mu4 * (r * r);
          sk = z3 * k3;
          ku = (z4 * k4a - k4b) * ik4c;
        } else {
          zv = true;
        }
        stage_out(ws, STG, D2, 0, colA + h, CONS ? med : sh + dl);
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
  commit_staged<NT>(ws, STG, D2, D, tid, p.consensus + ob, p.skew + ob, p.kurt + ob);
  for (int t = tid; t < N; t += NT) {
    p.reliable[(int64_t)b * N + t] = (relmask[t >> 6] >> (t & 63)) & 1;
    p.qr[(int64_t)b * N + t] = qr_lds[t];
  }
  if (tid == 0) {
    p.rel[2 * (int64_t)b] = misc_f[0];
    p.rel[2 * (int64_t)b + 1] = misc_f[1];
    p.status[b] = ST_OK;
  }
}

template <int NSEG, int WAVES, int MODE>
static void launch_reg_mode(const FastParams& p, hipStream_t stream) {
  auto k = p.constrained ? consensus_fast_reg_kernel<NSEG, WAVES, true, MODE>
                         : consensus_fast_reg_kernel<NSEG, WAVES, false, MODE>;
  hipLaunchKernelGGL(k, dim3(p.B), dim3(WAVES * 64), 0, stream, p);
}

template <int NSEG, int WAVES>
static int launch_reg(const FastParams& p, hipStream_t stream) {
  if (p.mode == 1) {
    launch_reg_mode<NSEG, WAVES, 1>(p, stream);
  } else if (p.mode == 2) {
    launch_reg_mode<NSEG, WAVES, 2>(p, stream);
  } else {
    // fused single launch.  (The former split form, hint -1, published the qr partials into the
    // output qr between its two launches: not revert-safe, removed.)
    launch_reg_mode<NSEG, WAVES, 0>(p, stream);
  }
  return (int)hipGetLastError();
}

}  // namespace svoc

using namespace svoc;

extern "C" int svoc_fast_round_bf16_reg(const FastParams* p, hipStream_t stream) {
  if (p->B <= 0) return 0;
  if (p->N < 2 || p->N > 4096 || p->ld % 8 != 0 || p->D > p->ld) return -1;
  if (p->mode != 1 && (!p->work || p->work_pairs < fast_work_pairs(p->D) || p->work_stride < fast_work_words(p->D)))
    return -1;   // pass 2 stages its outputs in the workspace
  // 4 waves per workgroup (16 waves per CU at <= 128 VGPRs)
  if (p->N <= 64) return launch_reg<1, 4>(*p, stream);
  if (p->N <= 128) return launch_reg<2, 4>(*p, stream);
  if (p->N <= 256) return launch_reg<4, 4>(*p, stream);
  if (p->N <= 512) return launch_reg<8, 4>(*p, stream);
  if (p->N <= 1024) return launch_reg<16, 4>(*p, stream);
  // N > 1024: 32 / 64 lanes per column pair (two / one pair per wave), the same cross-lane bitonic sort
  if (p->N <= 2048) return launch_reg<32, 4>(*p, stream);
  return launch_reg<64, 4>(*p, stream);
}
