// Fused encoder epilogues for the sentiment path (svoc/models/encoder.py, post-LN BERT/RoBERTa).
//
// add_layernorm: out = LayerNorm(x + y) * w + b over the hidden dim, bf16 in/out, fp32 math.
// One wave per row; each lane holds H/64 elements (H = 768: 12 per lane, three 8-byte loads per
// operand) so the row never leaves registers: mean and variance (two-pass, on registers) by wave
// butterflies.  Replaces an elementwise add + a separate LayerNorm (two extra HBM round trips of the
// [tokens, H] activation) -- the post-LN residual is consumed only through the LayerNorm output.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace svoc {

__device__ __forceinline__ float bf2f(uint16_t h) { return __builtin_bit_cast(float, (uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // round to nearest even (finite inputs)
  const uint32_t u = __builtin_bit_cast(uint32_t, f);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// EPL elements per lane (multiple of 4), H = 64 * EPL
template <int EPL>
__global__ __launch_bounds__(256) void add_layernorm_kernel(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ y,
                                                            const uint16_t* __restrict__ w,
                                                            const uint16_t* __restrict__ bias,
                                                            uint16_t* __restrict__ out, int64_t rows, float eps,
                                                            int64_t y_stride) {
  constexpr int H = 64 * EPL;
  constexpr int V = EPL / 4;  // 8-byte vectors per lane
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const uint2* xr = (const uint2*)(x + row * H);
  const uint2* yr = (const uint2*)(y + row * y_stride);  // y_stride 0: one [H] row for all
  float v[EPL];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int c = k * 64 + lane;  // coalesced: consecutive lanes read consecutive 8-byte pieces
    const uint2 a = xr[c], b = yr[c];
    const uint32_t aw[2] = {a.x, a.y}, bw[2] = {b.x, b.y};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float lo = bf2f(aw[j] & 0xffffu) + bf2f(bw[j] & 0xffffu);
      const float hi = bf2f(aw[j] >> 16) + bf2f(bw[j] >> 16);
      v[4 * k + 2 * j] = lo;
      v[4 * k + 2 * j + 1] = hi;
      s += lo + hi;
    }
  }
  const float mean = wave_sum(s) * (1.f / H);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) * (1.f / H) + eps);
  uint2* orow = (uint2*)(out + row * H);
  const uint2* wr = (const uint2*)w;
  const uint2* br = (const uint2*)bias;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int c = k * 64 + lane;
    const uint2 gw = wr[c], gb = br[c];
    const uint32_t ww[2] = {gw.x, gw.y}, bb[2] = {gb.x, gb.y};
    uint32_t o[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float lo = (v[4 * k + 2 * j] - mean) * rstd * bf2f(ww[j] & 0xffffu) + bf2f(bb[j] & 0xffffu);
      const float hi = (v[4 * k + 2 * j + 1] - mean) * rstd * bf2f(ww[j] >> 16) + bf2f(bb[j] >> 16);
      o[j] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
    }
    orow[c] = make_uint2(o[0], o[1]);
  }
}

}  // namespace svoc

using namespace svoc;

namespace svoc {

// embed_layernorm: out[t] = LayerNorm(tok[ids[t]] + pos[pos_ids[t]] + typ) * w + b (RoBERTa embeddings,
// client/oracle_scheduler.py's classifier input), bf16 in/out.  The two adds round to bf16 as the
// PyTorch expression they replace (bf16 tensors), the LayerNorm is fp32; one wave per token row as
// add_layernorm.  Replaces an embedding gather, two elementwise adds and a LayerNorm (four passes).
template <int EPL>
__global__ __launch_bounds__(256) void embed_layernorm_kernel(const int64_t* __restrict__ ids,
                                                              const int64_t* __restrict__ pos_ids,
                                                              const uint16_t* __restrict__ tok,
                                                              const uint16_t* __restrict__ pos,
                                                              const uint16_t* __restrict__ typ,
                                                              const uint16_t* __restrict__ w,
                                                              const uint16_t* __restrict__ bias,
                                                              uint16_t* __restrict__ out, int64_t rows, float eps) {
  constexpr int H = 64 * EPL;
  constexpr int V = EPL / 4;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const uint2* tr = (const uint2*)(tok + ids[row] * H);
  const uint2* pr = (const uint2*)(pos + pos_ids[row] * H);
  const uint2* yr = (const uint2*)typ;
  float v[EPL];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int c = k * 64 + lane;
    const uint2 a = tr[c], b = pr[c], t = yr[c];
    const uint32_t aw[2] = {a.x, a.y}, bw[2] = {b.x, b.y}, tw[2] = {t.x, t.y};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int sh = 16 * h;
        const float ab = bf2f(f2bf(bf2f((aw[j] >> sh) & 0xffffu) + bf2f((bw[j] >> sh) & 0xffffu)));
        const float e = bf2f(f2bf(ab + bf2f((tw[j] >> sh) & 0xffffu)));
        v[4 * k + 2 * j + h] = e;
        s += e;
      }
    }
  }
  const float mean = wave_sum(s) * (1.f / H);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) * (1.f / H) + eps);
  uint2* orow = (uint2*)(out + row * H);
  const uint2* wr = (const uint2*)w;
  const uint2* br = (const uint2*)bias;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int c = k * 64 + lane;
    const uint2 gw = wr[c], gb = br[c];
    const uint32_t ww[2] = {gw.x, gw.y}, bb[2] = {gb.x, gb.y};
    uint32_t o[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float lo = (v[4 * k + 2 * j] - mean) * rstd * bf2f(ww[j] & 0xffffu) + bf2f(bb[j] & 0xffffu);
      const float hi = (v[4 * k + 2 * j + 1] - mean) * rstd * bf2f(ww[j] >> 16) + bf2f(bb[j] >> 16);
      o[j] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
    }
    orow[c] = make_uint2(o[0], o[1]);
  }
}

// segment_mean: out[b] = mean of x[t] over t in [cu[b], cu[b+1]) (the masked mean pooling of the
// classification head over the real tokens), fp32 sums in token order, bf16 out (empty segment: 0).
// One workgroup per segment: thread (g, c) sums 8 columns (one 16-B load per row) of rows g, g + G, ...;
// the G partial sums meet in LDS.  Replaces a scatter into the padded grid, an fp32 copy and a sum.
__global__ __launch_bounds__(256) void segment_mean_kernel(const uint16_t* __restrict__ x, const int* __restrict__ cu,
                                                           uint16_t* __restrict__ out, int H, int G) {
  __shared__ float part[256 * 8];
  const int b = blockIdx.x, chunks = H / 8;
  const int tid = threadIdx.x, g = tid / chunks, c = tid % chunks;
  const int lo = cu[b], hi = cu[b + 1];
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (g < G) {
    for (int t = lo + g; t < hi; t += G) {
      const uint4 w = *(const uint4*)(x + (int64_t)t * H + 8 * c);
      const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[2 * j] += bf2f(ws[j] & 0xffffu);
        acc[2 * j + 1] += bf2f(ws[j] >> 16);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) part[tid * 8 + j] = acc[j];
  }
  __syncthreads();
  if (g == 0) {
    const float inv = 1.f / (float)(hi - lo > 1 ? hi - lo : 1);
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float a0 = 0.f, a1 = 0.f;
      for (int gg = 0; gg < G; ++gg) {
        a0 += part[(gg * chunks + c) * 8 + 2 * j];
        a1 += part[(gg * chunks + c) * 8 + 2 * j + 1];
      }
      o[j] = (uint32_t)f2bf(a0 * inv) | ((uint32_t)f2bf(a1 * inv) << 16);
    }
    *(uint4*)(out + (int64_t)b * H + 8 * c) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

}  // namespace svoc

// Returns 0 on success, -1 if the hidden size is not supported (caller falls back to ATen).
// y_stride: H (y is [rows, H]) or 0 (y is one [H] row added to every row, e.g. a GEMM bias when the
// residual was accumulated into the GEMM output).
extern "C" int svoc_add_layernorm_bf16(const void* x, const void* y, const void* w, const void* b, void* out,
                                       int64_t rows, int H, float eps, int64_t y_stride, hipStream_t stream) {
  if (rows <= 0) return 0;
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  const auto* X = (const uint16_t*)x;
  const auto* Y = (const uint16_t*)y;
  const auto* W = (const uint16_t*)w;
  const auto* B = (const uint16_t*)b;
  auto* O = (uint16_t*)out;
  switch (H) {
    case 256: hipLaunchKernelGGL(add_layernorm_kernel<4>, grid, block, 0, stream, X, Y, W, B, O, rows, eps, y_stride); break;
    case 512: hipLaunchKernelGGL(add_layernorm_kernel<8>, grid, block, 0, stream, X, Y, W, B, O, rows, eps, y_stride); break;
    case 768: hipLaunchKernelGGL(add_layernorm_kernel<12>, grid, block, 0, stream, X, Y, W, B, O, rows, eps, y_stride); break;
    case 1024: hipLaunchKernelGGL(add_layernorm_kernel<16>, grid, block, 0, stream, X, Y, W, B, O, rows, eps, y_stride); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// attention_qkv: softmax(Q Kᵀ / sqrt(64) + key-padding mask) V for short sequences (S <= 128,
// S % 32 == 0, head dim 64), reading the fused QKV projection [B, S, 3, H, 64] directly and
// writing [B, S, H, 64] (the out-projection's input layout: no transpose copies).
//
// One workgroup per (sequence, head), one wave per 32 queries.  MFMA orientation "key on the
// register, query on the lane": X = K·Qᵀ (mfma_f32_32x32x16_bf16, A = K rows, B = Q rows, both 16-B
// contiguous global loads) leaves each lane with one query's scores for 64 keys (its partner
// lane ^ 32 holds the other 64), so the softmax is lane-local plus one xor-32 exchange, and the
// accumulator registers ARE the A operand of Z = P·V (pairs of registers -> bf16, k order
// 16s + 8(j>>2) + 4h + (j&3)).  V is staged ROW-major in LDS (one 16-B store per 16-B global load;
// 128-B rows, 16-B chunk c of row k at chunk c ^ 4((k >> 1) & 1)) and each B fragment is two gfx950
// transposed reads (ds_read_b64_tr_b16: a 16-lane group reads 4 keys x 16 dims and every lane gets
// its dim's 4 keys), conflict-free under that swizzle.  (The previous image was transposed on the
// write side: 16 two-byte LDS stores per 16-B chunk, with bank conflicts.)  P is normalised before
// the PV product (bf16 P, as flash attention).  At S = 128 the whole problem is 32 MFMAs per wave.
// ---------------------------------------------------------------------------------------------
namespace svoc {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short v4i16 __attribute__((ext_vector_type(4)));

template <int NQB>  // S_max / 32: query blocks = waves = key blocks
__global__ __launch_bounds__(64 * NQB) __attribute__((amdgpu_waves_per_eu(4))) void attn_short_kernel(const uint16_t* __restrict__ qkv,
                                                             const uint8_t* __restrict__ kmask,
                                                             const int* __restrict__ cu_seqlens,
                                                             int64_t rows_total, uint16_t* __restrict__ out,
                                                             int H, float scale_log2) {
  constexpr int S = 32 * NQB, DH = 64;
  __shared__ __attribute__((aligned(16))) uint16_t Vs[S * DH];   // row-major V, swizzled 16-B chunks
  __shared__ __attribute__((aligned(16))) uint16_t Ks[S * DH];   // row-major K, same image
  __shared__ uint8_t km[S];
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int64_t ts = (int64_t)3 * H * DH;  // token stride in qkv (elements)
  // padded batch: sequence b = rows [b*S, b*S + S), keys masked by kmask.
  // packed (varlen): sequence b = rows [cu[b], cu[b+1]), keys past its length masked; rows read past
  // the end of the buffer are clamped (their scores are masked, their V rows get P = 0).
  const int64_t base = cu_seqlens ? cu_seqlens[b] : (int64_t)b * S;
  const int L = cu_seqlens ? cu_seqlens[b + 1] - cu_seqlens[b] : S;
  const int nkb = (L + 31) >> 5;  // key / query blocks holding real tokens
  auto row = [&](int k) -> int64_t {
    const int64_t t = base + k;
    return t < rows_total ? t : rows_total - 1;
  };
  const uint16_t* Qb = qkv + h * DH;
  const uint16_t* Kb = Qb + H * DH;
  const uint16_t* Vb = Qb + 2 * H * DH;

  // stage K and V once per workgroup (row-major, swizzled; every query wave reads them from LDS).
  // Fixed trip count (S * 8 chunks over 64 * NQB threads = 4 per thread), all loads -- K, V and this
  // wave's Q fragments -- issued before the first LDS store: one memory round trip per workgroup.
  constexpr int ITER = S * (DH / 8) / (64 * NQB);
  const int nchunks = nkb * 32 * (DH / 8);
  uint4 kv[ITER], vv[ITER];
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    int c = tid + it * 64 * NQB;
    c = c < nchunks ? c : tid;   // past the sequence: re-read the thread's first chunk (cache hit), unused
    const int64_t g = row(c >> 3) * ts + (c & 7) * 8;
    kv[it] = *(const uint4*)(Kb + g);
    vv[it] = *(const uint4*)(Vb + g);
  }
  // X = K·Qᵀ for this wave's 32 queries: rows = keys (registers), column = query (lane)
  const int q0 = wave * 32;
  const bool active = q0 < L;
  bf16x8 qf[4];
  if (active) {
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) qf[ds] = *(const bf16x8*)(Qb + row(q0 + r) * ts + ds * 16 + 8 * hh);
  }
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    const int c = tid + it * 64 * NQB;
    if (c < nchunks) {
      const int key = c >> 3, ch = c & 7;
      const int off = 128 * key + 16 * (ch ^ (((key >> 1) & 1) << 2));
      *(uint4*)((unsigned char*)Ks + off) = kv[it];
      *(uint4*)((unsigned char*)Vs + off) = vv[it];
    }
  }
  for (int k = tid; k < S; k += 64 * NQB)
    km[k] = cu_seqlens ? (uint8_t)(k < L) : (kmask ? kmask[(int64_t)b * S + k] : (uint8_t)1);
  __syncthreads();  // K, V and km staged
  if (!active) return;
  f32x16 x[NQB];
#pragma unroll
  for (int kb = 0; kb < NQB; ++kb) x[kb] = f32x16{};
#pragma unroll
  for (int kb = 0; kb < NQB; ++kb) {
    if (kb < nkb) {
      const int key = kb * 32 + r;
#pragma unroll
      for (int ds = 0; ds < 4; ++ds) {
        const int ch = 2 * ds + hh;
        const bf16x8 kf = *(const bf16x8*)((unsigned char*)Ks + 128 * key + 16 * (ch ^ (((key >> 1) & 1) << 2)));
        x[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ds], x[kb], 0, 0, 0);
      }
    }
  }

  // softmax over the keys of query q0 + r (this lane: key rows (i&3) + 8(i>>2) + 4hh of each block)
  float m = -__builtin_inff();
#pragma unroll
  for (int kb = 0; kb < NQB; ++kb)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint32_t mk4 = kb < nkb ? *(const uint32_t*)(km + kb * 32 + 8 * g + 4 * hh) : 0u;  // 4 keys
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int i = 4 * g + t;
        const bool on = (mk4 >> (8 * t)) & 0xffu;
        const float v = on ? x[kb][i] * scale_log2 : -__builtin_inff();
        x[kb][i] = v;
        m = fmaxf(m, v);
      }
    }
  m = fmaxf(m, __shfl_xor(m, 32));
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < NQB; ++kb)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = exp2f(x[kb][i] - m);
      x[kb][i] = p;
      sum += p;
    }
  sum += __shfl_xor(sum, 32);
  const float inv = 1.f / sum;

  // Z = P·V: A = P (accumulator registers, rows = keys), B = V by transposed LDS reads: lane
  // (group g = lane >> 4, i = lane & 15) addresses key key0 + 8t + (i >> 2), dims 4 (i & 3) .. +3 of
  // its group's 16-dim block; it receives its own dim's 4 keys
  f32x16 z[2] = {f32x16{}, f32x16{}};
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg = (lane >> 4) & 1;
#pragma unroll
  for (int kb = 0; kb < NQB; ++kb) {
    if (kb >= nkb) continue;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 pa;
#pragma unroll
      for (int j = 0; j < 8; ++j) pa[j] = (__bf16)(x[kb][8 * s + j] * inv);
      const int key0 = kb * 32 + 16 * s + 4 * hh;
#pragma unroll
      for (int eb = 0; eb < 2; ++eb) {
        bf16x8 vf;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int key = key0 + 8 * t + tq, ch = eb * 4 + 2 * tg + (tp >> 1);
          const int off = 128 * key + 16 * (ch ^ (((key >> 1) & 1) << 2)) + 8 * (tp & 1);
          const v4i16 w = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4i16*)((unsigned char*)Vs + off));
#pragma unroll
          for (int j = 0; j < 4; ++j) vf[4 * t + j] = __builtin_bit_cast(__bf16, (short)w[j]);
        }
        z[eb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, vf, z[eb], 0, 0, 0);
      }
    }
  }
  // store: z[eb][i] = Z[query (i&3)+8(i>>2)+4hh][e = eb*32 + r]; queries past the length skipped
#pragma unroll
  for (int eb = 0; eb < 2; ++eb)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int q = q0 + (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (q < L) out[(base + q) * H * DH + h * DH + eb * 32 + r] = f2bf(z[eb][i]);
    }
}

}  // namespace svoc

// qkv: [B, S, 3, H, 64] bf16 contiguous; kmask: [B, S] uint8 (1 = attend) or null; out: [B, S, H, 64].
// Packed variant: cu_seqlens [B + 1] (device) with sequence b at rows [cu[b], cu[b+1]), lengths <= S;
// qkv: [rows_total, 3, H, 64], out: [rows_total, H, 64].
extern "C" int svoc_attention_short_bf16(const void* qkv, const void* kmask, const int* cu_seqlens, int64_t rows_total,
                                         void* out, int64_t B, int S, int H, int DH, hipStream_t stream) {
  if (DH != 64 || S % 32 != 0 || S < 32 || S > 128 || B * H > 0x7fffffffll) return -1;
  if (B == 0) return 0;
  const float scale_log2 = 1.4426950408889634f / 8.f;  // log2(e) / sqrt(64)
  const auto* Q = (const uint16_t*)qkv;
  const auto* M = (const uint8_t*)kmask;
  auto* O = (uint16_t*)out;
  const int64_t R = cu_seqlens ? rows_total : B * S;
  const dim3 grid((unsigned)(B * H));
  switch (S / 32) {
    case 1: hipLaunchKernelGGL(attn_short_kernel<1>, grid, dim3(64), 0, stream, Q, M, cu_seqlens, R, O, H, scale_log2); break;
    case 2: hipLaunchKernelGGL(attn_short_kernel<2>, grid, dim3(128), 0, stream, Q, M, cu_seqlens, R, O, H, scale_log2); break;
    case 3: hipLaunchKernelGGL(attn_short_kernel<3>, grid, dim3(192), 0, stream, Q, M, cu_seqlens, R, O, H, scale_log2); break;
    default: hipLaunchKernelGGL(attn_short_kernel<4>, grid, dim3(256), 0, stream, Q, M, cu_seqlens, R, O, H, scale_log2); break;
  }
  return (int)hipGetLastError();
}

extern "C" int svoc_embed_layernorm_bf16(const int64_t* ids, const int64_t* pos_ids, const void* tok, const void* pos,
                                         const void* typ, const void* w, const void* b, void* out, int64_t rows, int H,
                                         float eps, hipStream_t stream) {
  if (rows <= 0) return 0;
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  const auto* T = (const uint16_t*)tok;
  const auto* P = (const uint16_t*)pos;
  const auto* Y = (const uint16_t*)typ;
  const auto* W = (const uint16_t*)w;
  const auto* B = (const uint16_t*)b;
  auto* O = (uint16_t*)out;
  switch (H) {
    case 256: hipLaunchKernelGGL(embed_layernorm_kernel<4>, grid, block, 0, stream, ids, pos_ids, T, P, Y, W, B, O, rows, eps); break;
    case 512: hipLaunchKernelGGL(embed_layernorm_kernel<8>, grid, block, 0, stream, ids, pos_ids, T, P, Y, W, B, O, rows, eps); break;
    case 768: hipLaunchKernelGGL(embed_layernorm_kernel<12>, grid, block, 0, stream, ids, pos_ids, T, P, Y, W, B, O, rows, eps); break;
    case 1024: hipLaunchKernelGGL(embed_layernorm_kernel<16>, grid, block, 0, stream, ids, pos_ids, T, P, Y, W, B, O, rows, eps); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int svoc_segment_mean_bf16(const void* x, const int* cu, void* out, int64_t B, int H, hipStream_t stream) {
  if (B <= 0) return 0;
  if (H % 8 != 0 || H / 8 > 256 || B > 0x7fffffffll) return -1;
  const int chunks = H / 8;
  int G = 256 / chunks;
  if (G > 8) G = 8;
  hipLaunchKernelGGL(segment_mean_kernel, dim3((unsigned)B), dim3(chunks * G), 0, stream, (const uint16_t*)x, cu,
                     (uint16_t*)out, H, G);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// fp32 variants (the reference's precision: the HF pipeline runs the classifier in fp32,
// client/oracle_scheduler.py:23-40).  Same one-wave-per-row layout as the bf16 kernels, 16-B loads
// of 4 floats; the adds happen in fp32 in the order of the PyTorch expressions they replace.
// ---------------------------------------------------------------------------------------------
namespace svoc {

template <int EPL>
__device__ __forceinline__ void ln_store_f32(const float (&v)[EPL], float s, const float* __restrict__ w,
                                             const float* __restrict__ bias, float* __restrict__ orow, float eps,
                                             int lane) {
  constexpr int H = 64 * EPL, V = EPL / 4;
  const float mean = wave_sum(s) * (1.f / H);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) * (1.f / H) + eps);
  const float4* wr = (const float4*)w;
  const float4* br = (const float4*)bias;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int c = k * 64 + lane;
    const float4 gw = wr[c], gb = br[c];
    float4 o;
    o.x = (v[4 * k] - mean) * rstd * gw.x + gb.x;
    o.y = (v[4 * k + 1] - mean) * rstd * gw.y + gb.y;
    o.z = (v[4 * k + 2] - mean) * rstd * gw.z + gb.z;
    o.w = (v[4 * k + 3] - mean) * rstd * gw.w + gb.w;
    ((float4*)orow)[c] = o;
  }
}

template <int EPL>
__global__ __launch_bounds__(256) void add_layernorm_f32_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ bias, float* __restrict__ out,
                                                                int64_t rows, float eps, int64_t y_stride) {
  constexpr int H = 64 * EPL, V = EPL / 4;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float4* xr = (const float4*)(x + row * H);
  const float4* yr = (const float4*)(y + row * y_stride);
  float v[EPL];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int c = k * 64 + lane;
    const float4 a = xr[c], b = yr[c];
    v[4 * k] = a.x + b.x;
    v[4 * k + 1] = a.y + b.y;
    v[4 * k + 2] = a.z + b.z;
    v[4 * k + 3] = a.w + b.w;
    s += (v[4 * k] + v[4 * k + 1]) + (v[4 * k + 2] + v[4 * k + 3]);
  }
  ln_store_f32<EPL>(v, s, w, bias, out + row * H, eps, lane);
}

template <int EPL>
__global__ __launch_bounds__(256) void embed_layernorm_f32_kernel(const int64_t* __restrict__ ids,
                                                                  const int64_t* __restrict__ pos_ids,
                                                                  const float* __restrict__ tok,
                                                                  const float* __restrict__ pos,
                                                                  const float* __restrict__ typ,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ bias,
                                                                  float* __restrict__ out, int64_t rows, float eps) {
  constexpr int H = 64 * EPL, V = EPL / 4;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float4* tr = (const float4*)(tok + ids[row] * H);
  const float4* pr = (const float4*)(pos + pos_ids[row] * H);
  const float4* yr = (const float4*)typ;
  float v[EPL];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int c = k * 64 + lane;
    const float4 a = tr[c], b = pr[c], t = yr[c];
    v[4 * k] = (a.x + b.x) + t.x;
    v[4 * k + 1] = (a.y + b.y) + t.y;
    v[4 * k + 2] = (a.z + b.z) + t.z;
    v[4 * k + 3] = (a.w + b.w) + t.w;
    s += (v[4 * k] + v[4 * k + 1]) + (v[4 * k + 2] + v[4 * k + 3]);
  }
  ln_store_f32<EPL>(v, s, w, bias, out + row * H, eps, lane);
}

// segment mean of fp32 rows: thread (g, c) sums 4 columns (one 16-B load per row) of rows g, g + G, ...
__global__ __launch_bounds__(256) void segment_mean_f32_kernel(const float* __restrict__ x, const int* __restrict__ cu,
                                                               float* __restrict__ out, int H, int G) {
  __shared__ float4 part[256];
  const int b = blockIdx.x, chunks = H / 4;
  const int tid = threadIdx.x, g = tid / chunks, c = tid % chunks;
  const int lo = cu[b], hi = cu[b + 1];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (g < G) {
    for (int t = lo + g; t < hi; t += G) {
      const float4 w = *(const float4*)(x + (int64_t)t * H + 4 * c);
      acc.x += w.x;
      acc.y += w.y;
      acc.z += w.z;
      acc.w += w.w;
    }
    part[tid] = acc;
  }
  __syncthreads();
  if (g == 0) {
    const float inv = 1.f / (float)(hi - lo > 1 ? hi - lo : 1);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int gg = 0; gg < G; ++gg) {
      const float4 p = part[gg * chunks + c];
      a.x += p.x;
      a.y += p.y;
      a.z += p.z;
      a.w += p.w;
    }
    *(float4*)(out + (int64_t)b * H + 4 * c) = make_float4(a.x * inv, a.y * inv, a.z * inv, a.w * inv);
  }
}

// ---------------------------------------------------------------------------------------------
// attn_f32_kernel: fp32 softmax(Q Kᵀ / 8) V for S <= 128, head dim 64, on v_mfma_f32_32x32x2_f32 (exact
// fp32 products, fp32 accumulation).  Same orientation as the bf16 kernel: X = K·Qᵀ puts one query per lane
// (its 64 key scores in the accumulator registers, the other 64 in lane ^ 32), so the softmax is
// lane-local plus one xor-32 exchange.  The 64 head dims are split between the two lane halves
// (instruction t sums dims t and 32 + t): every lane reads one contiguous half row of Q / K.
// Z is computed transposed, Zᵀ = Vᵀ·Pᵀ: the B operand of instruction (key block, register i) is exactly
// accumulator register x[kb][i] (keys (i&3) + 8(i>>2) + 4·hh), so P never moves; Vᵀ rows are read from
// LDS one dim per lane (conflict-free).  K / V rows are staged with a 4-float pad (272-B stride).
// ---------------------------------------------------------------------------------------------
template <int NQB>
__global__ __launch_bounds__(64 * NQB) void attn_f32_kernel(const float* __restrict__ qkv,
                                                            const uint8_t* __restrict__ kmask,
                                                            const int* __restrict__ cu_seqlens, int64_t rows_total,
                                                            float* __restrict__ out, int H, float scale_log2) {
  constexpr int S = 32 * NQB, DH = 64, RS = DH + 4;   // RS: padded LDS row stride (floats)
  __shared__ __attribute__((aligned(16))) float Ks[S * RS];
  __shared__ __attribute__((aligned(16))) float Vs[S * RS];
  __shared__ uint8_t km[S];
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int64_t ts = (int64_t)3 * H * DH;
  const int64_t base = cu_seqlens ? cu_seqlens[b] : (int64_t)b * S;
  const int L = cu_seqlens ? cu_seqlens[b + 1] - cu_seqlens[b] : S;
  const int nkb = (L + 31) >> 5;
  auto row = [&](int k) -> int64_t {
    const int64_t t = base + k;
    return t < rows_total ? t : rows_total - 1;
  };
  const float* Qb = qkv + h * DH;
  const float* Kb = Qb + H * DH;
  const float* Vb = Qb + 2 * H * DH;
  // stage K and V (16 float4 per row)
  const int nchunks = nkb * 32 * (DH / 4);
  for (int c = tid; c < nchunks; c += 64 * NQB) {
    const int key = c >> 4, ch = c & 15;
    const int64_t g = row(key) * ts + ch * 4;
    *(float4*)(Ks + key * RS + ch * 4) = *(const float4*)(Kb + g);
    *(float4*)(Vs + key * RS + ch * 4) = *(const float4*)(Vb + g);
  }
  for (int k = tid; k < S; k += 64 * NQB)
    km[k] = cu_seqlens ? (uint8_t)(k < L) : (kmask ? kmask[(int64_t)b * S + k] : (uint8_t)1);
  const int q0 = wave * 32;
  const bool active = q0 < L;
  float qf[32];
  if (active) {
    const float4* qp = (const float4*)(Qb + row(q0 + r) * ts + 32 * hh);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 v = qp[j];
      qf[4 * j] = v.x;
      qf[4 * j + 1] = v.y;
      qf[4 * j + 2] = v.z;
      qf[4 * j + 3] = v.w;
    }
  }
  __syncthreads();
  if (!active) return;
  f32x16 x[NQB];
#pragma unroll
  for (int kb = 0; kb < NQB; ++kb) {
    x[kb] = f32x16{};
    if (kb < nkb) {
      const float* kr = Ks + (kb * 32 + r) * RS + 32 * hh;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float4 kv = *(const float4*)(kr + 4 * j);
        x[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.x, qf[4 * j], x[kb], 0, 0, 0);
        x[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.y, qf[4 * j + 1], x[kb], 0, 0, 0);
        x[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.z, qf[4 * j + 2], x[kb], 0, 0, 0);
        x[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.w, qf[4 * j + 3], x[kb], 0, 0, 0);
      }
    }
  }
  // softmax over this lane's query (keys (i&3) + 8(i>>2) + 4hh of each block; lane ^ 32 the others)
  float m = -__builtin_inff();
#pragma unroll
  for (int kb = 0; kb < NQB; ++kb)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kb * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
      const bool on = kb < nkb && km[key];
      const float v = on ? x[kb][i] * scale_log2 : -__builtin_inff();
      x[kb][i] = v;
      m = fmaxf(m, v);
    }
  m = fmaxf(m, __shfl_xor(m, 32));
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < NQB; ++kb)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = exp2f(x[kb][i] - m);
      x[kb][i] = p;
      sum += p;
    }
  sum += __shfl_xor(sum, 32);
  const float inv = 1.f / sum;
  // Zᵀ[e][query] = sum over keys of V[key][e] P[query][key]
  f32x16 z[2] = {f32x16{}, f32x16{}};
#pragma unroll
  for (int kb = 0; kb < NQB; ++kb) {
    if (kb >= nkb) continue;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kb * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
#pragma unroll
      for (int eb = 0; eb < 2; ++eb)
        z[eb] = __builtin_amdgcn_mfma_f32_32x32x2f32(Vs[key * RS + eb * 32 + r], x[kb][i], z[eb], 0, 0, 0);
    }
  }
  // z[eb][i] = Zᵀ[e = eb*32 + (i&3) + 8(i>>2) + 4hh][query q0 + r]: four consecutive dims per float4
  const int q = q0 + r;
  if (q < L) {
    float* orow = out + (base + q) * H * DH + h * DH;
#pragma unroll
    for (int eb = 0; eb < 2; ++eb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int e = eb * 32 + 8 * g + 4 * hh;
        *(float4*)(orow + e) = make_float4(z[eb][4 * g] * inv, z[eb][4 * g + 1] * inv, z[eb][4 * g + 2] * inv,
                                           z[eb][4 * g + 3] * inv);
      }
  }
}

}  // namespace svoc

extern "C" int svoc_add_layernorm_f32(const float* x, const float* y, const float* w, const float* b, float* out,
                                      int64_t rows, int H, float eps, int64_t y_stride, hipStream_t stream) {
  if (rows <= 0) return 0;
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  switch (H) {
    case 256: hipLaunchKernelGGL(add_layernorm_f32_kernel<4>, grid, block, 0, stream, x, y, w, b, out, rows, eps, y_stride); break;
    case 512: hipLaunchKernelGGL(add_layernorm_f32_kernel<8>, grid, block, 0, stream, x, y, w, b, out, rows, eps, y_stride); break;
    case 768: hipLaunchKernelGGL(add_layernorm_f32_kernel<12>, grid, block, 0, stream, x, y, w, b, out, rows, eps, y_stride); break;
    case 1024: hipLaunchKernelGGL(add_layernorm_f32_kernel<16>, grid, block, 0, stream, x, y, w, b, out, rows, eps, y_stride); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int svoc_embed_layernorm_f32(const int64_t* ids, const int64_t* pos_ids, const float* tok, const float* pos,
                                        const float* typ, const float* w, const float* b, float* out, int64_t rows, int H,
                                        float eps, hipStream_t stream) {
  if (rows <= 0) return 0;
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  switch (H) {
    case 256: hipLaunchKernelGGL(embed_layernorm_f32_kernel<4>, grid, block, 0, stream, ids, pos_ids, tok, pos, typ, w, b, out, rows, eps); break;
    case 512: hipLaunchKernelGGL(embed_layernorm_f32_kernel<8>, grid, block, 0, stream, ids, pos_ids, tok, pos, typ, w, b, out, rows, eps); break;
    case 768: hipLaunchKernelGGL(embed_layernorm_f32_kernel<12>, grid, block, 0, stream, ids, pos_ids, tok, pos, typ, w, b, out, rows, eps); break;
    case 1024: hipLaunchKernelGGL(embed_layernorm_f32_kernel<16>, grid, block, 0, stream, ids, pos_ids, tok, pos, typ, w, b, out, rows, eps); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int svoc_segment_mean_f32(const float* x, const int* cu, float* out, int64_t B, int H, hipStream_t stream) {
  if (B <= 0) return 0;
  if (H % 4 != 0 || H / 4 > 256 || B > 0x7fffffffll) return -1;
  const int chunks = H / 4;
  int G = 256 / chunks;
  if (G > 8) G = 8;
  hipLaunchKernelGGL(segment_mean_f32_kernel, dim3((unsigned)B), dim3(chunks * G), 0, stream, x, cu, out, H, G);
  return (int)hipGetLastError();
}

// fp32 twin of svoc_attention_short_bf16 (same layouts and packed / padded modes)
extern "C" int svoc_attention_short_f32(const float* qkv, const void* kmask, const int* cu_seqlens, int64_t rows_total,
                                        float* out, int64_t B, int S, int H, int DH, hipStream_t stream) {
  if (DH != 64 || S % 32 != 0 || S < 32 || S > 128 || B * H > 0x7fffffffll) return -1;
  if (B == 0) return 0;
  const float scale_log2 = 1.4426950408889634f / 8.f;
  const auto* M = (const uint8_t*)kmask;
  const int64_t R = cu_seqlens ? rows_total : B * S;
  const dim3 grid((unsigned)(B * H));
  switch (S / 32) {
    case 1: hipLaunchKernelGGL(attn_f32_kernel<1>, grid, dim3(64), 0, stream, qkv, M, cu_seqlens, R, out, H, scale_log2); break;
    case 2: hipLaunchKernelGGL(attn_f32_kernel<2>, grid, dim3(128), 0, stream, qkv, M, cu_seqlens, R, out, H, scale_log2); break;
    case 3: hipLaunchKernelGGL(attn_f32_kernel<3>, grid, dim3(192), 0, stream, qkv, M, cu_seqlens, R, out, H, scale_log2); break;
    default: hipLaunchKernelGGL(attn_f32_kernel<4>, grid, dim3(256), 0, stream, qkv, M, cu_seqlens, R, out, H, scale_log2); break;
  }
  return (int)hipGetLastError();
}

// ---- fp32 GEMMs on the bf16 matrix cores: three-way split ------------------------------------------------
// x = x0 + x1 + x2 with x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1) (each difference is exact in
// fp32): 24 significant bits, the fp32 mantissa.  Row r of the output holds [x0 | x1 | x2] (3K bf16), so the
// encoder's emulated fp32 linear (encoder.py _emul_linear) runs X W^T as three bf16 GEMMs with fp32 outputs,
// [x0|x1|x2] [w0|w0|w0]^T + [x0|x1] [w1|w1]^T + x0 w2^T: the six products above 2^-24 (the dropped x1 w2,
// x2 w1, x2 w2 are below it) at the bf16 MFMA rate, 16x the fp32 one on gfx950.  GELU = 1 applies RoBERTa's
// erf GELU to x first (the FC1 output -> the FC2 input).  4 elements per thread: one 16-byte load, three
// 8-byte stores.
namespace svoc {

template <bool GELU>
__global__ __launch_bounds__(256) void split3_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ out,
                                                          int64_t rows, int K) {
  const int kq = K / 4;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= rows * kq) return;
  const int64_t r = t / kq;
  const int c = (int)(t - r * kq) * 4;
  float4 v = *(const float4*)(x + r * K + c);
  float a[4] = {v.x, v.y, v.z, v.w};
  uint16_t h0[4], h1[4], h2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float f = a[i];
    if (GELU) f = 0.5f * f * (1.f + erff(f * 0.70710678118654752440f));
    h0[i] = f2bf(f);
    const float r1 = f - bf2f(h0[i]);
    h1[i] = f2bf(r1);
    h2[i] = f2bf(r1 - bf2f(h1[i]));
  }
  uint16_t* o = out + r * 3 * (int64_t)K + c;
  auto pack = [](const uint16_t (&h)[4]) {
    return make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
  };
  *(uint2*)o = pack(h0);
  *(uint2*)(o + K) = pack(h1);
  *(uint2*)(o + 2 * K) = pack(h2);
}

}  // namespace svoc

extern "C" int svoc_split3_bf16(const float* x, void* out, int64_t rows, int K, int gelu, hipStream_t stream) {
  using namespace svoc;
  if (rows <= 0) return 0;
  if (K % 4 != 0 || K <= 0) return -1;
  const int64_t n = rows * (K / 4);
  const int64_t blocks = (n + 255) / 256;
  if (blocks > 0x7fffffffll) return -1;
  if (gelu) hipLaunchKernelGGL(split3_bf16_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, stream, x, (uint16_t*)out, rows, K);
  else hipLaunchKernelGGL(split3_bf16_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, stream, x, (uint16_t*)out, rows, K);
  return (int)hipGetLastError();
}

