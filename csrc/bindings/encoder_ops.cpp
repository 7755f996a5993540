// torch.ops.svoc.add_layernorm: fused residual add + LayerNorm for the sentiment encoder.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <cmath>
#include <limits>

#include "svoc/ops.hpp"

extern "C" int svoc_add_layernorm_bf16(const void* x, const void* y, const void* w, const void* b, void* out,
                                       int64_t rows, int H, float eps, int64_t y_stride, hipStream_t stream);
extern "C" int svoc_embed_layernorm_bf16(const int64_t* ids, const int64_t* pos_ids, const void* tok, const void* pos,
                                         const void* typ, const void* w, const void* b, void* out, int64_t rows, int H,
                                         float eps, hipStream_t stream);
extern "C" int svoc_segment_mean_bf16(const void* x, const int* cu, void* out, int64_t B, int H, hipStream_t stream);
extern "C" int svoc_add_layernorm_f32(const float* x, const float* y, const float* w, const float* b, float* out,
                                      int64_t rows, int H, float eps, int64_t y_stride, hipStream_t stream);
extern "C" int svoc_embed_layernorm_f32(const int64_t* ids, const int64_t* pos_ids, const float* tok, const float* pos,
                                        const float* typ, const float* w, const float* b, float* out, int64_t rows, int H,
                                        float eps, hipStream_t stream);
extern "C" int svoc_segment_mean_f32(const float* x, const int* cu, float* out, int64_t B, int H, hipStream_t stream);
extern "C" int svoc_split3_bf16(const float* x, void* out, int64_t rows, int K, int gelu, hipStream_t stream);
extern "C" int svoc_attention_short_f32(const float* qkv, const void* kmask, const int* cu_seqlens, int64_t rows_total,
                                        float* out, int64_t B, int S, int H, int DH, hipStream_t stream);

namespace svoc {
namespace {

at::Tensor add_layernorm_ref(const at::Tensor& x, const at::Tensor& y, const at::Tensor& w, const at::Tensor& b,
                             double eps) {
  const int64_t H = x.size(-1);
  return at::layer_norm(x + y, {H}, w, b, eps);
}

at::Tensor add_layernorm_cpu(const at::Tensor& x, const at::Tensor& y, const at::Tensor& w, const at::Tensor& b,
                             double eps) {
  return add_layernorm_ref(x, y, w, b, eps);
}

bool hip_supported(int64_t H) { return H == 256 || H == 512 || H == 768 || H == 1024; }

at::Tensor add_layernorm_hip(const at::Tensor& x, const at::Tensor& y, const at::Tensor& w, const at::Tensor& b,
                             double eps) {
  const int64_t H = x.size(-1);
  const bool y_row = y.dim() == 1 && y.numel() == H;   // one [H] row broadcast over x's rows
  TORCH_CHECK(y_row || x.sizes() == y.sizes(), "add_layernorm: y must have x's shape or be one [H] row");
  TORCH_CHECK(w.numel() == H && b.numel() == H, "add_layernorm: weight/bias must have H elements");
  const auto dt = x.scalar_type();
  const bool same = y.scalar_type() == dt && w.scalar_type() == dt && b.scalar_type() == dt;
  const bool fast = same && (dt == at::kBFloat16 || dt == at::kFloat) && hip_supported(H);
  if (!fast) return add_layernorm_ref(x, y, w, b, eps);  // other dtypes / widths: ATen (documented)
  auto xc = x.contiguous(), yc = y.contiguous(), wc = w.contiguous(), bc = b.contiguous();
  auto out = at::empty_like(xc);
  if (dt == at::kFloat) {
    const int rc = svoc_add_layernorm_f32(xc.data_ptr<float>(), yc.data_ptr<float>(), wc.data_ptr<float>(),
                                          bc.data_ptr<float>(), out.data_ptr<float>(), xc.numel() / H, (int)H,
                                          (float)eps, y_row ? 0 : H,
                                          c10::hip::getCurrentHIPStream(x.device().index()).stream());
    TORCH_CHECK(rc == 0, "svoc_add_layernorm_f32 failed: ", rc);
    return out;
  }
  const int rc = svoc_add_layernorm_bf16(xc.data_ptr(), yc.data_ptr(), wc.data_ptr(), bc.data_ptr(), out.data_ptr(),
                                         xc.numel() / H, (int)H, (float)eps, y_row ? 0 : H,
                                         c10::hip::getCurrentHIPStream(x.device().index()).stream());
  TORCH_CHECK(rc == 0, "svoc_add_layernorm_bf16 failed: ", rc);
  return out;
}

// embeddings: LayerNorm(tok[ids] + pos[pos_ids] + typ[0]) (the sum in the weights' dtype, as the
// PyTorch expression it replaces)
at::Tensor embed_layernorm_ref(const at::Tensor& ids, const at::Tensor& pos_ids, const at::Tensor& tok,
                               const at::Tensor& pos, const at::Tensor& typ, const at::Tensor& w, const at::Tensor& b,
                               double eps) {
  const int64_t H = tok.size(1);
  auto e = tok.index_select(0, ids) + pos.index_select(0, pos_ids) + typ.reshape({-1, H}).select(0, 0);
  return at::layer_norm(e, {H}, w, b, eps);
}

at::Tensor embed_layernorm_cpu(const at::Tensor& ids, const at::Tensor& pos_ids, const at::Tensor& tok,
                               const at::Tensor& pos, const at::Tensor& typ, const at::Tensor& w, const at::Tensor& b,
                               double eps) {
  return embed_layernorm_ref(ids, pos_ids, tok, pos, typ, w, b, eps);
}

at::Tensor embed_layernorm_hip(const at::Tensor& ids, const at::Tensor& pos_ids, const at::Tensor& tok,
                               const at::Tensor& pos, const at::Tensor& typ, const at::Tensor& w, const at::Tensor& b,
                               double eps) {
  TORCH_CHECK(ids.dim() == 1 && pos_ids.sizes() == ids.sizes(), "ids / pos_ids: [T]");
  TORCH_CHECK(tok.dim() == 2 && pos.dim() == 2 && pos.size(1) == tok.size(1), "tok / pos tables: [V, H]");
  const int64_t H = tok.size(1);
  TORCH_CHECK(typ.numel() >= H && w.numel() == H && b.numel() == H, "typ / weight / bias: H elements");
  const auto bf = tok.scalar_type();
  const bool fast = (bf == at::kBFloat16 || bf == at::kFloat) && pos.scalar_type() == bf && typ.scalar_type() == bf &&
                    w.scalar_type() == bf && b.scalar_type() == bf && hip_supported(H);
  if (!fast) return embed_layernorm_ref(ids, pos_ids, tok, pos, typ, w, b, eps);
  auto ic = ids.to(at::kLong).contiguous(), pc = pos_ids.to(at::kLong).contiguous();
  auto tc = tok.contiguous(), qc = pos.contiguous(), yc = typ.contiguous(), wc = w.contiguous(), bc = b.contiguous();
  auto out = at::empty({ids.size(0), H}, tc.options());
  if (bf == at::kFloat) {
    const int rc = svoc_embed_layernorm_f32(ic.data_ptr<int64_t>(), pc.data_ptr<int64_t>(), tc.data_ptr<float>(),
                                            qc.data_ptr<float>(), yc.data_ptr<float>(), wc.data_ptr<float>(),
                                            bc.data_ptr<float>(), out.data_ptr<float>(), ids.size(0), (int)H, (float)eps,
                                            c10::hip::getCurrentHIPStream(tok.device().index()).stream());
    TORCH_CHECK(rc == 0, "svoc_embed_layernorm_f32 failed: ", rc);
    return out;
  }
  const int rc = svoc_embed_layernorm_bf16(ic.data_ptr<int64_t>(), pc.data_ptr<int64_t>(), tc.data_ptr(), qc.data_ptr(),
                                           yc.data_ptr(), wc.data_ptr(), bc.data_ptr(), out.data_ptr(), ids.size(0),
                                           (int)H, (float)eps, c10::hip::getCurrentHIPStream(tok.device().index()).stream());
  TORCH_CHECK(rc == 0, "svoc_embed_layernorm_bf16 failed: ", rc);
  return out;
}

// mean of x[t] over each segment [cu[b], cu[b+1]) (fp32 sums, empty segment -> 0)
at::Tensor segment_mean_ref(const at::Tensor& x, const at::Tensor& cu) {
  const int64_t B = cu.numel() - 1, H = x.size(1);
  auto cul = cu.to(at::kLong);
  auto lens = cul.slice(0, 1) - cul.slice(0, 0, B);
  auto seg = at::repeat_interleave(at::arange(B, cul.options()), lens, c10::nullopt);
  auto s = at::zeros({B, H}, x.options().dtype(at::kFloat)).index_add_(0, seg, x.to(at::kFloat));
  return (s / lens.clamp_min(1).to(at::kFloat).unsqueeze(1)).to(x.scalar_type());
}

at::Tensor segment_mean_cpu(const at::Tensor& x, const at::Tensor& cu) { return segment_mean_ref(x, cu); }

at::Tensor segment_mean_hip(const at::Tensor& x, const at::Tensor& cu) {
  TORCH_CHECK(x.dim() == 2 && cu.dim() == 1 && cu.numel() >= 1, "x: [T, H], cu_seqlens: [B + 1]");
  TORCH_CHECK(cu.scalar_type() == at::kInt && cu.is_contiguous() && cu.device() == x.device(),
              "cu_seqlens: int32 on the device");
  const int64_t B = cu.numel() - 1, H = x.size(1);
  if (x.scalar_type() == at::kFloat && H % 4 == 0 && H / 4 <= 256) {
    auto xc = x.contiguous();
    auto out = at::empty({B, H}, xc.options());
    const int rc = svoc_segment_mean_f32(xc.data_ptr<float>(), cu.data_ptr<int>(), out.data_ptr<float>(), B, (int)H,
                                         c10::hip::getCurrentHIPStream(x.device().index()).stream());
    TORCH_CHECK(rc == 0, "svoc_segment_mean_f32 failed: ", rc);
    return out;
  }
  if (x.scalar_type() != at::kBFloat16 || H % 8 != 0 || H / 8 > 256) return segment_mean_ref(x, cu);
  auto xc = x.contiguous();
  auto out = at::empty({B, H}, xc.options());
  const int rc = svoc_segment_mean_bf16(xc.data_ptr(), cu.data_ptr<int>(), out.data_ptr(), B, (int)H,
                                        c10::hip::getCurrentHIPStream(x.device().index()).stream());
  TORCH_CHECK(rc == 0, "svoc_segment_mean_bf16 failed: ", rc);
  return out;
}

// [rows, K] fp32 -> [rows, 3K] bf16 planes [x0 | x1 | x2] of the three-way split (encoder_ops.hip
// split3_bf16_kernel); gelu: RoBERTa's erf GELU first.  The CPU form is the reference of the same arithmetic.
at::Tensor split3_ref(const at::Tensor& x, bool gelu) {
  auto f = x.to(at::kFloat);
  if (gelu) f = at::gelu(f);
  auto x0 = f.to(at::kBFloat16);
  auto r1 = f - x0.to(at::kFloat);
  auto x1 = r1.to(at::kBFloat16);
  auto x2 = (r1 - x1.to(at::kFloat)).to(at::kBFloat16);
  return at::cat({x0, x1, x2}, -1);
}

at::Tensor split3_cpu(const at::Tensor& x, bool gelu) { return split3_ref(x, gelu); }

at::Tensor split3_hip(const at::Tensor& x, bool gelu) {
  TORCH_CHECK(x.dim() == 2, "split3: x must be [rows, K]");
  TORCH_CHECK(x.scalar_type() == at::kFloat, "split3: fp32 input");
  const int64_t rows = x.size(0), K = x.size(1);
  if (K % 4 != 0) return split3_ref(x, gelu);
  auto xc = x.contiguous();
  auto out = at::empty({rows, 3 * K}, xc.options().dtype(at::kBFloat16));
  const int rc = svoc_split3_bf16(xc.data_ptr<float>(), out.data_ptr(), rows, (int)K, gelu ? 1 : 0,
                                  c10::hip::getCurrentHIPStream(x.device().index()).stream());
  TORCH_CHECK(rc == 0, "svoc_split3_bf16 failed: ", rc);
  return out;
}

}  // namespace

void register_attention_defs(torch::Library& m);
void register_attention_cpu(torch::Library& m);
void register_attention_hip(torch::Library& m);

void register_encoder_defs(torch::Library& m) {
  m.def("add_layernorm(Tensor x, Tensor y, Tensor weight, Tensor bias, float eps) -> Tensor");
  m.def("embed_layernorm(Tensor ids, Tensor pos_ids, Tensor tok, Tensor pos, Tensor typ, Tensor weight, Tensor bias, "
        "float eps) -> Tensor");
  m.def("segment_mean(Tensor x, Tensor cu_seqlens) -> Tensor");
  m.def("split3(Tensor x, bool gelu) -> Tensor");
  register_attention_defs(m);
}
void register_encoder_cpu(torch::Library& m) {
  m.impl("add_layernorm", &add_layernorm_cpu);
  m.impl("embed_layernorm", &embed_layernorm_cpu);
  m.impl("segment_mean", &segment_mean_cpu);
  m.impl("split3", &split3_cpu);
  register_attention_cpu(m);
}
void register_encoder_hip(torch::Library& m) {
  m.impl("add_layernorm", &add_layernorm_hip);
  m.impl("embed_layernorm", &embed_layernorm_hip);
  m.impl("segment_mean", &segment_mean_hip);
  m.impl("split3", &split3_hip);
  register_attention_hip(m);
}

}  // namespace svoc

extern "C" int svoc_attention_short_bf16(const void* qkv, const void* kmask, const int* cu_seqlens,
                                         int64_t rows_total, void* out, int64_t B, int S, int H, int DH,
                                         hipStream_t stream);

namespace svoc {
namespace {

// qkv [B, S, 3*H*DH] -> [B, S, H*DH]; key_mask [B, S] (nonzero = attend)
at::Tensor attention_ref(const at::Tensor& qkv, const c10::optional<at::Tensor>& key_mask, int64_t heads) {
  const int64_t B = qkv.size(0), S = qkv.size(1), HD = qkv.size(2) / 3, DH = HD / heads;
  auto t = qkv.view({B, S, 3, heads, DH}).permute({2, 0, 3, 1, 4});
  auto q = t[0].to(at::kFloat), k = t[1].to(at::kFloat), v = t[2].to(at::kFloat);
  auto s = at::matmul(q, k.transpose(-1, -2)) / std::sqrt((double)DH);
  if (key_mask.has_value()) {
    auto m = key_mask->to(at::kBool).view({B, 1, 1, S});
    s = s.masked_fill(m.logical_not(), -std::numeric_limits<float>::infinity());
  }
  auto o = at::matmul(at::softmax(s, -1), v);  // [B, H, S, DH]
  return o.transpose(1, 2).reshape({B, S, HD}).to(qkv.scalar_type());
}

at::Tensor attention_cpu(const at::Tensor& qkv, const c10::optional<at::Tensor>& key_mask, int64_t heads) {
  return attention_ref(qkv, key_mask, heads);
}

at::Tensor attention_hip(const at::Tensor& qkv, const c10::optional<at::Tensor>& key_mask, int64_t heads) {
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) % (3 * heads) == 0, "qkv: [B, S, 3*H*DH]");
  const int64_t B = qkv.size(0), S = qkv.size(1), HD = qkv.size(2) / 3, DH = HD / heads;
  const bool f32 = qkv.scalar_type() == at::kFloat;
  const bool ok = (qkv.scalar_type() == at::kBFloat16 || f32) && DH == 64 && S % 32 == 0 && S >= 32 && S <= 128;
  if (!ok) return attention_ref(qkv, key_mask, heads);  // other shapes: ATen (documented)
  auto x = qkv.contiguous();
  at::Tensor m;
  if (key_mask.has_value()) {
    TORCH_CHECK(key_mask->numel() == B * S, "key_mask: [B, S]");
    m = key_mask->to(at::kByte).contiguous();
  }
  auto out = at::empty({B, S, HD}, x.options());
  if (f32) {
    const int rc = svoc_attention_short_f32(x.data_ptr<float>(), key_mask.has_value() ? m.data_ptr() : nullptr, nullptr,
                                            0, out.data_ptr<float>(), B, (int)S, (int)heads, (int)DH,
                                            c10::hip::getCurrentHIPStream(x.device().index()).stream());
    TORCH_CHECK(rc == 0, "svoc_attention_short_f32 failed: ", rc);
    return out;
  }
  const int rc = svoc_attention_short_bf16(x.data_ptr(), key_mask.has_value() ? m.data_ptr() : nullptr, nullptr, 0,
                                           out.data_ptr(), B, (int)S, (int)heads, (int)DH,
                                           c10::hip::getCurrentHIPStream(x.device().index()).stream());
  TORCH_CHECK(rc == 0, "svoc_attention_short_bf16 failed: ", rc);
  return out;
}

// packed (unpadded) tokens: qkv [T, 3*H*DH], sequence b = rows [cu[b], cu[b+1])
at::Tensor attention_varlen_ref(const at::Tensor& qkv, const at::Tensor& cu, int64_t max_len, int64_t heads) {
  (void)max_len;
  const int64_t T = qkv.size(0), HD = qkv.size(1) / 3, DH = HD / heads;
  auto cuh = cu.to(at::kCPU, at::kLong);
  auto out = at::empty({T, HD}, qkv.options());
  for (int64_t b = 0; b + 1 < cuh.numel(); ++b) {
    const int64_t lo = cuh[b].item<int64_t>(), hi = cuh[b + 1].item<int64_t>();
    if (hi <= lo) continue;
    auto t = qkv.slice(0, lo, hi).view({hi - lo, 3, heads, DH}).permute({1, 2, 0, 3}).to(at::kFloat);
    auto s = at::matmul(t[0], t[1].transpose(-1, -2)) / std::sqrt((double)DH);
    auto o = at::matmul(at::softmax(s, -1), t[2]);  // [heads, L, DH]
    out.slice(0, lo, hi).copy_(o.transpose(0, 1).reshape({hi - lo, HD}));
  }
  return out;
}

at::Tensor attention_varlen_cpu(const at::Tensor& qkv, const at::Tensor& cu, int64_t max_len, int64_t heads) {
  return attention_varlen_ref(qkv, cu, max_len, heads);
}

at::Tensor attention_varlen_hip(const at::Tensor& qkv, const at::Tensor& cu, int64_t max_len, int64_t heads) {
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(1) % (3 * heads) == 0, "qkv: [T, 3*H*DH]");
  TORCH_CHECK(cu.scalar_type() == at::kInt && cu.dim() == 1 && cu.is_contiguous() && cu.device() == qkv.device(),
              "cu_seqlens: int32 [B+1] on the device");
  const int64_t T = qkv.size(0), HD = qkv.size(1) / 3, DH = HD / heads, B = cu.numel() - 1;
  const int64_t S = (max_len + 31) / 32 * 32;
  const bool f32 = qkv.scalar_type() == at::kFloat;
  const bool ok = (qkv.scalar_type() == at::kBFloat16 || f32) && DH == 64 && S >= 32 && S <= 128;
  if (!ok) return attention_varlen_ref(qkv, cu, max_len, heads);
  auto x = qkv.contiguous();
  auto out = at::empty({T, HD}, x.options());
  if (T == 0) return out;
  if (f32) {
    const int rc = svoc_attention_short_f32(x.data_ptr<float>(), nullptr, cu.data_ptr<int>(), T, out.data_ptr<float>(),
                                            B, (int)S, (int)heads, (int)DH,
                                            c10::hip::getCurrentHIPStream(x.device().index()).stream());
    TORCH_CHECK(rc == 0, "svoc_attention_short_f32 (varlen) failed: ", rc);
    return out;
  }
  const int rc = svoc_attention_short_bf16(x.data_ptr(), nullptr, cu.data_ptr<int>(), T, out.data_ptr(), B, (int)S,
                                           (int)heads, (int)DH,
                                           c10::hip::getCurrentHIPStream(x.device().index()).stream());
  TORCH_CHECK(rc == 0, "svoc_attention_short_bf16 (varlen) failed: ", rc);
  return out;
}

}  // namespace

void register_attention_defs(torch::Library& m) {
  m.def("attention_qkv(Tensor qkv, Tensor? key_mask, int heads) -> Tensor");
  m.def("attention_varlen(Tensor qkv, Tensor cu_seqlens, int max_len, int heads) -> Tensor");
}
void register_attention_cpu(torch::Library& m) {
  m.impl("attention_qkv", &attention_cpu);
  m.impl("attention_varlen", &attention_varlen_cpu);
}
void register_attention_hip(torch::Library& m) {
  m.impl("attention_qkv", &attention_hip);
  m.impl("attention_varlen", &attention_varlen_hip);
}

}  // namespace svoc
