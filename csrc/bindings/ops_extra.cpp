// Extra torch.ops.svoc ops: batched updates (storage half of update_prediction).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <cmath>
#include <initializer_list>
#include <utility>
#include <cstring>

#include "svoc/launch.hpp"
#include "svoc/ops.hpp"
#include "svoc/status.hpp"

namespace svoc {
namespace {

// every tensor a kernel dereferences must live on the state's device (a CPU index tensor handed to a GPU
// kernel would be read through a host pointer)
void same_device(const at::Tensor& ref, std::initializer_list<std::pair<const at::Tensor*, const char*>> ts) {
  for (const auto& t : ts)
    TORCH_CHECK(t.first->device() == ref.device(), t.second, " must be on ", ref.device(), " (got ",
                t.first->device(), ")");
}

int dtype_code(at::ScalarType t) {
  if (t == at::kBFloat16) return 0;
  if (t == at::kFloat) return 1;
  if (t == at::kLong) return 2;
  if (t == at::kInt) return 3;
  TORCH_CHECK(false, "values dtype must be bf16, fp32, int64 or int32 (wsad)");
  return -1;
}

UpdateParams make_update_params(at::Tensor& values, at::Tensor& enabled, at::Tensor& n_active,
                                at::Tensor& touched, const at::Tensor& inst, const at::Tensor& oracle,
                                const at::Tensor& upd, bool constrained, at::Tensor& upd_status) {
  TORCH_CHECK(values.dim() == 3 && values.stride(2) == 1 && values.stride(1) == values.size(2),
              "values: [B, N, ld] with dense rows");
  const int64_t B = values.size(0), N = values.size(1), U = inst.numel();
  TORCH_CHECK(upd.dim() == 2 && upd.size(0) == U && upd.is_contiguous(), "upd: contiguous [U, D]");
  TORCH_CHECK(upd.scalar_type() == values.scalar_type(), "upd dtype must match values");
  TORCH_CHECK(upd.size(1) <= values.size(2), "D > ld");
  TORCH_CHECK(oracle.numel() == U && inst.scalar_type() == at::kLong && oracle.scalar_type() == at::kLong,
              "inst/oracle: int64 [U]");
  TORCH_CHECK(inst.is_contiguous() && oracle.is_contiguous(), "inst/oracle contiguous");
  TORCH_CHECK(enabled.scalar_type() == at::kByte && enabled.numel() == B * N && enabled.is_contiguous(),
              "enabled: uint8 [B, N]");
  TORCH_CHECK(n_active.scalar_type() == at::kInt && n_active.numel() == B && n_active.is_contiguous(),
              "n_active: int32 [B]");
  TORCH_CHECK(touched.scalar_type() == at::kByte && touched.numel() == B, "touched: uint8 [B]");
  TORCH_CHECK(upd_status.scalar_type() == at::kInt && upd_status.numel() == U, "upd_status: int32 [U]");
  same_device(values, {{&enabled, "enabled"}, {&n_active, "n_active"}, {&touched, "touched"}, {&inst, "inst"},
                       {&oracle, "oracle"}, {&upd, "upd"}, {&upd_status, "upd_status"}});
  UpdateParams p{};
  p.values = values.data_ptr();
  p.enabled = enabled.data_ptr<uint8_t>();
  p.n_active = n_active.data_ptr<int32_t>();
  p.touched = touched.data_ptr<uint8_t>();
  p.inst = inst.data_ptr<int64_t>();
  p.oracle = oracle.data_ptr<int64_t>();
  p.upd = upd.data_ptr();
  p.upd_status = upd_status.data_ptr<int32_t>();
  p.inst_stride = values.stride(0);
  p.B = (int)B; p.N = (int)N; p.D = (int)upd.size(1); p.ld = (int)values.size(2); p.U = (int)U;
  p.dtype = dtype_code(values.scalar_type());
  p.elem_bytes = (int)values.element_size();
  p.constrained = constrained ? 1 : 0;
  return p;
}

bool in_range_cpu(const UpdateParams& p, int64_t u, int d) {
  if (p.dtype == 0) {
    uint32_t w = (uint32_t)((const uint16_t*)p.upd)[u * p.D + d] << 16;
    float f;
    std::memcpy(&f, &w, 4);
    return f >= 0.f && f <= 1.f;
  }
  if (p.dtype == 1) {
    const float f = ((const float*)p.upd)[u * p.D + d];
    return f >= 0.f && f <= 1.f;
  }
  const int64_t v = p.dtype == 3 ? (int64_t)((const int32_t*)p.upd)[u * p.D + d] : ((const int64_t*)p.upd)[u * p.D + d];
  return v >= 0 && v <= 1000000;
}

// transactional streaming buffers (optional): saved [U, D] in the values' dtype, saved_en uint8 [U]
void set_saved(UpdateParams& p, const c10::optional<at::Tensor>& saved, const c10::optional<at::Tensor>& saved_en,
               const at::Tensor& upd) {
  p.saved = nullptr;
  p.saved_en = nullptr;
  if (!saved.has_value() || !saved->defined()) return;
  TORCH_CHECK(saved_en.has_value() && saved_en->defined(), "saved and saved_en go together");
  TORCH_CHECK(saved->scalar_type() == upd.scalar_type() && saved->is_contiguous() && saved->dim() == 2 &&
                  saved->size(0) == upd.size(0) && saved->size(1) == upd.size(1),
              "saved: contiguous [U, D] in the values' dtype");
  TORCH_CHECK(saved_en->scalar_type() == at::kByte && saved_en->is_contiguous() && saved_en->numel() == upd.size(0),
              "saved_en: uint8 [U]");
  same_device(upd, {{&*saved, "saved"}, {&*saved_en, "saved_en"}});
  p.saved = saved->data_ptr();
  p.saved_en = saved_en->data_ptr<uint8_t>();
}

void apply_updates_cpu(at::Tensor values, at::Tensor enabled, at::Tensor n_active, at::Tensor touched,
                       at::Tensor winner, const at::Tensor& inst, const at::Tensor& oracle, const at::Tensor& upd,
                       bool constrained, at::Tensor upd_status, bool unique, const c10::optional<at::Tensor>& saved,
                       const c10::optional<at::Tensor>& saved_en) {
  (void)winner;
  (void)unique;  // sequential CPU loop: last writer wins either way
  UpdateParams p = make_update_params(values, enabled, n_active, touched, inst, oracle, upd, constrained, upd_status);
  set_saved(p, saved, saved_en, upd);
  const int64_t row_bytes = (int64_t)p.D * p.elem_bytes;
  for (int64_t u = 0; u < p.U; ++u) {  // sequential = last writer wins
    const int64_t b = p.inst[u], o = p.oracle[u];
    // the contract's check order (contract.cairo:588-596): the prediction's interval check before the
    // caller's oracle lookup (as row_status in updates.hip)
    int st = ST_OK;
    if (p.constrained)
      for (int d = 0; d < p.D; ++d)
        if (!in_range_cpu(p, u, d)) { st = ST_INTERVAL_INPUT; break; }
    if (st == ST_OK && !p.constrained && p.dtype <= 1)
      for (int d = 0; d < p.D; ++d) {
        const float f = p.dtype == 1 ? ((const float*)p.upd)[u * p.D + d] : [&] {
          uint32_t w = (uint32_t)((const uint16_t*)p.upd)[u * p.D + d] << 16;
          float x;
          std::memcpy(&x, &w, 4);
          return x;
        }();
        if (!std::isfinite(f)) { st = ST_NON_FINITE; break; }
      }
    if (st == ST_OK && (b < 0 || b >= p.B || o < 0 || o >= p.N)) st = ST_NOT_ORACLE;
    p.upd_status[u] = st;
    if (p.saved_en) p.saved_en[u] = kNotSaved;
    if (st != ST_OK) continue;
    unsigned char* dst = (unsigned char*)p.values + (b * p.inst_stride + o * p.ld) * p.elem_bytes;
    if (p.saved) {
      // sequential: an earlier update of the same slot in this batch is superseded (coalesced); the
      // restore runs in reverse batch order, so every saved row is the one its update overwrote
      std::memcpy((unsigned char*)p.saved + u * row_bytes, dst, row_bytes);
      p.saved_en[u] = p.enabled[b * p.N + o];
    }
    std::memcpy(dst, (const unsigned char*)p.upd + u * row_bytes, row_bytes);
    if (!p.enabled[b * p.N + o]) {
      p.enabled[b * p.N + o] = 1;
      p.n_active[b] += 1;
    }
    p.touched[b] = 1;
  }
}

void apply_updates_hip(at::Tensor values, at::Tensor enabled, at::Tensor n_active, at::Tensor touched,
                       at::Tensor winner, const at::Tensor& inst, const at::Tensor& oracle, const at::Tensor& upd,
                       bool constrained, at::Tensor upd_status, bool unique, const c10::optional<at::Tensor>& saved,
                       const c10::optional<at::Tensor>& saved_en) {
  UpdateParams p = make_update_params(values, enabled, n_active, touched, inst, oracle, upd, constrained, upd_status);
  set_saved(p, saved, saved_en, upd);
  p.unique = unique ? 1 : 0;
  TORCH_CHECK(winner.scalar_type() == at::kInt && winner.numel() == (int64_t)p.B * p.N && winner.is_contiguous(),
              "winner workspace: int32 [B, N] filled with -1");
  p.winner = winner.data_ptr<int32_t>();
  auto stream = c10::hip::getCurrentHIPStream(values.device().index()).stream();
  const int rc = svoc_apply_updates(&p, stream);
  TORCH_CHECK(rc == 0, "svoc_apply_updates failed: ", rc);
}

RestoreParams make_restore_params(at::Tensor& values, at::Tensor& enabled, at::Tensor& n_active, const at::Tensor& inst,
                                  const at::Tensor& oracle, at::Tensor& upd_status, const at::Tensor& saved,
                                  const at::Tensor& saved_en, const at::Tensor& status, const at::Tensor& active) {
  TORCH_CHECK(values.dim() == 3 && values.stride(2) == 1 && values.stride(1) == values.size(2),
              "values: [B, N, ld] with dense rows");
  const int64_t B = values.size(0), N = values.size(1), U = inst.numel();
  TORCH_CHECK(inst.scalar_type() == at::kLong && oracle.scalar_type() == at::kLong && oracle.numel() == U &&
                  inst.is_contiguous() && oracle.is_contiguous(), "inst/oracle: contiguous int64 [U]");
  TORCH_CHECK(upd_status.scalar_type() == at::kInt && upd_status.numel() == U, "upd_status: int32 [U]");
  TORCH_CHECK(saved.scalar_type() == values.scalar_type() && saved.is_contiguous() && saved.dim() == 2 &&
                  saved.size(0) == U && saved.size(1) <= values.size(2), "saved: contiguous [U, D]");
  TORCH_CHECK(saved_en.scalar_type() == at::kByte && saved_en.numel() == U, "saved_en: uint8 [U]");
  TORCH_CHECK(status.scalar_type() == at::kInt && status.numel() == B && status.is_contiguous(), "status: int32 [B]");
  TORCH_CHECK(active.scalar_type() == at::kByte && active.numel() == B && active.is_contiguous(), "active: uint8 [B]");
  TORCH_CHECK(enabled.scalar_type() == at::kByte && enabled.numel() == B * N && n_active.scalar_type() == at::kInt &&
                  n_active.numel() == B, "enabled uint8 [B, N], n_active int32 [B]");
  same_device(values, {{&enabled, "enabled"}, {&n_active, "n_active"}, {&inst, "inst"}, {&oracle, "oracle"},
                       {&upd_status, "upd_status"}, {&saved, "saved"}, {&saved_en, "saved_en"}, {&status, "status"},
                       {&active, "active"}});
  RestoreParams p{};
  p.inactive_status = -1;
  p.values = values.data_ptr();
  p.enabled = enabled.data_ptr<uint8_t>();
  p.n_active = n_active.data_ptr<int32_t>();
  p.inst = inst.data_ptr<int64_t>();
  p.oracle = oracle.data_ptr<int64_t>();
  p.upd_status = upd_status.data_ptr<int32_t>();
  p.saved = saved.data_ptr();
  p.saved_en = saved_en.data_ptr<uint8_t>();
  p.status = status.data_ptr<int32_t>();
  p.active = active.data_ptr<uint8_t>();
  p.inst_stride = values.stride(0);
  p.B = (int)B; p.N = (int)N; p.D = (int)saved.size(1); p.ld = (int)values.size(2); p.U = (int)U;
  p.elem_bytes = (int)values.element_size();
  return p;
}

void restore_updates_cpu(at::Tensor values, at::Tensor enabled, at::Tensor n_active, const at::Tensor& inst,
                         const at::Tensor& oracle, at::Tensor upd_status, const at::Tensor& saved,
                         const at::Tensor& saved_en, const at::Tensor& status, const at::Tensor& active,
                         int64_t inactive_status) {
  RestoreParams p = make_restore_params(values, enabled, n_active, inst, oracle, upd_status, saved, saved_en, status,
                                        active);
  const int64_t row_bytes = (int64_t)p.D * p.elem_bytes;
  for (int64_t u = p.U - 1; u >= 0; --u) {   // reverse batch order (a slot updated twice: see apply)
    if (p.upd_status[u] != ST_OK) continue;
    const int64_t b = p.inst[u], o = p.oracle[u];
    if (b < 0 || b >= p.B || o < 0 || o >= p.N) continue;
    if (!p.active[b]) {
      if (inactive_status >= 0) p.upd_status[u] = (int32_t)inactive_status;
      continue;
    }
    if (p.status[b] == ST_OK) continue;
    const uint8_t was = p.saved_en[u];
    if (was != kNotSaved) {
      std::memcpy((unsigned char*)p.values + (b * p.inst_stride + o * p.ld) * p.elem_bytes,
                  (const unsigned char*)p.saved + u * row_bytes, row_bytes);
      if (was == 0) {
        p.enabled[b * p.N + o] = 0;
        p.n_active[b] -= 1;
      }
    }
    p.upd_status[u] = p.status[b];
  }
}

void restore_updates_hip(at::Tensor values, at::Tensor enabled, at::Tensor n_active, const at::Tensor& inst,
                         const at::Tensor& oracle, at::Tensor upd_status, const at::Tensor& saved,
                         const at::Tensor& saved_en, const at::Tensor& status, const at::Tensor& active,
                         int64_t inactive_status) {
  RestoreParams p = make_restore_params(values, enabled, n_active, inst, oracle, upd_status, saved, saved_en, status,
                                        active);
  p.inactive_status = (int)inactive_status;
  auto stream = c10::hip::getCurrentHIPStream(values.device().index()).stream();
  const int rc = svoc_restore_updates(&p, stream);
  TORCH_CHECK(rc == 0, "svoc_restore_updates failed: ", rc);
}

void commit_updates_hip(const at::Tensor& rows, const at::Tensor& oracle, const at::Tensor& upd_status, at::Tensor values,
                        int64_t upd_per_inst) {
  TORCH_CHECK(values.dim() == 3 && values.stride(2) == 1 && values.stride(1) == values.size(2),
              "values: [B, N, ld] with dense rows");
  const int64_t n = oracle.numel();
  TORCH_CHECK(rows.dim() == 2 && rows.size(0) == n && rows.is_contiguous() && rows.scalar_type() == values.scalar_type(),
              "rows: contiguous [n, D] in the values' dtype");
  TORCH_CHECK(oracle.scalar_type() == at::kLong && oracle.is_contiguous(), "oracle: contiguous int64 [n]");
  TORCH_CHECK(upd_status.scalar_type() == at::kInt && upd_status.numel() == n, "upd_status: int32 [n]");
  TORCH_CHECK(upd_per_inst > 0 && n <= values.size(0) * upd_per_inst, "upd_per_inst: rows b * U .. b * U + U - 1 "
              "belong to instance b");
  same_device(values, {{&rows, "rows"}, {&oracle, "oracle"}, {&upd_status, "upd_status"}});
  auto stream = c10::hip::getCurrentHIPStream(values.device().index()).stream();
  const int rc = svoc_commit_updates(rows.data_ptr(), oracle.data_ptr<int64_t>(), upd_status.data_ptr<int32_t>(),
                                     values.data_ptr(), values.stride(0), (int)values.size(1), (int)rows.size(1),
                                     (int)values.size(2), (int)upd_per_inst, n, (int)values.element_size(), stream);
  TORCH_CHECK(rc == 0, "svoc_commit_updates failed: ", rc);
}

void commit_updates_cpu(const at::Tensor& rows, const at::Tensor& oracle, const at::Tensor& upd_status, at::Tensor values,
                        int64_t upd_per_inst) {
  const int64_t n = oracle.numel(), D = rows.size(1);
  auto o = oracle.accessor<int64_t, 1>();
  auto st = upd_status.accessor<int32_t, 1>();
  for (int64_t u = 0; u < n; ++u)
    if (st[u] == ST_OK && o[u] >= 0 && o[u] < values.size(1))
      values[u / upd_per_inst][o[u]].narrow(0, 0, D).copy_(rows[u]);
}

}  // namespace

void register_extra_defs(torch::Library& m) {
  m.def(
      "apply_updates(Tensor(a!) values, Tensor(b!) enabled, Tensor(c!) n_active, Tensor(d!) touched, "
      "Tensor(e!) winner, Tensor inst, Tensor oracle, Tensor upd, bool constrained, Tensor(f!) upd_status, bool unique=False, "
      "Tensor(g!)? saved=None, Tensor(h!)? saved_en=None) -> ()");
  m.def(
      "restore_updates(Tensor(a!) values, Tensor(b!) enabled, Tensor(c!) n_active, Tensor inst, Tensor oracle, "
      "Tensor(d!) upd_status, Tensor saved, Tensor saved_en, Tensor status, Tensor active, int inactive_status=-1) -> ()");
  m.def("commit_updates(Tensor rows, Tensor oracle, Tensor upd_status, Tensor(a!) values, int upd_per_inst) -> ()");
  register_governance_defs(m);
  register_generator_defs(m);
  register_io_defs(m);
  register_bookkeeping_defs(m);
  register_encoder_defs(m);
}

void register_extra_cpu(torch::Library& m) {
  m.impl("apply_updates", &apply_updates_cpu);
  m.impl("restore_updates", &restore_updates_cpu);
  m.impl("commit_updates", &commit_updates_cpu);
  register_governance_cpu(m);
  register_generator_cpu(m);
  register_bookkeeping_cpu(m);
  register_encoder_cpu(m);
}

void register_extra_hip(torch::Library& m) {
  m.impl("apply_updates", &apply_updates_hip);
  m.impl("restore_updates", &restore_updates_hip);
  m.impl("commit_updates", &commit_updates_hip);
  register_governance_hip(m);
  register_generator_hip(m);
  register_bookkeeping_hip(m);
  register_encoder_hip(m);
}

}  // namespace svoc
