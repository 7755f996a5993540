// torch.ops.svoc.* registration.  CPU kernels = the golden C++ engines (reference_cpu.cpp);
// CUDA (= HIP on ROCm) kernels = the hand-written gfx950 kernels in csrc/kernels/*.hip.
// All ops write into caller-provided outputs ("out" semantics) so the Python engine owns the state
// tensors and can capture steady-state steps in HIP graphs.
#include <cstdlib>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <thread>

#include "../engine/engine.hpp"
#include "svoc/launch.hpp"
#include "svoc/ops.hpp"

namespace svoc {
namespace {

int cpu_threads() {
  static int n = [] {
    unsigned h = std::thread::hardware_concurrency();
    return (int)(h == 0 ? 1 : (h > 32 ? 32 : h));
  }();
  return n;
}

void check_out(const at::Tensor& t, at::ScalarType dt, std::initializer_list<int64_t> shape, const char* name,
               const at::Device& dev) {
  TORCH_CHECK(t.scalar_type() == dt, name, ": wrong dtype ", t.scalar_type());
  TORCH_CHECK(t.device() == dev, name, ": wrong device");
  TORCH_CHECK(t.is_contiguous(), name, ": must be contiguous");
  TORCH_CHECK(t.sizes().vec() == std::vector<int64_t>(shape), name, ": wrong shape ", t.sizes());
}

const uint8_t* active_ptr(const c10::optional<at::Tensor>& active, int64_t B, const at::Device& dev) {
  if (!active.has_value()) return nullptr;
  const auto& a = *active;
  TORCH_CHECK(a.scalar_type() == at::kByte || a.scalar_type() == at::kBool, "active: uint8/bool");
  TORCH_CHECK(a.numel() == B && a.is_contiguous() && a.device() == dev, "active: [B] contiguous");
  return (const uint8_t*)a.data_ptr();
}

// --------------------------------------------------------------------------------------- fast
void fast_round_checks(const at::Tensor& values, int64_t D, const at::Tensor& c1, const at::Tensor& cons,
                       const at::Tensor& skew, const at::Tensor& kurt, const at::Tensor& rel,
                       const at::Tensor& qr, const at::Tensor& reliable, const at::Tensor& status) {
  TORCH_CHECK(values.dim() == 3, "values: [B, N, ld]");
  TORCH_CHECK(values.stride(2) == 1 && values.stride(1) == values.size(2), "values: rows must be dense");
  const int64_t B = values.size(0), N = values.size(1);
  TORCH_CHECK(D >= 1 && D <= values.size(2), "D must be <= ld");
  const auto dev = values.device();
  check_out(c1, at::kFloat, {B, D}, "c1", dev);
  check_out(cons, at::kFloat, {B, D}, "consensus", dev);
  check_out(skew, at::kFloat, {B, D}, "skew", dev);
  check_out(kurt, at::kFloat, {B, D}, "kurt", dev);
  check_out(rel, at::kFloat, {B, 2}, "rel", dev);
  check_out(qr, at::kFloat, {B, N}, "qr", dev);
  check_out(reliable, at::kByte, {B, N}, "reliable", dev);
  check_out(status, at::kInt, {B}, "status", dev);
}

void fast_round_cpu(const at::Tensor& values, const c10::optional<at::Tensor>& active, int64_t D,
                    int64_t n_failing, bool constrained, double max_spread, at::Tensor c1, at::Tensor cons,
                    at::Tensor skew, at::Tensor kurt, at::Tensor rel, at::Tensor qr, at::Tensor reliable,
                    at::Tensor status, int64_t wave_hint, int64_t mode, int64_t rel_dim, bool legacy,
                    const c10::optional<at::Tensor>& work, const c10::optional<at::Tensor>& stats,
                    const c10::optional<at::Tensor>& upd_rows, const c10::optional<at::Tensor>& upd_oracle,
                    const c10::optional<at::Tensor>& upd_status, int64_t upd_per_inst,
                    const c10::optional<at::Tensor>& rst_saved, const c10::optional<at::Tensor>& rst_saved_en,
                    const c10::optional<at::Tensor>& rst_enabled, const c10::optional<at::Tensor>& rst_n_active) {
  (void)wave_hint;
  (void)work;
  (void)stats;   // (GPU pruned-network counter; the CPU twin runs full sorts)
  TORCH_CHECK(!upd_rows.has_value() || !upd_rows->defined(), "fused transactional streaming is a GPU path");
  TORCH_CHECK(!rst_saved.has_value() || !rst_saved->defined(), "in-kernel rollback is a GPU path");
  (void)rst_saved_en;
  (void)rst_enabled;
  (void)rst_n_active;
  (void)upd_oracle;
  (void)upd_status;
  (void)upd_per_inst;
  fast_round_checks(values, D, c1, cons, skew, kurt, rel, qr, reliable, status);
  const int64_t B = values.size(0), N = values.size(1), ld = values.size(2), is = values.stride(0);
  TORCH_CHECK(values.scalar_type() == at::kBFloat16 || values.scalar_type() == at::kFloat,
              "values: bf16 or fp32");
  FastBatch fb;
  fb.values = values.data_ptr();
  const bool bf = values.scalar_type() == at::kBFloat16;
  fb.load = [=](const void* base, int64_t i, float* dst) {
    for (int64_t r = 0; r < N; ++r)
      for (int64_t d = 0; d < D; ++d) {
        const int64_t o = i * is + r * ld + d;
        if (bf) {
          uint32_t w = (uint32_t)((const uint16_t*)base)[o] << 16;
          float f;
          std::memcpy(&f, &w, 4);
          dst[r * D + d] = f;
        } else {
          dst[r * D + d] = ((const float*)base)[o];
        }
      }
  };
  fb.active = active_ptr(active, B, values.device());
  fb.B = B; fb.N = N; fb.D = D;
  fb.n_failing = n_failing;
  fb.constrained = constrained;
  fb.max_spread = (float)max_spread;
  fb.c1 = c1.data_ptr<float>();
  fb.consensus = cons.data_ptr<float>();
  fb.rel = rel.data_ptr<float>();
  fb.skew = skew.data_ptr<float>();
  fb.kurt = kurt.data_ptr<float>();
  fb.reliable = reliable.data_ptr<uint8_t>();
  fb.qr = qr.data_ptr<float>();
  fb.status = status.data_ptr<int32_t>();
  fb.mode = (int)mode;
  fb.rel_dim = rel_dim;
  fb.legacy = legacy;
  fast_round_batch_cpu(fb, cpu_threads());
}

void fast_round_hip(const at::Tensor& values, const c10::optional<at::Tensor>& active, int64_t D,
                    int64_t n_failing, bool constrained, double max_spread, at::Tensor c1, at::Tensor cons,
                    at::Tensor skew, at::Tensor kurt, at::Tensor rel, at::Tensor qr, at::Tensor reliable,
                    at::Tensor status, int64_t wave_hint, int64_t mode, int64_t rel_dim, bool legacy,
                    const c10::optional<at::Tensor>& work, const c10::optional<at::Tensor>& stats,
                    const c10::optional<at::Tensor>& upd_rows, const c10::optional<at::Tensor>& upd_oracle,
                    const c10::optional<at::Tensor>& upd_status, int64_t upd_per_inst,
                    const c10::optional<at::Tensor>& rst_saved, const c10::optional<at::Tensor>& rst_saved_en,
                    const c10::optional<at::Tensor>& rst_enabled, const c10::optional<at::Tensor>& rst_n_active) {
  fast_round_checks(values, D, c1, cons, skew, kurt, rel, qr, reliable, status);
  TORCH_CHECK(values.scalar_type() == at::kBFloat16 || values.scalar_type() == at::kFloat,
              "GPU fast path stores values in bf16 or fp32");
  const bool f32 = values.scalar_type() == at::kFloat;
  const int64_t B = values.size(0), N = values.size(1), ld = values.size(2);
  if (f32) {
    // reference-resolution storage: the column-parallel fp32 kernel (consensus_fast_f32.hip)
    TORCH_CHECK(N >= 2 && N <= 4096, "GPU fp32 fast path supports 2 <= N <= 4096 oracles");
    TORCH_CHECK(B < (1ll << 31) && D < (1 << 30), "size limits");
    TORCH_CHECK(N * ld * 4 < (1ll << 31) && fast_work_words(D) * 4 < (1ll << 31),
                "instance too large for 32-bit buffer offsets (N * ld * 4 B and the workspace must stay < 2 GiB)");
  }
  if (!f32) {
    TORCH_CHECK(N >= 2 && N <= 4096, "GPU fast path supports 2 <= N <= 4096 oracles");
    TORCH_CHECK(ld % 8 == 0, "row stride (ld) must be a multiple of 8 bf16 (16 B)");
    TORCH_CHECK(((uintptr_t)values.data_ptr() & 15) == 0 && values.stride(0) % 8 == 0, "values must be 16-B aligned");
    TORCH_CHECK(B < (1ll << 31) && D < (1 << 30), "size limits");
    // the kernels address one instance with 32-bit buffer offsets (rows x ld x 2 B, workspace x 4 B)
    TORCH_CHECK(N * ld * 2 < (1ll << 31) && fast_work_words(D) * 4 < (1ll << 31),
                "instance too large for 32-bit buffer offsets (N * ld * 2 B and the workspace must stay < 2 GiB)");
  }
  FastParams p{};
  p.values = values.data_ptr();
  p.active = active_ptr(active, B, values.device());
  p.inst_stride = values.stride(0);
  p.B = (int)B; p.N = (int)N; p.D = (int)D; p.ld = (int)ld;
  p.n_failing = (int)n_failing;
  p.constrained = constrained ? 1 : 0;
  p.max_spread = (float)max_spread;
  p.wave_hint = (int)wave_hint;
  TORCH_CHECK(mode >= 0 && mode <= 2, "mode must be 0, 1 or 2");
  p.mode = (int)mode;
  p.rel_dim = (int)rel_dim;
  p.legacy = legacy ? 1 : 0;
  // a whole round stages c1 and commits it only where the round succeeded (a reverted round leaves
  // every output untouched); the D-sharded halves write it directly (mode 2 reads mode 1's c1)
  at::Tensor c1_stage;
  if (mode == 0) c1_stage = at::empty_like(c1);
  p.c1 = mode == 0 ? c1_stage.data_ptr<float>() : c1.data_ptr<float>();
  p.consensus = cons.data_ptr<float>();
  p.skew = skew.data_ptr<float>();
  p.kurt = kurt.data_ptr<float>();
  p.rel = rel.data_ptr<float>();
  p.qr = qr.data_ptr<float>();
  p.reliable = reliable.data_ptr<uint8_t>();
  p.status = status.data_ptr<int32_t>();
  // window-kernel workspace: the caller's (it must persist between mode 1 and mode 2 of a
  // D-sharded round), else a temporary one for a full round
  at::Tensor wtmp;
  const int64_t words = fast_work_words(D);
  if (work.has_value() && work->defined()) {
    TORCH_CHECK(work->is_contiguous() && work->element_size() == 4 && work->device() == values.device(),
                "work: contiguous 4-byte elements on the values' device");
    TORCH_CHECK(work->numel() >= fast_work_numel(B, D), "work: needs ", fast_work_numel(B, D),
                " elements (svoc.ops.fast_work_numel)");
    p.work = (uint32_t*)work->data_ptr();
  } else if (mode != 1 && (f32 || !(mode == 0 && wave_hint == 0 && N <= 16 && D <= 128))) {
    // a temporary one: every kernel but the small-instance one stages its pass-2 outputs there
    wtmp = at::empty({fast_work_numel(B, D)}, values.options().dtype(at::kInt));
    p.work = (uint32_t*)wtmp.data_ptr();
    p.work_fresh = 1;
  }
  {
    const char* wc = std::getenv("SVOC_WIN_CANCEL");   // tests / experiments: force or avoid the cleanup
    p.win_cancel = wc ? (float)std::atof(wc) : 64.f;
  }
  p.work_pairs = (int)fast_work_pairs(D);
  p.work_stride = words;
  auto stream = c10::hip::getCurrentHIPStream(values.device().index()).stream();
  // (mode 0: the kernel, or its dispatcher, commits the staged c1 into c1_out)
  p.c1_out = mode == 0 ? c1.data_ptr<float>() : nullptr;
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(stats->scalar_type() == at::kInt && stats->numel() >= 1 && stats->device() == values.device(),
                "stats: int32 [>= 1] on the values' device ([0] += pruned-network fallbacks)");
    p.net_fallbacks = (unsigned int*)stats->data_ptr();
  }
  for (const c10::optional<at::Tensor>* t : {&upd_rows, &upd_oracle, &upd_status, &rst_saved, &rst_saved_en,
                                              &rst_enabled, &rst_n_active})
    TORCH_CHECK(!t->has_value() || !(*t)->defined() || (*t)->device() == values.device(),
                "fast_round: every update / rollback tensor must be on the values' device");
  if (upd_rows.has_value() && upd_rows->defined()) {
    TORCH_CHECK(f32 && mode == 0 && constrained, "fused streaming: fp32 storage, whole constrained rounds");
    TORCH_CHECK(upd_per_inst > 0 && upd_oracle.has_value() && upd_status.has_value(), "fused streaming: "
                "upd_oracle, upd_status and upd_per_inst > 0 go with upd_rows");
    const int64_t n = B * upd_per_inst;
    TORCH_CHECK(upd_rows->scalar_type() == values.scalar_type() && upd_rows->is_contiguous() && upd_rows->dim() == 2 &&
                    upd_rows->size(0) == n && upd_rows->size(1) == D && upd_rows->device() == values.device(),
                "upd_rows: contiguous [B * U, D] in the values' dtype on the values' device");
    TORCH_CHECK(upd_oracle->scalar_type() == at::kLong && upd_oracle->is_contiguous() && upd_oracle->numel() == n,
                "upd_oracle: contiguous int64 [B * U]");
    TORCH_CHECK(upd_status->scalar_type() == at::kInt && upd_status->is_contiguous() && upd_status->numel() == n,
                "upd_status: contiguous int32 [B * U]");
    p.upd_rows = (const float*)upd_rows->data_ptr();   // (bf16 rows for the bf16 kernel)
    p.upd_oracle = upd_oracle->data_ptr<int64_t>();
    p.upd_status = upd_status->data_ptr<int32_t>();
    p.upd_per_inst = (int)upd_per_inst;
  }
  if (rst_saved.has_value() && rst_saved->defined()) {
    // in-kernel rollback of the generic transactional path (launch.hpp FastParams.rst_saved): the update
    // kernel's saved rows / flags and statuses for B * U instance-grouped updates; -3 from the dispatcher when
    // the kernel that runs cannot do it (the caller then launches svoc_restore_updates)
    TORCH_CHECK(!(upd_rows.has_value() && upd_rows->defined()), "rst_saved: not with the fused path's upd_rows");
    TORCH_CHECK(mode == 0 && upd_per_inst > 0 && upd_oracle.has_value() && upd_status.has_value() &&
                    rst_saved_en.has_value() && rst_enabled.has_value() && rst_n_active.has_value(),
                "rst_saved: mode 0, with upd_oracle, upd_status, upd_per_inst, rst_saved_en, rst_enabled, rst_n_active");
    // (checked before any launch: the rc == -3 fallback below needs it after the plain round has run)
    TORCH_CHECK(active.has_value() && active->defined(), "rst_saved: needs the round's active mask");
    const int64_t n = B * upd_per_inst;
    TORCH_CHECK(rst_saved->scalar_type() == values.scalar_type() && rst_saved->is_contiguous() &&
                    rst_saved->dim() == 2 && rst_saved->size(0) == n && rst_saved->size(1) == D,
                "rst_saved: contiguous [B * U, D] in the values' dtype");
    TORCH_CHECK(rst_saved_en->scalar_type() == at::kByte && rst_saved_en->is_contiguous() && rst_saved_en->numel() == n,
                "rst_saved_en: contiguous uint8 [B * U]");
    TORCH_CHECK(upd_oracle->scalar_type() == at::kLong && upd_oracle->is_contiguous() && upd_oracle->numel() == n,
                "upd_oracle: contiguous int64 [B * U]");
    TORCH_CHECK(upd_status->scalar_type() == at::kInt && upd_status->is_contiguous() && upd_status->numel() == n,
                "upd_status: contiguous int32 [B * U]");
    TORCH_CHECK(rst_enabled->scalar_type() == at::kByte && rst_enabled->is_contiguous() && rst_enabled->numel() == B * N,
                "rst_enabled: contiguous uint8 [B, N]");
    TORCH_CHECK(rst_n_active->scalar_type() == at::kInt && rst_n_active->is_contiguous() && rst_n_active->numel() == B,
                "rst_n_active: contiguous int32 [B]");
    p.rst_saved = rst_saved->data_ptr();
    p.rst_saved_en = rst_saved_en->data_ptr<uint8_t>();
    p.rst_oracle = upd_oracle->data_ptr<int64_t>();
    p.rst_status = upd_status->data_ptr<int32_t>();
    p.rst_enabled = rst_enabled->data_ptr<uint8_t>();
    p.rst_n_active = rst_n_active->data_ptr<int32_t>();
    p.rst_U = (int)upd_per_inst;
    const int rc = f32 ? svoc_fast_round_f32(&p, stream) : svoc_fast_round_bf16(&p, stream);
    TORCH_CHECK(rc == 0 || rc == -3, f32 ? "svoc_fast_round_f32" : "svoc_fast_round_bf16", " launch failed: ", rc);
    if (rc == -3) {
      // the kernel that runs this round cannot roll back (the dispatcher returns -3 before any launch): the
      // plain round, then the restore kernel over the same saved batch -- the updates are already stored, so
      // the round must run and the reverted instances must be rolled back here, not left to the caller
      p.rst_saved = nullptr;
      p.rst_saved_en = nullptr;
      p.rst_oracle = nullptr;
      p.rst_status = nullptr;
      p.rst_enabled = nullptr;
      p.rst_n_active = nullptr;
      p.rst_U = 0;
      const int rc2 = f32 ? svoc_fast_round_f32(&p, stream) : svoc_fast_round_bf16(&p, stream);
      TORCH_CHECK(rc2 == 0, f32 ? "svoc_fast_round_f32" : "svoc_fast_round_bf16", " launch failed: ", rc2);
      // instance-grouped batch: update u belongs to instance u / U
      at::Tensor inst = at::arange(n, upd_oracle->options()).div(upd_per_inst, "floor");
      RestoreParams r{};
      r.inactive_status = -1;
      r.values = values.data_ptr();
      r.enabled = rst_enabled->data_ptr<uint8_t>();
      r.n_active = rst_n_active->data_ptr<int32_t>();
      r.inst = inst.data_ptr<int64_t>();
      r.oracle = upd_oracle->data_ptr<int64_t>();
      r.upd_status = upd_status->data_ptr<int32_t>();
      r.saved = rst_saved->data_ptr();
      r.saved_en = rst_saved_en->data_ptr<uint8_t>();
      r.status = status.data_ptr<int32_t>();
      r.active = active->data_ptr<uint8_t>();
      r.inst_stride = values.stride(0);
      r.B = (int)B; r.N = (int)N; r.D = (int)D; r.ld = (int)ld; r.U = (int)n;
      r.elem_bytes = (int)values.element_size();
      const int rc3 = svoc_restore_updates(&r, stream);
      TORCH_CHECK(rc3 == 0, "svoc_restore_updates failed: ", rc3);
    }
    return;
  }
  const int rc = f32 ? svoc_fast_round_f32(&p, stream) : svoc_fast_round_bf16(&p, stream);
  TORCH_CHECK(rc == 0, f32 ? "svoc_fast_round_f32" : "svoc_fast_round_bf16", " launch failed: ", rc);
}

// -------------------------------------------------------------------------------------- exact
void exact_checks(const at::Tensor& values, const at::Tensor& c1, const at::Tensor& cons, const at::Tensor& skew,
                  const at::Tensor& kurt, const at::Tensor& rel, const at::Tensor& qr, const at::Tensor& reliable,
                  const at::Tensor& status) {
  TORCH_CHECK(values.dim() == 3 && (values.scalar_type() == at::kLong || values.scalar_type() == at::kInt) &&
                  values.is_contiguous(),
              "values: contiguous int64 or int32 [B, N, D] wsad");
  const int64_t B = values.size(0), N = values.size(1), D = values.size(2);
  const auto dev = values.device();
  check_out(c1, at::kLong, {B, D}, "c1", dev);
  check_out(cons, at::kLong, {B, D}, "consensus", dev);
  check_out(skew, at::kLong, {B, D}, "skew", dev);
  check_out(kurt, at::kLong, {B, D}, "kurt", dev);
  check_out(rel, at::kLong, {B, 2}, "rel", dev);
  check_out(qr, at::kLong, {B, N}, "qr", dev);
  check_out(reliable, at::kByte, {B, N}, "reliable", dev);
  check_out(status, at::kInt, {B}, "status", dev);
}

void exact_round_cpu(const at::Tensor& values, const c10::optional<at::Tensor>& active, int64_t n_failing,
                     bool constrained, int64_t max_spread, at::Tensor c1, at::Tensor cons, at::Tensor skew,
                     at::Tensor kurt, at::Tensor rel, at::Tensor qr, at::Tensor reliable, at::Tensor status,
                     bool legacy, int64_t mode, int64_t rel_dim, const c10::optional<at::Tensor>& stats) {
  (void)stats;   // (GPU kernel routing counters; the CPU engine is one path)
  exact_checks(values, c1, cons, skew, kurt, rel, qr, reliable, status);
  TORCH_CHECK(mode >= 0 && mode <= 2, "mode: 0 (whole round), 1 / 2 (D-sharded halves)");
  if (values.scalar_type() == at::kInt) {   // int32 wsad storage: the CPU engine works on int64
    exact_round_cpu(values.to(at::kLong), active, n_failing, constrained, max_spread, c1, cons, skew, kurt, rel, qr,
                    reliable, status, legacy, mode, rel_dim, stats);
    return;
  }
  ExactBatch eb{};
  eb.legacy = legacy;
  eb.mode = (int)mode;
  eb.rel_dim = rel_dim;
  eb.values = values.data_ptr<int64_t>();
  eb.B = values.size(0); eb.N = values.size(1); eb.D = values.size(2);
  eb.active = active_ptr(active, eb.B, values.device());
  eb.n_failing = n_failing;
  eb.constrained = constrained;
  eb.max_spread = max_spread;
  eb.consensus = cons.data_ptr<int64_t>();
  eb.rel = rel.data_ptr<int64_t>();
  eb.skew = skew.data_ptr<int64_t>();
  eb.kurt = kurt.data_ptr<int64_t>();
  eb.reliable = reliable.data_ptr<uint8_t>();
  eb.qr = qr.data_ptr<int64_t>();
  eb.c1 = c1.data_ptr<int64_t>();
  eb.status = status.data_ptr<int32_t>();
  exact_round_batch_cpu(eb, cpu_threads());
}

void exact_round_hip(const at::Tensor& values, const c10::optional<at::Tensor>& active, int64_t n_failing,
                     bool constrained, int64_t max_spread, at::Tensor c1, at::Tensor cons, at::Tensor skew,
                     at::Tensor kurt, at::Tensor rel, at::Tensor qr, at::Tensor reliable, at::Tensor status,
                     bool legacy, int64_t mode, int64_t rel_dim, const c10::optional<at::Tensor>& stats) {
  exact_checks(values, c1, cons, skew, kurt, rel, qr, reliable, status);
  TORCH_CHECK(mode >= 0 && mode <= 2, "mode: 0 (whole round), 1 / 2 (D-sharded halves)");
  ExactParams p{};
  p.legacy = legacy ? 1 : 0;
  p.mode = (int)mode;
  p.rel_dim = (int)rel_dim;
  p.values = values.data_ptr();
  p.val32 = values.scalar_type() == at::kInt ? 1 : 0;
  p.B = (int)values.size(0); p.N = (int)values.size(1); p.D = (int)values.size(2);
  TORCH_CHECK(p.N >= 1 && p.N <= kExactMaxN, "GPU exact path supports N <= ", kExactMaxN);
  p.active = active_ptr(active, p.B, values.device());
  p.n_failing = (int)n_failing;
  p.constrained = constrained ? 1 : 0;
  p.max_spread = max_spread;
  at::Tensor c1_stage;   // whole rounds: c1 staged, committed where the round succeeded (as fast_round_hip)
  if (mode == 0) c1_stage = at::empty_like(c1);
  p.c1 = mode == 0 ? c1_stage.data_ptr<int64_t>() : c1.data_ptr<int64_t>();
  p.consensus = cons.data_ptr<int64_t>();
  p.skew = skew.data_ptr<int64_t>();
  p.kurt = kurt.data_ptr<int64_t>();
  p.rel = rel.data_ptr<int64_t>();
  p.qr = qr.data_ptr<int64_t>();
  p.reliable = reliable.data_ptr<uint8_t>();
  p.status = status.data_ptr<int32_t>();
  if (stats.has_value() && stats->defined()) {
    // [0] += rounds the wide-column unconstrained kernel committed, [1] += rounds left to the i128 kernel
    TORCH_CHECK(stats->scalar_type() == at::kInt && stats->numel() >= 2 && stats->device() == values.device(),
                "stats: int32 [>= 2] on the values' device");
    p.xstats = (unsigned int*)stats->data_ptr();
  }
  at::Tensor work;
  if ((int64_t)p.D * kExactWsCols * 8 > 64 * 1024) {  // wide instances: per-column intermediates in HBM
    work = at::empty({(int64_t)p.B, kExactWsCols, (int64_t)p.D}, values.options().dtype(at::kLong));
    p.work = work.data_ptr<int64_t>();
  }
  // column-parallel kernel (consensus_wsad.hip), the i128 kernel for the instances it flags;
  // SVOC_EXACT_I128=1 forces the i128 kernel everywhere (tests, A/B)
  at::Tensor stage, fallback;
  const char* force = std::getenv("SVOC_EXACT_I128");
  if (p.N >= 4 && !(force && force[0] == '1')) {
    p.win_h = mode == 0 && constrained && !legacy ? exact_win_h(p.N, p.n_failing) : 0;
    // (c1, consensus, skewness, kurtosis; the window keys; unconstrained: the columns' base words)
    stage = at::empty({(int64_t)p.B, 4 + 2 * p.win_h + (constrained ? 0 : 2), (int64_t)p.D},
                      values.options().dtype(at::kInt));
    fallback = at::empty({(int64_t)p.B}, values.options().dtype(at::kByte));
    p.stage = stage.data_ptr<int32_t>();
    p.fallback = fallback.data_ptr<uint8_t>();
    const char* only = std::getenv("SVOC_EXACT_WSAD_ONLY");
    p.skip_fallback = only && only[0] == '1';
    const char* md = std::getenv("SVOC_EXACT_WSAD_MIN_D");   // tests: route small instances through it too
    p.wsad_min_d = md ? std::atoi(md) : 64;
  }
  auto stream = c10::hip::getCurrentHIPStream(values.device().index()).stream();
  const int rc = svoc_exact_round(&p, stream);
  TORCH_CHECK(rc == 0, "svoc_exact_round launch failed: ", rc);
  if (mode == 0) {
    const int rc2 = svoc_commit_rows(c1_stage.data_ptr(), c1.data_ptr(), p.status, p.active, p.B, 2 * (int64_t)p.D, stream);
    TORCH_CHECK(rc2 == 0, "svoc_commit_rows failed: ", rc2);
  }
}

}  // namespace
}  // namespace svoc

TORCH_LIBRARY(svoc, m) {
  m.def(
      "fast_round(Tensor values, Tensor? active, int D, int n_failing, bool constrained, float max_spread, "
      "Tensor(a!) c1, Tensor(b!) consensus, Tensor(c!) skew, Tensor(d!) kurt, Tensor(e!) rel, Tensor(f!) qr, "
      "Tensor(g!) reliable, Tensor(h!) status, int wave_hint=0, int mode=0, int rel_dim=0, bool legacy=False, "
      "Tensor? work=None, Tensor(i!)? stats=None, Tensor? upd_rows=None, Tensor? upd_oracle=None, "
      "Tensor(j!)? upd_status=None, int upd_per_inst=0, Tensor? rst_saved=None, Tensor? rst_saved_en=None, "
      "Tensor(k!)? rst_enabled=None, Tensor(l!)? rst_n_active=None) -> ()");
  m.def(
      "exact_round(Tensor values, Tensor? active, int n_failing, bool constrained, int max_spread, "
      "Tensor(a!) c1, Tensor(b!) consensus, Tensor(c!) skew, Tensor(d!) kurt, Tensor(e!) rel, Tensor(f!) qr, "
      "Tensor(g!) reliable, Tensor(h!) status, bool legacy=False, int mode=0, int rel_dim=0, "
      "Tensor(i!)? stats=None) -> ()");
  svoc::register_extra_defs(m);
}

TORCH_LIBRARY_IMPL(svoc, CPU, m) {
  m.impl("fast_round", &svoc::fast_round_cpu);
  m.impl("exact_round", &svoc::exact_round_cpu);
  svoc::register_extra_cpu(m);
}

TORCH_LIBRARY_IMPL(svoc, CUDA, m) {
  m.impl("fast_round", &svoc::fast_round_hip);
  m.impl("exact_round", &svoc::exact_round_hip);
  svoc::register_extra_hip(m);
}
