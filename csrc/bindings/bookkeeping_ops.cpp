// torch.ops.svoc.round_prologue / round_epilogue (CPU twin + HIP launch).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "svoc/bookkeeping.hpp"
#include "svoc/ops.hpp"

extern "C" int svoc_round_prologue(const svoc::RoundBook* r, hipStream_t stream);
extern "C" int svoc_round_epilogue(const svoc::RoundBook* r, hipStream_t stream);
extern "C" int svoc_bench_marker(int* flag, int code, hipStream_t stream);

namespace svoc {
namespace {

void check_u8(const at::Tensor& t, int64_t B, const char* n) {
  TORCH_CHECK((t.scalar_type() == at::kByte || t.scalar_type() == at::kBool) && t.numel() == B && t.is_contiguous(),
              n, ": uint8/bool [B] contiguous");
}

RoundBook make_prologue(const at::Tensor& n_active, at::Tensor& touched, int64_t N, bool only_touched,
                        at::Tensor& active) {
  const int64_t B = n_active.numel();
  TORCH_CHECK(n_active.scalar_type() == at::kInt && n_active.is_contiguous(), "n_active: int32 [B]");
  check_u8(touched, B, "touched");
  check_u8(active, B, "active");
  RoundBook r{};
  r.n_active = n_active.data_ptr<int32_t>();
  r.touched = (uint8_t*)touched.data_ptr();
  r.active = (uint8_t*)active.data_ptr();
  r.B = B;
  r.N = (int)N;
  r.only_touched = only_touched ? 1 : 0;
  return r;
}

RoundBook make_epilogue(at::Tensor& active, const at::Tensor& status, const at::Tensor& rel,
                        at::Tensor& consensus_active, at::Tensor& touched, const c10::optional<at::Tensor>& acc) {
  const int64_t B = active.numel();
  check_u8(active, B, "active");
  check_u8(consensus_active, B, "consensus_active");
  check_u8(touched, B, "touched");
  TORCH_CHECK(status.scalar_type() == at::kInt && status.numel() == B && status.is_contiguous(), "status: int32 [B]");
  TORCH_CHECK(rel.numel() == 2 * B && rel.is_contiguous() &&
              (rel.scalar_type() == at::kFloat || rel.scalar_type() == at::kLong), "rel: fp32/int64 [B, 2]");
  RoundBook r{};
  r.active = (uint8_t*)active.data_ptr();
  r.status = status.data_ptr<int32_t>();
  r.rel = rel.data_ptr();
  r.consensus_active = (uint8_t*)consensus_active.data_ptr();
  r.touched = (uint8_t*)touched.data_ptr();
  r.B = B;
  r.fast = rel.scalar_type() == at::kFloat ? 1 : 0;
  if (acc.has_value()) {
    TORCH_CHECK(acc->scalar_type() == at::kLong && acc->numel() == 4 && acc->is_contiguous(), "acc: int64 [4]");
    r.acc = (unsigned long long*)acc->data_ptr<int64_t>();
  }
  return r;
}

void prologue_cpu(const at::Tensor& n_active, at::Tensor touched, int64_t N, bool only_touched, at::Tensor active) {
  RoundBook r = make_prologue(n_active, touched, N, only_touched, active);
  for (int64_t b = 0; b < r.B; ++b) r.active[b] = book_active(r, b);
}

void epilogue_cpu(at::Tensor active, const at::Tensor& status, const at::Tensor& rel, at::Tensor consensus_active,
                  at::Tensor touched, const c10::optional<at::Tensor>& acc) {
  RoundBook r = make_epilogue(active, status, rel, consensus_active, touched, acc);
  unsigned long long v[4] = {0, 0, 0, 0};
  for (int64_t b = 0; b < r.B; ++b) {
    const bool act = r.active[b] != 0, ok = book_ok(r, b);
    if (ok) {
      r.consensus_active[b] = 1;
      v[0] += book_rel2_fx(r, b);
      v[1] += 1;
    }
    v[2] += act;
    v[3] += act && !ok;
    r.touched[b] = 0;
  }
  if (r.acc)
    for (int k = 0; k < 4; ++k) r.acc[k] += v[k];
}

void prologue_hip(const at::Tensor& n_active, at::Tensor touched, int64_t N, bool only_touched, at::Tensor active) {
  RoundBook r = make_prologue(n_active, touched, N, only_touched, active);
  const int rc = svoc_round_prologue(&r, c10::hip::getCurrentHIPStream(n_active.device().index()).stream());
  TORCH_CHECK(rc == 0, "svoc_round_prologue failed: ", rc);
}

void epilogue_hip(at::Tensor active, const at::Tensor& status, const at::Tensor& rel, at::Tensor consensus_active,
                  at::Tensor touched, const c10::optional<at::Tensor>& acc) {
  RoundBook r = make_epilogue(active, status, rel, consensus_active, touched, acc);
  const int rc = svoc_round_epilogue(&r, c10::hip::getCurrentHIPStream(active.device().index()).stream());
  TORCH_CHECK(rc == 0, "svoc_round_epilogue failed: ", rc);
}

void bench_marker_hip(at::Tensor flag, int64_t code) {
  TORCH_CHECK(flag.scalar_type() == at::kInt && flag.numel() >= 1, "flag: int32 [>= 1]");
  const int rc = svoc_bench_marker(flag.data_ptr<int32_t>(), (int)code,
                                   c10::hip::getCurrentHIPStream(flag.device().index()).stream());
  TORCH_CHECK(rc == 0, "svoc_bench_marker failed: ", rc);
}
void bench_marker_cpu(at::Tensor flag, int64_t code) { flag.fill_(code); }

}  // namespace

void register_bookkeeping_defs(torch::Library& m) {
  m.def("bench_marker(Tensor(a!) flag, int code) -> ()");
  m.def("round_prologue(Tensor n_active, Tensor(a!) touched, int N, bool only_touched, Tensor(b!) active) -> ()");
  m.def("round_epilogue(Tensor(a!) active, Tensor status, Tensor rel, Tensor(b!) consensus_active, "
        "Tensor(c!) touched, Tensor(d!)? acc) -> ()");
}
void register_bookkeeping_cpu(torch::Library& m) {
  m.impl("round_prologue", &prologue_cpu);
  m.impl("round_epilogue", &epilogue_cpu);
  m.impl("bench_marker", &bench_marker_cpu);
}
void register_bookkeeping_hip(torch::Library& m) {
  m.impl("round_prologue", &prologue_hip);
  m.impl("round_epilogue", &epilogue_hip);
  m.impl("bench_marker", &bench_marker_hip);
}

}  // namespace svoc
