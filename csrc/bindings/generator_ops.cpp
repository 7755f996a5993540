// torch.ops.svoc.bootstrap_oracles: fused sentiment scores -> stochastic oracle predictions.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <vector>

#include "svoc/bootstrap.hpp"
#include "svoc/ops.hpp"

extern "C" int svoc_bootstrap(const svoc::BootParams* p, hipStream_t s);

namespace svoc {
namespace {

BootParams prep(const at::Tensor& scores, const at::Tensor& label_idx, at::Tensor& out, int64_t n_failing,
                int64_t subset, int64_t seed) {
  TORCH_CHECK(scores.dim() == 3 && scores.size(2) == 28 && scores.scalar_type() == at::kFloat &&
              scores.is_contiguous(), "scores: float32 [W, C, 28]");
  TORCH_CHECK(label_idx.scalar_type() == at::kInt && label_idx.is_contiguous(), "label_idx: int32 [D]");
  TORCH_CHECK(out.dim() == 3 && out.scalar_type() == at::kFloat && out.is_contiguous() &&
              out.size(0) == scores.size(0) && out.size(2) == label_idx.numel(), "out: float32 [W, N, D]");
  TORCH_CHECK(scores.size(1) <= 64 && out.size(1) <= 256 && out.size(2) <= 16, "C <= 64, N <= 256, D <= 16");
  BootParams p{};
  p.scores = scores.data_ptr<float>();
  p.label_idx = label_idx.data_ptr<int32_t>();
  p.out = out.data_ptr<float>();
  p.W = (int)scores.size(0); p.C = (int)scores.size(1); p.N = (int)out.size(1); p.D = (int)out.size(2);
  p.n_failing = (int)n_failing; p.subset = (int)subset; p.seed = (uint64_t)seed;
  return p;
}

void bootstrap_cpu(const at::Tensor& scores, const at::Tensor& label_idx, at::Tensor out, int64_t n_failing,
                   int64_t subset, int64_t seed) {
  BootParams p = prep(scores, label_idx, out, n_failing, subset, seed);
  std::vector<int> perm(p.N);
  for (int w = 0; w < p.W; ++w) {
    boot_perm(p, w, perm.data());
    for (int j = 0; j < p.N; ++j) boot_slot(p, w, j, p.out + ((int64_t)w * p.N + perm[j]) * p.D);
  }
}

void bootstrap_hip(const at::Tensor& scores, const at::Tensor& label_idx, at::Tensor out, int64_t n_failing,
                   int64_t subset, int64_t seed) {
  BootParams p = prep(scores, label_idx, out, n_failing, subset, seed);
  auto stream = c10::hip::getCurrentHIPStream(scores.device().index()).stream();
  const int rc = svoc_bootstrap(&p, stream);
  TORCH_CHECK(rc == 0, "svoc_bootstrap failed: ", rc);
}

}  // namespace

void register_generator_defs(torch::Library& m) {
  m.def("bootstrap_oracles(Tensor scores, Tensor label_idx, Tensor(a!) out, int n_failing, int subset, int seed) -> ()");
}
void register_generator_cpu(torch::Library& m) { m.impl("bootstrap_oracles", &bootstrap_cpu); }
void register_generator_hip(torch::Library& m) { m.impl("bootstrap_oracles", &bootstrap_hip); }

}  // namespace svoc
