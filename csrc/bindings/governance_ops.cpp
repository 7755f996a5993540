// torch.ops.svoc.governance: batched update_proposition / vote_for_a_proposition.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "svoc/governance.hpp"
#include "svoc/ops.hpp"

extern "C" int svoc_governance(const svoc::GovState* g, const svoc::GovAction* a, hipStream_t s);

namespace svoc {
namespace {

void prep(const at::Tensor& admins, at::Tensor& oracle_addr, at::Tensor& votes, at::Tensor& prop_tag,
          at::Tensor& prop_idx, at::Tensor& prop_addr, const at::Tensor& inst, const at::Tensor& caller,
          const at::Tensor& kind, const at::Tensor& arg0, const at::Tensor& arg1, const at::Tensor& addr,
          at::Tensor& status, at::Tensor& applied, bool enable, int64_t majority, GovState& g, GovAction& a) {
  auto chk = [](const at::Tensor& t, at::ScalarType dt, const char* n) {
    TORCH_CHECK(t.scalar_type() == dt && t.is_contiguous(), n, ": wrong dtype or not contiguous");
  };
  chk(admins, at::kLong, "admins"); chk(oracle_addr, at::kLong, "oracle_addr");
  chk(votes, at::kLong, "votes"); chk(prop_tag, at::kChar, "prop_tag"); chk(prop_idx, at::kInt, "prop_idx");
  chk(prop_addr, at::kLong, "prop_addr"); chk(inst, at::kLong, "inst"); chk(caller, at::kLong, "caller");
  chk(kind, at::kInt, "kind"); chk(arg0, at::kInt, "arg0"); chk(arg1, at::kLong, "arg1"); chk(addr, at::kLong, "addr");
  chk(status, at::kInt, "status"); chk(applied, at::kByte, "applied");
  TORCH_CHECK(admins.dim() == 3 && admins.size(2) == 4, "admins: [B, A, 4]");
  TORCH_CHECK(oracle_addr.dim() == 3 && oracle_addr.size(2) == 4, "oracle_addr: [B, N, 4]");
  g.B = (int)admins.size(0); g.A = (int)admins.size(1); g.N = (int)oracle_addr.size(1);
  TORCH_CHECK(g.A <= 64, "at most 64 admins (bit-packed vote columns)");
  TORCH_CHECK(votes.numel() == (int64_t)g.B * g.A && prop_tag.numel() == votes.numel() &&
              prop_idx.numel() == votes.numel() && prop_addr.numel() == votes.numel() * 4, "proposition shapes");
  const int64_t K = inst.numel();
  TORCH_CHECK(caller.numel() == K * 4 && kind.numel() == K && arg0.numel() == K && arg1.numel() == K &&
              addr.numel() == K * 4 && status.numel() == K && applied.numel() == K, "action shapes");
  g.admins = admins.data_ptr<int64_t>();
  g.oracle_addr = oracle_addr.data_ptr<int64_t>();
  g.votes = (uint64_t*)votes.data_ptr<int64_t>();
  g.prop_tag = prop_tag.data_ptr<int8_t>();
  g.prop_idx = prop_idx.data_ptr<int32_t>();
  g.prop_addr = prop_addr.data_ptr<int64_t>();
  g.enable = enable ? 1 : 0;
  g.majority = (int)majority;
  a.inst = inst.data_ptr<int64_t>(); a.caller = caller.data_ptr<int64_t>(); a.kind = kind.data_ptr<int32_t>();
  a.arg0 = arg0.data_ptr<int32_t>(); a.arg1 = arg1.data_ptr<int64_t>(); a.addr = addr.data_ptr<int64_t>();
  a.status = status.data_ptr<int32_t>(); a.applied = applied.data_ptr<uint8_t>(); a.K = (int)K;
}

void governance_cpu(const at::Tensor& admins, at::Tensor oracle_addr, at::Tensor votes, at::Tensor prop_tag,
                    at::Tensor prop_idx, at::Tensor prop_addr, const at::Tensor& inst, const at::Tensor& caller,
                    const at::Tensor& kind, const at::Tensor& arg0, const at::Tensor& arg1, const at::Tensor& addr,
                    bool enable, int64_t majority, at::Tensor status, at::Tensor applied) {
  GovState g{}; GovAction a{};
  prep(admins, oracle_addr, votes, prop_tag, prop_idx, prop_addr, inst, caller, kind, arg0, arg1, addr, status,
       applied, enable, majority, g, a);
  for (int k = 0; k < a.K; ++k) a.status[k] = gov_apply_one(g, a, k);  // in order
}

void governance_hip(const at::Tensor& admins, at::Tensor oracle_addr, at::Tensor votes, at::Tensor prop_tag,
                    at::Tensor prop_idx, at::Tensor prop_addr, const at::Tensor& inst, const at::Tensor& caller,
                    const at::Tensor& kind, const at::Tensor& arg0, const at::Tensor& arg1, const at::Tensor& addr,
                    bool enable, int64_t majority, at::Tensor status, at::Tensor applied) {
  GovState g{}; GovAction a{};
  prep(admins, oracle_addr, votes, prop_tag, prop_idx, prop_addr, inst, caller, kind, arg0, arg1, addr, status,
       applied, enable, majority, g, a);
  auto stream = c10::hip::getCurrentHIPStream(admins.device().index()).stream();
  const int rc = svoc_governance(&g, &a, stream);
  TORCH_CHECK(rc == 0, "svoc_governance failed: ", rc);
}

// Ordered batches: any number of actions per instance, applied in submission order per instance.  `order`:
// the action indices sorted stably by instance (Governance.submit_batch sorts on the device).
void governance_seq_cpu(const at::Tensor& admins, at::Tensor oracle_addr, at::Tensor votes, at::Tensor prop_tag,
                        at::Tensor prop_idx, at::Tensor prop_addr, const at::Tensor& inst, const at::Tensor& caller,
                        const at::Tensor& kind, const at::Tensor& arg0, const at::Tensor& arg1, const at::Tensor& addr,
                        bool enable, int64_t majority, const at::Tensor& order, at::Tensor status, at::Tensor applied) {
  (void)order;   // the CPU applies the whole list in order (instances are independent)
  governance_cpu(admins, oracle_addr, votes, prop_tag, prop_idx, prop_addr, inst, caller, kind, arg0, arg1, addr,
                 enable, majority, status, applied);
}

void governance_seq_hip(const at::Tensor& admins, at::Tensor oracle_addr, at::Tensor votes, at::Tensor prop_tag,
                        at::Tensor prop_idx, at::Tensor prop_addr, const at::Tensor& inst, const at::Tensor& caller,
                        const at::Tensor& kind, const at::Tensor& arg0, const at::Tensor& arg1, const at::Tensor& addr,
                        bool enable, int64_t majority, const at::Tensor& order, at::Tensor status, at::Tensor applied) {
  GovState g{}; GovAction a{};
  prep(admins, oracle_addr, votes, prop_tag, prop_idx, prop_addr, inst, caller, kind, arg0, arg1, addr, status,
       applied, enable, majority, g, a);
  TORCH_CHECK(order.scalar_type() == at::kLong && order.is_contiguous() && order.numel() == inst.numel(),
              "order: contiguous int64 [K]");
  a.order = order.data_ptr<int64_t>();
  auto stream = c10::hip::getCurrentHIPStream(admins.device().index()).stream();
  const int rc = svoc_governance(&g, &a, stream);
  TORCH_CHECK(rc == 0, "svoc_governance failed: ", rc);
}

}  // namespace

void register_governance_defs(torch::Library& m) {
  m.def(
      "governance(Tensor admins, Tensor(a!) oracle_addr, Tensor(b!) votes, Tensor(c!) prop_tag, "
      "Tensor(d!) prop_idx, Tensor(e!) prop_addr, Tensor inst, Tensor caller, Tensor kind, Tensor arg0, "
      "Tensor arg1, Tensor addr, bool enable, int majority, Tensor(f!) status, Tensor(g!) applied) -> ()");
  m.def(
      "governance_seq(Tensor admins, Tensor(a!) oracle_addr, Tensor(b!) votes, Tensor(c!) prop_tag, "
      "Tensor(d!) prop_idx, Tensor(e!) prop_addr, Tensor inst, Tensor caller, Tensor kind, Tensor arg0, "
      "Tensor arg1, Tensor addr, bool enable, int majority, Tensor order, Tensor(f!) status, "
      "Tensor(g!) applied) -> ()");
}
void register_governance_cpu(torch::Library& m) {
  m.impl("governance", &governance_cpu);
  m.impl("governance_seq", &governance_seq_cpu);
}
void register_governance_hip(torch::Library& m) {
  m.impl("governance", &governance_hip);
  m.impl("governance_seq", &governance_seq_hip);
}

}  // namespace svoc
