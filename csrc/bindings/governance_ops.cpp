#include "svoc/ops.hpp"
namespace svoc {
void register_governance_defs(torch::Library&) {}
void register_governance_cpu(torch::Library&) {}
void register_governance_hip(torch::Library&) {}
}  // namespace svoc
