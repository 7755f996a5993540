#include "svoc/ops.hpp"
namespace svoc {
void register_generator_defs(torch::Library&) {}
void register_generator_cpu(torch::Library&) {}
void register_generator_hip(torch::Library&) {}
}  // namespace svoc
