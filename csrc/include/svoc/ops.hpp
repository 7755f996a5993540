// Registration hooks for the ops defined outside torch_ops.cpp (updates, governance, generators).
#pragma once

#include <torch/library.h>

namespace svoc {
void register_extra_defs(torch::Library& m);
void register_extra_cpu(torch::Library& m);
void register_extra_hip(torch::Library& m);
}  // namespace svoc

namespace svoc {
void register_governance_defs(torch::Library& m);
void register_governance_cpu(torch::Library& m);
void register_governance_hip(torch::Library& m);
void register_generator_defs(torch::Library& m);
void register_generator_cpu(torch::Library& m);
void register_generator_hip(torch::Library& m);
void register_io_defs(torch::Library& m);
void register_io_cpu(torch::Library& m);
void register_bookkeeping_defs(torch::Library& m);
void register_bookkeeping_cpu(torch::Library& m);
void register_bookkeeping_hip(torch::Library& m);
void register_encoder_defs(torch::Library& m);
void register_encoder_cpu(torch::Library& m);
void register_encoder_hip(torch::Library& m);
}  // namespace svoc
