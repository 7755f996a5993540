// Host-side engine interfaces (CPU golden engines + shared batch descriptors).
#pragma once

#include <stdint.h>

#include <functional>

#include "svoc/status.hpp"
#include "svoc/wsad.hpp"

namespace svoc {

// ---- exact (wsad int64 storage) ---------------------------------------------------------------
struct ExactOut {
  int64_t* c1;
  int64_t* qr;
  uint8_t* reliable;
  int64_t* consensus;
  int64_t* skew;
  int64_t* kurt;
  int64_t rel1, rel2;
};

struct ExactBatch {
  const int64_t* values;  // [B, N, D]
  const uint8_t* active;  // [B] or null (all)
  int64_t B, N, D;
  int64_t n_failing;
  bool constrained;
  int64_t max_spread;
  int64_t* consensus;  // [B, D]
  int64_t* rel;        // [B, 2]
  int64_t* skew;       // [B, D]
  int64_t* kurt;       // [B, D]
  uint8_t* reliable;   // [B, N]
  int64_t* qr;         // [B, N]
  int64_t* c1;         // [B, D] or null
  int32_t* status;     // [B]
  bool legacy = false;  // obsolete contracts (contract_nd.cairo / contract_1d_constrained.cairo)
  int mode = 0;         // D-sharded split (launch.hpp ExactParams::mode): 1 = c1 + qr partials, 2 = rest
  int64_t rel_dim = 0;  // reliability dimension (global D), 0 = D
};

// legacy: reliability W - 2 sqrt(mean qr) without the /D (contract_nd.cairo:418,437) and no moments.
// mode 1 / 2: D-sharded split (ExactBatch::mode); mode 2 reads o.c1 and o.qr (the all-reduced qr).
int exact_round_one(const int64_t* X, int64_t N, int64_t D, int64_t n_failing, bool constrained,
                    int64_t max_spread, ExactOut& o, bool legacy = false, int mode = 0, int64_t rel_dim = 0);
void exact_round_batch_cpu(const ExactBatch& b, int threads);

// ---- fast (float compute, bf16/fp32 storage) ---------------------------------------------------
struct FastOut {
  float* c1;
  float* qr;
  uint8_t* reliable;
  float* consensus;
  float* skew;
  float* kurt;
  float rel1, rel2;
};

struct FastBatch {
  const void* values;
  // copies instance i ([N, D]) into dst as float
  std::function<void(const void*, int64_t, float*)> load;
  const uint8_t* active;
  int64_t B, N, D;
  int64_t n_failing;
  bool constrained;
  float max_spread;
  float* c1;  // diagnostic: written for every processed instance, whatever the status
  float* consensus;
  float* rel;
  float* skew;
  float* kurt;
  uint8_t* reliable;
  float* qr;
  int32_t* status;
  int mode = 0;
  int64_t rel_dim = 0;
  bool legacy = false;
};

// mode 0: full round; 1: pass 1 only (c1 + qr partials); 2: pass 2 from o.qr (already reduced).
// rel_dim: divisor of the constrained reliability (0 = D).
int fast_round_one(const float* X, int64_t N, int64_t D, int64_t n_failing, bool constrained,
                   float max_spread, FastOut& o, int mode = 0, int64_t rel_dim = 0, bool legacy = false);
void fast_round_batch_cpu(const FastBatch& b, int threads);

}  // namespace svoc
