// Round bookkeeping shared by the HIP kernels and the CPU twin: which instances run a round
// (fully active: n_active_oracles == n_oracles, contract.cairo:447-449; and touched by an update),
// and the commit of the round's outcome (consensus_active, contract.cairo:502) plus the step's
// health counters.  Counters are integers so the sums are deterministic on any launch geometry and
// across ranks: [0] sum of rel2 in units of 2^-32 (fast) or wsad (exact), [1] committed rounds,
// [2] processed rounds, [3] reverted rounds.
#pragma once

#include <stdint.h>

#include "status.hpp"
#include "wsad.hpp"  // SVOC_HD

namespace svoc {

struct RoundBook {
  const int32_t* n_active;  // [B]
  uint8_t* touched;         // [B]
  uint8_t* active;          // [B] out (prologue) / in (epilogue)
  const int32_t* status;    // [B]
  const void* rel;          // [B, 2] float (fast) or int64 (exact)
  uint8_t* consensus_active;// [B] (bool storage)
  unsigned long long* acc;  // [4] or null
  int64_t B;
  int N;
  int only_touched;
  int fast;
};

SVOC_HD uint8_t book_active(const RoundBook& r, int64_t b) {
  return (r.n_active[b] == r.N && (!r.only_touched || r.touched[b])) ? 1 : 0;
}

// committed = ran and succeeded; every other status (fast-mode ZERO_VARIANCE included) reverted the
// round, which leaves consensus_active as it was (contract.cairo:588-603: the whole tx reverts)
SVOC_HD bool book_ok(const RoundBook& r, int64_t b) {
  return r.active[b] && r.status[b] == ST_OK;
}

SVOC_HD unsigned long long book_rel2_fx(const RoundBook& r, int64_t b) {
  if (r.fast) {
    const float v = ((const float*)r.rel)[2 * b + 1];
    const float c = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);
    return (unsigned long long)((double)c * 4294967296.0 + 0.5);
  }
  const int64_t v = ((const int64_t*)r.rel)[2 * b + 1];
  return (unsigned long long)(v < 0 ? 0 : v);
}

}  // namespace svoc
