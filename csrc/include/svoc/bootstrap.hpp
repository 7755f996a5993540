// Stochastic oracle generator (client/oracle_scheduler.py:73-92), host+device, counter-based RNG so
// the CPU twin and the HIP kernel draw bit-identical streams.
//   slot j <  f : failing oracle, U(0,1)^D                      (oracle_scheduler.py:82-83)
//   slot j >= f : mean of `subset` distinct comments' vectors  (random.sample, :84-86)
//   then the slots are shuffled onto oracle indices            (np.random.shuffle, :89)
// Comment vectors: the 28 go_emotions sigmoid scores -> the 6 oracle labels -> normalised to sum 1
// (oracle_scheduler.py:20-40).
#pragma once

#include <stdint.h>

#include "wsad.hpp"  // SVOC_HD

namespace svoc {

SVOC_HD uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct Rng {
  uint64_t s;
  SVOC_HD explicit Rng(uint64_t key) : s(splitmix64(key)) {}
  SVOC_HD uint64_t next() { s = splitmix64(s); return s; }
  SVOC_HD float uniform() { return (float)(next() >> 40) * (1.0f / 16777216.0f); }  // [0, 1)
  SVOC_HD uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) % n); }
};

struct BootParams {
  const float* scores;     // [W, C, 28] go_emotions sigmoid scores
  const int32_t* label_idx;// [D] indices of the oracle labels
  float* out;              // [W, N, D] predictions (already shuffled onto oracle indices)
  int W, C, N, D, n_failing, subset;
  uint64_t seed;
};

// permutation of the N slots for window w (Fisher-Yates, slot j -> oracle perm[j])
SVOC_HD void boot_perm(const BootParams& p, int w, int* perm) {
  for (int j = 0; j < p.N; ++j) perm[j] = j;
  Rng r(p.seed ^ ((uint64_t)w * 0x100000001B3ull) ^ 0xABCDEFull);
  for (int j = p.N - 1; j > 0; --j) {
    const int k = (int)r.below((uint32_t)(j + 1));
    const int t = perm[j]; perm[j] = perm[k]; perm[k] = t;
  }
}

// prediction of slot j of window w into dst[D]
SVOC_HD void boot_slot(const BootParams& p, int w, int j, float* dst) {
  Rng r(p.seed ^ ((uint64_t)w << 20) ^ ((uint64_t)j << 4) ^ 0x5151ull);
  if (j < p.n_failing) {
    for (int d = 0; d < p.D; ++d) dst[d] = r.uniform();
    return;
  }
  int pick[64];
  const int C = p.C < 64 ? p.C : 64;
  for (int c = 0; c < C; ++c) pick[c] = c;
  const int k = p.subset < C ? p.subset : C;
  for (int d = 0; d < p.D; ++d) dst[d] = 0.f;
  for (int i = 0; i < k; ++i) {  // partial Fisher-Yates: k distinct comments
    const int t = i + (int)r.below((uint32_t)(C - i));
    const int c = pick[t]; pick[t] = pick[i]; pick[i] = c;
    const float* s = p.scores + ((int64_t)w * p.C + c) * 28;
    float tot = 0.f;
    for (int d = 0; d < p.D; ++d) tot += s[p.label_idx[d]];
    for (int d = 0; d < p.D; ++d) dst[d] += s[p.label_idx[d]] / tot;
  }
  for (int d = 0; d < p.D; ++d) dst[d] = dst[d] / (float)k;
}

}  // namespace svoc
