// Rank mask of a round (contract.cairo:345-363; sort.cairo:96-101): sort the oracles by (qr asc, index desc),
// the first R = N - f are reliable.  One workgroup per instance, the N <= 256 per-oracle qr in LDS.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace svoc {

// For non-negative qr (every constrained round: sums of squares, never -0.0 or NaN) the float bits are
// order-preserving, so (qr asc, index desc) is the single 64-bit key  bits(qr) : ~index  and an oracle's rank is
// one 64-bit compare and one add per other oracle -- instead of two float compares, an index compare and the
// selects of the general form (~4x fewer VALU; the loop ran on one wave while the others waited at the barrier).
// key: LDS scratch of N uint64 (8-byte aligned).  relmask[w] = ballot of rows 64 w .. 64 w + 63 for every w the
// threads t = base + tid < NPAD cover (rows past N: 0), exactly as the general loop writes them.
template <int NT, int NPAD>
SVOC_DEV void rank_mask_nonneg(const float* qr, uint64_t* key, int N, int R, int tid, uint64_t* relmask) {
  for (int t = tid; t < N; t += NT) key[t] = ((uint64_t)__float_as_uint(qr[t]) << 32) | (uint32_t)~t;
  __syncthreads();
  for (int base = 0; base < NPAD; base += NT) {
    const int t = base + tid;
    bool rel = false;
    if (t < N) {
      const uint64_t my = key[t];
      int rank = 0;
      const int n2 = N & ~1;
      for (int j = 0; j < n2; j += 2) {
        rank += key[j] < my ? 1 : 0;
        rank += key[j + 1] < my ? 1 : 0;
      }
      if (N & 1) rank += key[N - 1] < my ? 1 : 0;
      rel = rank < R;
    }
    const uint64_t bal = __ballot(rel);
    if ((tid & 63) == 0 && (t >> 6) < 4) relmask[t >> 6] = bal;
  }
}

}  // namespace svoc
