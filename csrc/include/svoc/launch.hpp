// Launch descriptors shared by the HIP kernels and the torch bindings (plain C structs, passed by
// value as kernel arguments).
#pragma once

#include <stdint.h>

namespace svoc {

struct FastParams {
  const void* values;       // [B, N, ld] bf16 (instance stride inst_stride elements)
  const uint8_t* active;    // [B] or null
  int64_t inst_stride;
  int B, N, D, ld;
  int n_failing;
  int constrained;
  float max_spread;
  int wave_hint;            // 0 = auto, 2/4/8 = waves per workgroup for N <= 64
  int mode;                 // 0 full round, 1 pass 1 only (qr partials + c1), 2 pass 2 from qr (D-sharding)
  int rel_dim;              // divisor of the constrained reliability (0 = D; global D when D-sharded)
  float* c1;                // [B, D]
  float* consensus;         // [B, D]
  float* skew;              // [B, D]
  float* kurt;              // [B, D]
  float* rel;               // [B, 2]
  float* qr;                // [B, N]
  uint8_t* reliable;        // [B, N]
  int32_t* status;          // [B]
  int legacy;               // obsolete-contract variant: reliability without /D, no moments (C30/C31)
  // workspace (layout: fast_work_words below); required by every kernel but the small-instance one
  uint32_t* work;
  int work_pairs;           // column pairs per instance in `work` (multiple of 256, >= ceil(D / 2))
  int64_t work_stride;      // u32 words per instance in `work`
  float win_cancel;         // window kernel: max all-row / reliable power-sum ratio trusted (else cleanup)
  int work_fresh;           // the workspace holds no pass-1 state (mode 2 must not use the window kernel)
  // mode 0: c1 above is the round's staging row; c1_out [B, D] receives it only where the round
  // succeeded (the window kernels write it in their commit phase, the dispatchers commit it for the
  // others with svoc_commit_rows).  Null: the caller commits (or mode 1 / 2: c1 is the output itself).
  float* c1_out;
  // optional counter: slab networks of the pruned window path (N = 256) that failed their exact check and
  // reran the full network (consensus_fast_winf.hip); null = not counted
  unsigned int* net_fallbacks;
  // Fused transactional streaming (fp32 window kernel, mode 0; null upd_rows = off): this launch's update
  // batch, `upd_per_inst` rows per instance in instance order ([B * U, D] fp32, pitch D, row b * U + k for
  // instance b; upd_oracle [B * U] their oracles, distinct per instance).  The round reads an updated oracle's
  // row from the batch instead of the state (the state is not written), validates it, and writes every
  // update's transaction status to upd_status: OK (commit: svoc_commit_updates copies the row), the round's
  // revert code, or INTERVAL_INPUT for a row outside [0, 1] (the round is recomputed without it).
  const float* upd_rows;
  const int64_t* upd_oracle;
  int32_t* upd_status;
  int upd_per_inst;
  // In-kernel rollback of the generic transactional path (bf16 window kernel, mode 0; null rst_saved = off):
  // updates b * rst_U .. b * rst_U + rst_U - 1 of this launch belong to instance b, and the update kernel
  // saved what they overwrote (rst_saved [B * U, D] in the values' dtype, rst_saved_en the old `enabled`
  // flags, kNotSaved where it wrote nothing).  A reverting workgroup copies the rows back, undoes first
  // commits (`enabled`, n_active) and gives every applied update the round's status -- what
  // svoc_restore_updates does, without its launch after the round.  (The state rows are written only then.)
  const void* rst_saved;
  const uint8_t* rst_saved_en;
  const int64_t* rst_oracle;
  int32_t* rst_status;
  uint8_t* rst_enabled;
  int32_t* rst_n_active;
  int rst_U;
};

// Workspace per instance of the LDS-free fast kernels, in u32 words (Dp = fast_work_pairs(D)).
// bf16 kernels (column pairs):
//   [17][2][Dp]  window keys (consensus_fast_win.hip; H = 17 upper bound)
//   [4][Dp]      float2 all-row power sums
//   [2 Dp]       cleanup column list
//   [3][2 Dp]    staged pass-2 outputs (consensus, skewness, kurtosis): a round writes them here and
//                copies them to the outputs only once its status is known to be OK, so a reverted
//                round leaves every output untouched (contract.cairo:588-603: a failed assert
//                reverts the whole transaction)
// fp32 window kernel (consensus_fast_winf.hip, one column per lane, Dc = 2 Dp columns):
//   [17][2][Dc] window keys, [4][Dc] power sums, [Dc] cleanup list, [3][Dc] staged outputs
//   (at word kWinfStageCols * Dc)
inline int64_t fast_work_pairs(int64_t D) { return ((D + 1) / 2 + 255) / 256 * 256; }
inline int64_t fast_work_stage_word(int64_t D) { return fast_work_pairs(D) * (2 * 17 + 8 + 2); }
constexpr int kWinfStageCols = 2 * 17 + 4 + 1;
inline int64_t fast_work_words(int64_t D) { return fast_work_pairs(D) * 2 * (kWinfStageCols + 3); }
inline int64_t fast_work_numel(int64_t B, int64_t D) { return B * fast_work_words(D); }

// Window half-width of the one-network kernels for (N, f): the smallest H in {5, 17} with a + 1 <= H
// and f - a + 1 <= H (a = N/2 - R/2: the pass-2 middle pair sits f - a ranks above / a ranks below the
// pass-1 one at most); 0 when neither fits.
inline int fast_win_h(int N, int f) {
  const int R = N - f, a = N / 2 - R / 2;
  if (a + 1 <= 5 && f - a + 1 <= 5) return 5;
  if (a + 1 <= 17 && f - a + 1 <= 17) return 17;
  return 0;
}

struct ExactParams {
  const void* values;       // [B, N, D] wsad, int64 (or int32 when val32)
  const uint8_t* active;    // [B] or null
  int B, N, D;
  int n_failing;
  int constrained;
  int64_t max_spread;
  int64_t* c1;              // [B, D]
  int64_t* consensus;       // [B, D]
  int64_t* skew;            // [B, D]
  int64_t* kurt;            // [B, D]
  int64_t* rel;             // [B, 2]
  int64_t* qr;              // [B, N]
  uint8_t* reliable;        // [B, N]
  int32_t* status;          // [B]
  int legacy;               // obsolete-contract variant (see FastParams)
  int64_t* work;            // [B, 6, D] workspace for wide instances (null: per-column data in LDS)
  int val32;                // values are int32 wsad
  // column-parallel kernel (consensus_wsad.hip): per-instance staging [B, 4, D] int32 and the [B]
  // fallback flags of the instances it hands to the i128 kernel (null: i128 kernel only)
  int32_t* stage;
  uint8_t* fallback;
  int skip_fallback;        // tests: leave the flagged instances alone (shows which rounds it took)
  int wsad_min_d;           // fewest columns the column-parallel kernel takes (default 64: one lane per column)
  // D-sharded rounds (svoc/parallel/dshard.py): 0 = whole round; 1 = pass 1 only -> c1 and the
  // instance's qr PARTIALS (this shard's columns) into c1 / qr, status; 2 = from c1 and the all-reduced
  // qr (inputs) on instances whose status is OK: rank mask, pass 2, moments, commit.  rel_dim: the
  // reliability's dimension (the GLOBAL D; 0 = D).
  int mode;
  int rel_dim;
  int win_h;                // the column kernel's window half-width (exact_win_h; the stage holds 4 + 2 win_h rows)
  // [2] or null: += rounds committed by the wide-column unconstrained kernel (consensus_wsadx.hip), += rounds
  // left to the i128 kernel
  unsigned int* xstats;
};

// Window half-width of the column-parallel exact kernel's one-network path (consensus_wsad.hip): the
// smallest of {5, 17} covering ranks R/2 - 1 .. R/2 + f of the full column, i.e. >= max(a + 1, f - a + 1)
// with a = N/2 - R/2; 0 = no window (two median networks).
inline int exact_win_h(int N, int f) {
  if (N < 4 || N > 256 || f < 0 || f > N - 2) return 0;   // (N > 256: the wide lane groups, two networks)
  const int R = N - f, a = N / 2 - R / 2;
  const int need = a + 1 > f - a + 1 ? a + 1 : f - a + 1;
  // (N <= 64 with 17: the one-lane-group kernel goes past 256 VGPRs, one wave per SIMD -- two networks win)
  return need <= 5 ? 5 : (need <= 17 && N > 64) ? 17 : 0;
}


}  // namespace svoc

extern "C" {
typedef struct ihipStream_t* hipStream_t;
int svoc_fast_round_bf16(const svoc::FastParams* p, hipStream_t stream);
int svoc_fast_round_f32(const svoc::FastParams* p, hipStream_t stream);   // values fp32 [B, N, ld]
int svoc_fast_round_f32_win(const svoc::FastParams* p, hipStream_t stream);
int svoc_exact_round(const svoc::ExactParams* p, hipStream_t stream);
}

namespace svoc {

// Batched oracle updates (update_prediction's storage half, contract.cairo:331-343 + the input
// interval check of :591-593), last-writer-wins per (instance, oracle) within one batch.
struct UpdateParams {
  void* values;             // [B, N, ld] (elem_bytes each)
  uint8_t* enabled;         // [B, N]
  int32_t* n_active;        // [B]
  uint8_t* touched;         // [B]
  int32_t* winner;          // [B, N] workspace, -1 when idle (restored by the launch)
  const int64_t* inst;      // [U]
  const int64_t* oracle;    // [U]
  const void* upd;          // [U, D] same dtype as values
  int32_t* upd_status;      // [U]
  int64_t inst_stride;      // elements
  int B, N, D, ld, U;
  int elem_bytes;           // 2 (bf16), 4 (fp32) or 8 (int64 wsad)
  int dtype;                // 0 bf16, 1 fp32, 2 int64 wsad, 3 int32 wsad
  int constrained;
  int unique;               // caller guarantees distinct (instance, oracle) pairs: one fused pass
  // transactional fast streaming (optional, null = off): every applied update first copies the row it
  // overwrites to saved[u] ([U, D], the values' dtype) and its old `enabled` flag to saved_en[u]
  // (kNotSaved when the update did not store), so a reverted round can restore the pre-batch state
  void* saved;
  uint8_t* saved_en;
};
constexpr uint8_t kNotSaved = 0xFF;

// Roll back the applied updates of the instances whose round ran and reverted (active[b] set, status[b]
// not OK): rows from saved, enabled from saved_en, n_active decremented for first commits, and the
// update's transaction status set to the round's code (contract.cairo:588-603: the whole tx reverts).
struct RestoreParams {
  void* values;
  uint8_t* enabled;
  int32_t* n_active;
  const int64_t* inst;
  const int64_t* oracle;
  int32_t* upd_status;
  const void* saved;
  const uint8_t* saved_en;
  const int32_t* status;    // [B] round status
  const uint8_t* active;    // [B] the round ran
  int64_t inst_stride;
  int B, N, D, ld, U, elem_bytes;
  // >= 0: an applied update whose instance did not run its round (not fully active) gets this status (the exact
  // engine's per-update transactions report NOT_ACTIVE, the update stays stored); -1: it keeps OK
  int inactive_status;
};

}  // namespace svoc

extern "C" int svoc_apply_updates(const svoc::UpdateParams* p, hipStream_t stream);
extern "C" int svoc_restore_updates(const svoc::RestoreParams* p, hipStream_t stream);
// Commit of a fused transactional step (FastParams.upd_rows): update u's row -> values[u / U, oracle[u]] where
// upd_status[u] is OK (set by the round kernel).  rows [Btot * U, D] (elem_bytes each), values [Btot, N, ld].
extern "C" int svoc_commit_updates(const void* rows, const int64_t* oracle, const int32_t* upd_status, void* values,
                                   int64_t inst_stride, int N, int D, int ld, int U, int64_t n_upd, int elem_bytes,
                                   hipStream_t stream);
// row b of src -> dst (words 4-byte words per row) where status[b] == OK and (active null or set)
extern "C" int svoc_commit_rows(const void* src, void* dst, const int32_t* status, const uint8_t* active, int64_t B,
                                int64_t words, hipStream_t stream);

