// Admin replacement voting (contract/src/contract.cairo:547-580 check_for_replacement, :661-717
// update_proposition, :721-738 vote_for_a_proposition), one action per instance, host+device.
//
// Device layout per instance b (A <= 64 admins, N oracles, addresses = 4 x int64 limbs):
//   admins[b][A][4], oracle_addr[b][N][4]
//   votes[b][r]  : uint64, bit e set <=> vote_matrix[emitter e][receiver r] (column-packed)
//   prop_tag[b][r] (0 None / 1 Some), prop_idx[b][r], prop_addr[b][r][4]
// Every action is a transaction: on a revert nothing is written (the vote bit included).
#pragma once

#include <stdint.h>

#include "status.hpp"
#include "wsad.hpp"  // SVOC_HD

namespace svoc {

struct GovState {
  const int64_t* admins;   // [B, A, 4]
  int64_t* oracle_addr;    // [B, N, 4]
  uint64_t* votes;         // [B, A]
  int8_t* prop_tag;        // [B, A]
  int32_t* prop_idx;       // [B, A]
  int64_t* prop_addr;      // [B, A, 4]
  int B, A, N;
  int enable;              // enable_oracle_replacement
  int majority;            // required_majority
};

struct GovAction {         // batched actions, one per instance in a launch
  const int64_t* inst;     // [K]
  const int64_t* caller;   // [K, 4]
  const int32_t* kind;     // [K] 0 = update_proposition, 1 = vote_for_a_proposition
  const int32_t* arg0;     // propose: tag (0 None / 1 Some);  vote: which_admin
  const int64_t* arg1;     // propose: old oracle index;        vote: support (0/1)
  const int64_t* addr;     // [K, 4] propose: new oracle address
  int32_t* status;         // [K]
  uint8_t* applied;        // [K] replacement applied by this vote
  int K;
  // ordered batches (any number of actions per instance): the action indices sorted stably by instance, so
  // each instance's actions form one run in submission order (nullptr: one action per instance)
  const int64_t* order;
};

SVOC_HD bool addr_eq(const int64_t* a, const int64_t* b) {
  return a[0] == b[0] && a[1] == b[1] && a[2] == b[2] && a[3] == b[3];
}

SVOC_HD int find_admin(const GovState& g, int64_t b, const int64_t* caller) {
  for (int i = 0; i < g.A; ++i)
    if (addr_eq(g.admins + (b * g.A + i) * 4, caller)) return i;
  return -1;
}

SVOC_HD int find_oracle(const GovState& g, int64_t b, const int64_t* addr) {
  for (int i = 0; i < g.N; ++i)
    if (addr_eq(g.oracle_addr + (b * g.N + i) * 4, addr)) return i;
  return -1;
}

SVOC_HD int gov_apply_one(const GovState& g, const GovAction& act, int k) {
  const int64_t b = act.inst[k];
  const int64_t* caller = act.caller + (int64_t)k * 4;
  if (act.applied) act.applied[k] = 0;
  if (b < 0 || b >= g.B) return ST_NOT_ADMIN;
  if (!g.enable) return ST_REPLACEMENT_DISABLED;  // "replacement disabled"
  const int me = find_admin(g, b, caller);
  if (me < 0) return ST_NOT_ADMIN;                // 'not an admin'
  uint64_t* votes = g.votes + b * g.A;
  if (act.kind[k] == 0) {  // ---------------------------------------- update_proposition
    if (act.arg0[k] == 0) {  // None: stored without clearing the votes (contract.cairo:671)
      g.prop_tag[b * g.A + me] = 0;
      return ST_OK;
    }
    const int64_t idx = act.arg1[k];
    if (!(idx >= 0 && idx < g.N)) return ST_WRONG_ORACLE_INDEX;
    const int64_t* na = act.addr + (int64_t)k * 4;
    if (find_oracle(g, b, na) >= 0) return ST_ALREADY_ORACLE;
    votes[me] = (uint64_t)1 << me;  // clear column `me`, then self-vote
    g.prop_tag[b * g.A + me] = 1;
    g.prop_idx[b * g.A + me] = (int32_t)idx;
    for (int j = 0; j < 4; ++j) g.prop_addr[(b * g.A + me) * 4 + j] = na[j];
    return ST_OK;
  }
  // ------------------------------------------------------------------ vote_for_a_proposition
  const int w = act.arg0[k];
  if (w < 0 || w >= g.A) return ST_WRONG_ADMIN_INDEX;
  const uint64_t bit = (uint64_t)1 << me;
  const uint64_t nv = act.arg1[k] ? (votes[w] | bit) : (votes[w] & ~bit);
  int n_votes = 0;
  for (uint64_t x = nv; x; x &= x - 1) ++n_votes;
  if (g.majority > n_votes) {
    votes[w] = nv;
    return ST_OK;
  }
  if (!g.prop_tag[b * g.A + w]) return ST_UNWRAP_NONE;  // unwrap() on None: revert (vote dropped)
  const int o = g.prop_idx[b * g.A + w];
  for (int j = 0; j < 4; ++j) g.oracle_addr[(b * g.N + o) * 4 + j] = g.prop_addr[(b * g.A + w) * 4 + j];
  for (int a = 0; a < g.A; ++a) {  // reinitialize propositions and the vote matrix
    votes[a] = 0;
    g.prop_tag[b * g.A + a] = 0;
  }
  if (act.applied) act.applied[k] = 1;
  return ST_OK;
}

}  // namespace svoc
