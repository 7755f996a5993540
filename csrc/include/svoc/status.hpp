// Per-instance status codes. Mirror of svoc/status.py -- keep in sync.
// A non-OK status on an update means the reference transaction would have reverted
// (contract/src/contract.cairo:588-603); engines leave that instance's state untouched.
#pragma once

namespace svoc {

enum Status : int {
  ST_OK = 0,
  ST_NOT_ACTIVE = 1,
  ST_INTERVAL_INPUT = 2,
  ST_NOT_ORACLE = 3,
  ST_DIV_BY_ZERO = 4,
  ST_INDEX_OOB = 5,
  ST_RELIABILITY_INTERVAL = 6,
  ST_OVERFLOW = 7,
  ST_USIZE_UNDERFLOW = 8,
  ST_FELT_RANGE = 9,
  ST_REPLACEMENT_DISABLED = 16,
  ST_NOT_ADMIN = 17,
  ST_WRONG_ORACLE_INDEX = 18,
  ST_ALREADY_ORACLE = 19,
  ST_UNWRAP_NONE = 20,
  ST_WRONG_ADMIN_INDEX = 21,
  ST_ZERO_VARIANCE = 32,
  ST_TOO_FEW_RELIABLE = 33,
  ST_NON_FINITE = 34,  // unconstrained float update with NaN / inf
};

// D-sharded exact rounds (split mode 1): bound on |qr partial|, so the int64 all-reduce of up to 32
// shards' partials cannot wrap; a larger partial reverts the round with OVERFLOW.
constexpr long long kExactQrPartialMax = 1ll << 58;
// oracles per instance on the GPU exact path (the i128 kernel's 64 rows per lane); fast mode: 4096 too
constexpr int kExactMaxN = 4096;
// i128 exact kernel: per-column int64 intermediates (c1, consensus, mean, variance as i128, skew, kurt)
constexpr int kExactWsCols = 7;

}  // namespace svoc
