// CPU consensus engines: the bit-exact wsad engine (golden for every GPU path) and the float
// "fast" engine that mirrors the HIP fast kernel's semantics.  Both are batched over independent
// instances and threaded over the batch.
//
// Exact semantics: contract/src/contract.cairo:365-503 (two passes), math.cairo (statistics),
// sort.cairo (tie rule), signed_decimal.cairo (fixed point).  The evaluation order matches
// svoc/reference.py so the first-error status codes agree.
#include "engine.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <thread>
#include <vector>

namespace svoc {

namespace {

template <class F>
void parallel_for(int64_t n, int threads, F&& fn) {
  if (threads <= 1 || n < 2) {
    for (int64_t i = 0; i < n; ++i) fn(i);
    return;
  }
  threads = (int)std::min<int64_t>(threads, n);
  std::vector<std::thread> pool;
  pool.reserve(threads);
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([&, t] {
      for (int64_t i = t; i < n; i += threads) fn(i);
    });
  }
  for (auto& th : pool) th.join();
}

i128 smooth_median_exact(std::vector<i128>& col, int& st) {  // math.cairo:113-126
  size_t n = col.size();
  if (n == 0) { fail(st, ST_USIZE_UNDERFLOW); return 0; }
  if (n == 1) { fail(st, ST_INDEX_OOB); return 0; }
  std::sort(col.begin(), col.end());
  size_t mid = n / 2;
  return idiv_pos64(add(col[mid - 1], col[mid], st), 2, st);
}

i128 average_exact(const std::vector<i128>& v, int& st) {  // math.cairo:240-254
  i128 acc = 0;
  for (i128 x : v) acc = add(acc, x, st);
  return idiv(acc, (i128)v.size(), st);
}

}  // namespace

int exact_round_one(const int64_t* X, int64_t N, int64_t D, int64_t n_failing, bool constrained,
                    int64_t max_spread, ExactOut& o, bool legacy, int mode, int64_t rel_dim) {
  int st = ST_OK;
  const int64_t rdim = legacy ? 1 : (rel_dim > 0 ? rel_dim : D);
  std::vector<i128> col(N);
  std::vector<i128> qr(N);
  if (mode == 2) {   // D-sharded: c1 (this shard) and the all-reduced qr come in
    for (int64_t i = 0; i < N; ++i) qr[i] = o.qr[i];
  } else {
    // ---- pass 1: essence (contract.cairo:455-459)
    for (int64_t d = 0; d < D && st == ST_OK; ++d) {
      for (int64_t i = 0; i < N; ++i) col[i] = X[i * D + d];
      o.c1[d] = (int64_t)smooth_median_exact(col, st);
    }
    if (st) return st;
    // quadratic risk (math.cairo:225-238)
    for (int64_t i = 0; i < N; ++i) {
      i128 acc = 0;
      for (int64_t d = 0; d < D; ++d) acc = add(acc, qdev(X[i * D + d], o.c1[d], st), st);
      qr[i] = acc;
    }
    if (mode == 1) {   // partials for the shard all-reduce (int64 sum)
      if (st) return st;
      for (int64_t i = 0; i < N; ++i) {
        if (qr[i] >= kExactQrPartialMax || qr[i] <= -kExactQrPartialMax) return ST_OVERFLOW;
        o.qr[i] = (int64_t)qr[i];
      }
      return ST_OK;
    }
  }
  i128 mean_qr = average_exact(qr, st);
  i128 rel1 = constrained ? constrained_reliability(mean_qr, rdim, st)
                          : unconstrained_reliability(wsqrt(mean_qr, st), max_spread, st);
  if (st) return st;
  if (!in_unit_interval(rel1)) return ST_RELIABILITY_INTERVAL;
  // IndexedMergeSort: (qr asc, idx desc) (sort.cairo:96-101)
  std::vector<int64_t> order(N);
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
    return qr[a] != qr[b] ? qr[a] < qr[b] : a > b;
  });
  if (n_failing > N) return ST_USIZE_UNDERFLOW;
  int64_t threshold = N - n_failing;
  for (int64_t r = 0; r < N; ++r) o.reliable[order[r]] = r < threshold ? 1 : 0;
  // ---- pass 2 (contract.cairo:476-500)
  std::vector<int64_t> rows;
  for (int64_t i = 0; i < N; ++i)
    if (o.reliable[i]) rows.push_back(i);
  const int64_t R = (int64_t)rows.size();
  col.resize(R);
  for (int64_t d = 0; d < D && st == ST_OK; ++d) {
    for (int64_t k = 0; k < R; ++k) col[k] = X[rows[k] * D + d];
    o.consensus[d] = (int64_t)(constrained ? smooth_median_exact(col, st) : average_exact(col, st));
  }
  if (st) return st;
  std::vector<i128> qr2(R);
  for (int64_t k = 0; k < R; ++k) qr2[k] = qr[rows[k]];
  i128 mean_qr2 = average_exact(qr2, st);
  i128 rel2 = constrained ? constrained_reliability(mean_qr2, rdim, st)
                          : unconstrained_reliability(wsqrt(mean_qr2, st), max_spread, st);
  if (st) return st;
  if (!in_unit_interval(rel2)) return ST_RELIABILITY_INTERVAL;
  if (legacy) {  // the obsolete contracts stop here: no skewness / kurtosis storage
    for (int64_t d = 0; d < D; ++d) o.skew[d] = o.kurt[d] = 0;
    for (int64_t i = 0; i < N; ++i) o.qr[i] = (int64_t)qr[i];
    o.rel1 = (int64_t)rel1;
    o.rel2 = (int64_t)rel2;
    return ST_OK;
  }
  // moments (math.cairo:208-222, 320-398) -- means, variances, skewness(all d), kurtosis(all d)
  std::vector<i128> means(D), vars(D);
  for (int64_t d = 0; d < D && st == ST_OK; ++d) {
    for (int64_t k = 0; k < R; ++k) col[k] = X[rows[k] * D + d];
    means[d] = average_exact(col, st);
  }
  for (int64_t d = 0; d < D && st == ST_OK; ++d) {
    std::vector<i128> q(R);
    for (int64_t k = 0; k < R; ++k) q[k] = qdev(X[rows[k] * D + d], means[d], st);
    vars[d] = average_exact(q, st);
  }
  for (int64_t d = 0; d < D && st == ST_OK; ++d) {
    i128 sd = wsqrt(vars[d], st);
    i128 acc = 0;
    for (int64_t k = 0; k < R && st == ST_OK; ++k) {
      i128 z = wdiv(sub(X[rows[k] * D + d], means[d], st), sd, st);
      acc = add(acc, wmul(wmul(z, z, st), z, st), st);
    }
    o.skew[d] = (int64_t)skew_from_sum(acc, R, st);
  }
  for (int64_t d = 0; d < D && st == ST_OK; ++d) {
    i128 sd = wsqrt(vars[d], st);
    i128 acc = 0;
    for (int64_t k = 0; k < R && st == ST_OK; ++k) {
      i128 z = wdiv(sub(X[rows[k] * D + d], means[d], st), sd, st);
      i128 z2 = wmul(z, z, st);
      acc = add(acc, wmul(z2, z2, st), st);
    }
    o.kurt[d] = (int64_t)kurt_from_sum(acc, R, st);
  }
  if (st) return st;
  for (int64_t i = 0; i < N; ++i) o.qr[i] = (int64_t)qr[i];
  o.rel1 = (int64_t)rel1;
  o.rel2 = (int64_t)rel2;
  return ST_OK;
}

void exact_round_batch_cpu(const ExactBatch& b, int threads) {
  parallel_for(b.B, threads, [&](int64_t i) {
    if (b.active && !b.active[i]) return;
    const int64_t N = b.N, D = b.D;
    std::vector<int64_t> c1(D), cons(D), sk(D), ku(D), qr(N);
    std::vector<uint8_t> rel(N);
    if (b.mode == 2) {
      if (b.status[i] != ST_OK) return;   // a shard's pass 1 failed: the round reverts everywhere
      std::memcpy(c1.data(), b.c1 + i * D, D * sizeof(int64_t));
      std::memcpy(qr.data(), b.qr + i * N, N * sizeof(int64_t));
    }
    ExactOut o{c1.data(), qr.data(), rel.data(), cons.data(), sk.data(), ku.data(), 0, 0};
    int st = exact_round_one(b.values + i * N * D, N, D, b.n_failing, b.constrained, b.max_spread, o, b.legacy,
                             b.mode, b.rel_dim);
    b.status[i] = st;
    if (st != ST_OK) return;  // revert: outputs untouched
    if (b.mode == 1) {
      std::memcpy(b.qr + i * N, qr.data(), N * sizeof(int64_t));
      if (b.c1) std::memcpy(b.c1 + i * D, c1.data(), D * sizeof(int64_t));
      return;
    }
    std::memcpy(b.consensus + i * D, cons.data(), D * sizeof(int64_t));
    std::memcpy(b.skew + i * D, sk.data(), D * sizeof(int64_t));
    std::memcpy(b.kurt + i * D, ku.data(), D * sizeof(int64_t));
    std::memcpy(b.qr + i * N, qr.data(), N * sizeof(int64_t));
    std::memcpy(b.reliable + i * N, rel.data(), N);
    if (b.c1) std::memcpy(b.c1 + i * D, c1.data(), D * sizeof(int64_t));
    b.rel[i * 2 + 0] = o.rel1;
    b.rel[i * 2 + 1] = o.rel2;
  });
}

// ------------------------------------------------------------------------------------------------
// Fast (float) engine: same algorithm in fp32 over bf16/fp32 storage; mirrors consensus_fast.hip.
// ------------------------------------------------------------------------------------------------

int fast_round_one(const float* X, int64_t N, int64_t D, int64_t n_failing, bool constrained,
                   float max_spread, FastOut& o, int mode, int64_t rel_dim, bool legacy) {
  if (n_failing > N) return ST_USIZE_UNDERFLOW;
  if (N < 2) return ST_INDEX_OOB;
  std::vector<float> col(N);
  const int64_t m = N / 2;
  const double rd = legacy ? 1.0 : (double)(rel_dim > 0 ? rel_dim : D);
  for (int64_t d = 0; d < D && mode != 2; ++d) {
    for (int64_t i = 0; i < N; ++i) col[i] = X[i * D + d];
    std::nth_element(col.begin(), col.begin() + m, col.end());
    float hi = col[m];
    float lo = *std::max_element(col.begin(), col.begin() + m);
    o.c1[d] = 0.5f * (lo + hi);
  }
  double sum_qr = 0.0;
  for (int64_t i = 0; i < N; ++i) {
    if (mode != 2) {
      float acc = 0.f;
      for (int64_t d = 0; d < D; ++d) {
        float y = X[i * D + d] - o.c1[d];
        acc = std::fma(y, y, acc);
      }
      o.qr[i] = acc;
    }
    sum_qr += o.qr[i];
  }
  if (mode == 1) return ST_OK;
  auto rel_of = [&](double mean_qr) -> float {
    return constrained ? (float)(1.0 - 2.0 * std::sqrt(mean_qr / rd))
                       : (float)(1.0 - std::min((double)max_spread, std::sqrt(mean_qr)) / (double)max_spread);
  };
  float rel1 = rel_of(sum_qr / (double)N);
  if (!(rel1 >= 0.f && rel1 <= 1.f)) return ST_RELIABILITY_INTERVAL;
  std::vector<int64_t> order(N);
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
    return o.qr[a] != o.qr[b] ? o.qr[a] < o.qr[b] : a > b;
  });
  const int64_t R = N - n_failing;
  for (int64_t r = 0; r < N; ++r) o.reliable[order[r]] = r < R ? 1 : 0;
  if (R < 2) return R == 0 ? ST_USIZE_UNDERFLOW : ST_INDEX_OOB;
  double sum_qr2 = 0.0;
  for (int64_t i = 0; i < N; ++i)
    if (o.reliable[i]) sum_qr2 += o.qr[i];
  float rel2 = rel_of(sum_qr2 / (double)R);
  if (!(rel2 >= 0.f && rel2 <= 1.f)) return ST_RELIABILITY_INTERVAL;
  if (R < 4 && !legacy) return ST_TOO_FEW_RELIABLE;
  col.resize(R);
  const int64_t m2 = R / 2;
  for (int64_t d = 0; d < D; ++d) {
    int64_t k = 0;
    for (int64_t i = 0; i < N; ++i)
      if (o.reliable[i]) col[k++] = X[i * D + d];
    double mean = 0.0;
    for (float v : col) mean += v;
    mean /= (double)R;
    double s2 = 0, s3 = 0, s4 = 0;
    for (float v : col) {
      double y = v - mean;
      s2 += y * y;
      s3 += y * y * y;
      s4 += y * y * y * y;
    }
    double var = s2 / (double)R;
    if (legacy) {
      o.skew[d] = o.kurt[d] = 0.f;
    } else {
      if (var <= 0.0) return ST_ZERO_VARIANCE;
      double sd = std::sqrt(var);
      double z3 = s3 / (sd * sd * sd), z4 = s4 / (var * var);
      double n = (double)R;
      o.skew[d] = (float)(z3 * n / ((n - 1) * (n - 2)));
      o.kurt[d] = (float)(((z4 * n * (n + 1)) / (n - 1) - 3.0 * (n - 1) * (n - 1)) / ((n - 2) * (n - 3)));
    }
    if (constrained) {
      std::nth_element(col.begin(), col.begin() + m2, col.end());
      float hi = col[m2];
      float lo = *std::max_element(col.begin(), col.begin() + m2);
      o.consensus[d] = 0.5f * (lo + hi);
    } else {
      o.consensus[d] = (float)mean;
    }
  }
  o.rel1 = rel1;
  o.rel2 = rel2;
  return ST_OK;
}

void fast_round_batch_cpu(const FastBatch& b, int threads) {
  parallel_for(b.B, threads, [&](int64_t i) {
    if (b.active && !b.active[i]) return;
    const int64_t N = b.N, D = b.D;
    std::vector<float> x(N * D), c1(D), cons(D), sk(D), ku(D), qr(N);
    std::vector<uint8_t> rel(N);
    b.load(b.values, i, x.data());
    if (b.mode == 2) std::memcpy(qr.data(), b.qr + i * N, N * sizeof(float));
    FastOut o{c1.data(), qr.data(), rel.data(), cons.data(), sk.data(), ku.data(), 0.f, 0.f};
    int st = fast_round_one(x.data(), N, D, b.n_failing, b.constrained, b.max_spread, o, b.mode, b.rel_dim, b.legacy);
    b.status[i] = st;
    // c1: written by pass 1 for the D-sharded second half; a whole round commits it only on success
    if (b.c1 && b.n_failing <= N && N >= 2 && (b.mode == 1 || (b.mode == 0 && st == ST_OK)))
      std::memcpy(b.c1 + i * D, c1.data(), D * sizeof(float));
    if (b.mode == 1) {
      if (st == ST_OK) std::memcpy(b.qr + i * N, qr.data(), N * sizeof(float));
      return;
    }
    if (st != ST_OK) return;
    std::memcpy(b.consensus + i * D, cons.data(), D * sizeof(float));
    std::memcpy(b.skew + i * D, sk.data(), D * sizeof(float));
    std::memcpy(b.kurt + i * D, ku.data(), D * sizeof(float));
    std::memcpy(b.qr + i * N, qr.data(), N * sizeof(float));
    std::memcpy(b.reliable + i * N, rel.data(), N);
    b.rel[i * 2 + 0] = o.rel1;
    b.rel[i * 2 + 1] = o.rel2;
  });
}

}  // namespace svoc
