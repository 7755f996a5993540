// Host self-test of the native CPU runtime, built with sanitizers by tools/sanitize_host.sh
// (AddressSanitizer + UBSan, and ThreadSanitizer for the threaded batch loops).  GPU sanitizers are
// not available on the target pool, so the host code paths shared with the kernels (wsad.hpp,
// governance.hpp) and the host-only engines / checkpoint IO are exercised here instead.
//
// Checks: the reference fixture's golden outputs (contract/tests/test_contract.cairo:
// 150-158), threaded batch == sequential single-instance results (exact and fast engines),
// governance state machine invariants, and a .svoc save/load round trip with CRC verification.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "engine.hpp"
#include "svoc/governance.hpp"
#include "svoc/wsad_fast.hpp"
#include "svoc_io.hpp"

using namespace svoc;

static int failures = 0;
#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                      \
    }                                                                  \
  } while (0)

static void golden_fixture() {
  const int64_t X[7][2] = {{492954, 334814}, {437692, 410445}, {967794, 564219}, {431029, 387225},
                           {487609, 337990}, {284178, 485072}, {990059, 558600}};
  int64_t c1[2], qr[7], cons[2], sk[2], ku[2];
  uint8_t rel[7];
  ExactOut o{c1, qr, rel, cons, sk, ku, 0, 0};
  const int st = exact_round_one(&X[0][0], 7, 2, 2, true, 0, o);
  CHECK(st == ST_OK);
  CHECK(c1[0] == 462650 && c1[1] == 398835);
  CHECK(cons[0] == 434360 && cons[1] == 362607);
  CHECK(o.rel1 == 573480 && o.rel2 == 857846);
  CHECK(sk[0] == -2294596 && sk[1] == 1263429);
  CHECK(ku[0] == 9083020 && ku[1] == 4989576);
  const uint8_t exp_rel[7] = {1, 1, 0, 1, 1, 1, 0};
  CHECK(std::memcmp(rel, exp_rel, 7) == 0);
  // documented panics become status codes: sqrt(1 ulp) divides by zero (math.cairo:277)
  int s2 = ST_OK;
  (void)wsqrt(1, s2);
  CHECK(s2 == ST_DIV_BY_ZERO);
}

static void batch_vs_single(int threads) {
  std::mt19937_64 rng(7);
  const int64_t B = 64, N = 33, D = 5;
  std::vector<int64_t> X(B * N * D);
  for (auto& v : X) v = 300000 + (int64_t)(rng() % 400000);
  std::vector<int64_t> cons(B * D), sk(B * D), ku(B * D), qr(B * N), c1(B * D), rel(B * 2);
  std::vector<uint8_t> reliable(B * N);
  std::vector<int32_t> status(B);
  ExactBatch eb{};
  eb.values = X.data(); eb.B = B; eb.N = N; eb.D = D; eb.n_failing = 4; eb.constrained = true;
  eb.consensus = cons.data(); eb.rel = rel.data(); eb.skew = sk.data(); eb.kurt = ku.data();
  eb.reliable = reliable.data(); eb.qr = qr.data(); eb.c1 = c1.data(); eb.status = status.data();
  exact_round_batch_cpu(eb, threads);
  for (int64_t b = 0; b < B; ++b) {
    std::vector<int64_t> c(D), q(N), cs(D), s(D), k(D);
    std::vector<uint8_t> r(N);
    ExactOut o{c.data(), q.data(), r.data(), cs.data(), s.data(), k.data(), 0, 0};
    const int st = exact_round_one(X.data() + b * N * D, N, D, 4, true, 0, o);
    CHECK(st == status[b]);
    if (st == ST_OK) {
      CHECK(std::memcmp(cs.data(), cons.data() + b * D, D * 8) == 0);
      CHECK(std::memcmp(k.data(), ku.data() + b * D, D * 8) == 0);
      CHECK(o.rel2 == rel[b * 2 + 1]);
    }
  }
  // fast engine, threaded
  std::vector<float> xf(B * N * D);
  for (size_t i = 0; i < xf.size(); ++i) xf[i] = (float)X[i] * 1e-6f;
  std::vector<float> f_c1(B * D), f_cons(B * D), f_rel(B * 2), f_sk(B * D), f_ku(B * D), f_qr(B * N);
  std::vector<uint8_t> f_reliable(B * N);
  std::vector<int32_t> f_status(B);
  FastBatch fb;
  fb.values = xf.data();
  fb.load = [&](const void* base, int64_t i, float* dst) {
    std::memcpy(dst, (const float*)base + i * N * D, N * D * sizeof(float));
  };
  fb.active = nullptr; fb.B = B; fb.N = N; fb.D = D; fb.n_failing = 4; fb.constrained = true;
  fb.max_spread = 1.f; fb.c1 = f_c1.data(); fb.consensus = f_cons.data(); fb.rel = f_rel.data();
  fb.skew = f_sk.data(); fb.kurt = f_ku.data(); fb.reliable = f_reliable.data(); fb.qr = f_qr.data();
  fb.status = f_status.data();
  fast_round_batch_cpu(fb, threads);
  for (int64_t b = 0; b < B; ++b) CHECK(f_status[b] == ST_OK || f_status[b] == ST_ZERO_VARIANCE);
}

static void governance_flow() {
  const int A = 3, N = 4;
  int64_t admins[A * 4] = {0}, oracles[N * 4] = {0}, prop_addr[A * 4] = {0};
  uint64_t votes[A] = {0};
  int8_t prop_tag[A] = {0};
  int32_t prop_idx[A] = {0};
  for (int a = 0; a < A; ++a) admins[a * 4] = 100 + a;
  for (int o = 0; o < N; ++o) oracles[o * 4] = 500 + o;
  GovState g{};
  g.admins = admins; g.oracle_addr = oracles; g.votes = votes; g.prop_tag = prop_tag;
  g.prop_idx = prop_idx; g.prop_addr = prop_addr; g.B = 1; g.A = A; g.N = N; g.enable = 1; g.majority = 2;
  int64_t inst[1] = {0}, caller[4] = {100, 0, 0, 0}, a1[1] = {2}, addr[4] = {999, 0, 0, 0};
  int32_t kind[1] = {0}, a0[1] = {1}, st[1] = {0};
  uint8_t applied[1] = {0};
  GovAction act{};
  act.inst = inst; act.caller = caller; act.kind = kind; act.arg0 = a0; act.arg1 = a1; act.addr = addr;
  act.status = st; act.applied = applied; act.K = 1;
  CHECK(gov_apply_one(g, act, 0) == ST_OK);  // admin 0 proposes oracle 2 -> 999 (self-vote)
  caller[0] = 101; kind[0] = 1; a0[0] = 0; a1[0] = 1;
  CHECK(gov_apply_one(g, act, 0) == ST_OK);  // admin 1 supports: majority 2 reached
  CHECK(applied[0] == 1 && oracles[2 * 4] == 999);
  caller[0] = 77;
  CHECK(gov_apply_one(g, act, 0) == ST_NOT_ADMIN);
}

static void io_roundtrip() {
  std::vector<io::Section> secs(2);
  secs[0].name = "values"; secs[0].dtype = io::DType::I64; secs[0].shape = {2, 3};
  for (int i = 0; i < 6; ++i) {
    int64_t v = (int64_t)i * -123456789;
    const uint8_t* p = (const uint8_t*)&v;
    secs[0].bytes.insert(secs[0].bytes.end(), p, p + 8);
  }
  int64_t w[2] = {-5, 1234567};
  secs[1].name = "wide"; secs[1].dtype = io::DType::I128; secs[1].shape = {2};
  secs[1].bytes = io::i64_to_i128(w, 2);
  const std::string path = std::string(std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp") + "/svoc_selftest.svoc";
  io::save(path, "{\"selftest\": true}", secs);
  std::vector<io::Section> back;
  const std::string meta = io::load(path, back);
  CHECK(meta.find("selftest") != std::string::npos);
  CHECK(back.size() == 2 && back[0].bytes == secs[0].bytes && back[1].bytes == secs[1].bytes);
  int64_t w2[2];
  io::i128_to_i64(back[1].bytes.data(), 2, w2);
  CHECK(w2[0] == -5 && w2[1] == 1234567);
  std::remove(path.c_str());
}

// The fp64 exact fast paths (wsad_fast.hpp, used by the column-parallel exact kernel) against the
// i128 routines of wsad.hpp, on random and boundary operands inside their stated bounds.
static void wsad_fast_paths() {
  std::mt19937_64 rng(12345);
  auto uni = [&](int64_t lo, int64_t hi) { return lo + (int64_t)(rng() % (uint64_t)(hi - lo + 1)); };
  int bad = 0;
  for (int it = 0; it < 2000000 && bad < 10; ++it) {
    int st = ST_OK;
    // quadratic deviation of constrained values
    const int64_t a = uni(0, 1000000), b = uni(0, 1000000);
    if ((int64_t)qdev_d((double)a, (double)b) != (int64_t)qdev(a, b, st)) ++bad;
    // wsad_mul of z-score sized operands, both signs
    const int64_t z = uni(-(1 << 25), 1 << 25), y = uni(-(1 << 24), 1 << 24);
    if ((int64_t)wmul_d((double)z, (double)y) != (int64_t)wmul(z, y, st)) ++bad;
    // wsad_div by a standard deviation
    const int64_t num = uni(-1000000, 1000000), sd = uni(1, 2000000);
    if ((int64_t)wdiv_d((double)num, (double)sd, recip_lo((double)sd)) != (int64_t)wdiv(num, sd, st)) ++bad;
    // truncating division (means, variances): dividends below 2^51, quotients below 2^47 (the stated bound)
    const int64_t d = it % 4 == 0 ? uni(1, 16) : uni(16, 1 << 30);
    const int64_t s = d < 16 ? uni(-(1ll << 46), 1ll << 46) : uni(-(1ll << 50), 1ll << 50);
    if ((int64_t)trunc_div_d((double)s, (double)d, recip_lo((double)d)) != (int64_t)idiv(s, d, st)) ++bad;
    // sqrt of variances
    if (it % 16 == 0) {
      const int64_t v = it % 32 == 0 ? uni(0, 2000000) : uni(0, (1ll << 31) - 1);
      int st2 = ST_OK;
      const int64_t ref = (int64_t)wsqrt(v, st2);
      double out;
      const bool ok = wsqrt_d((double)v, out);
      if (ok != (st2 == ST_OK) || (ok && (int64_t)out != ref)) ++bad;
    }
    CHECK(st == ST_OK);
  }
  for (int64_t v : {(int64_t)0, (int64_t)1, (int64_t)2, (int64_t)3, (int64_t)4, (int64_t)999999, (int64_t)1000000, (int64_t)1000001, (int64_t)((1ll << 31) - 1)}) {
    int st2 = ST_OK;
    const int64_t ref = (int64_t)wsqrt(v, st2);
    double out;
    const bool ok = wsqrt_d((double)v, out);
    CHECK(ok == (st2 == ST_OK) && (!ok || (int64_t)out == ref));
  }
  // boundary quotients: remainders 0 and d - 1 around large dividends
  for (int64_t d : {(int64_t)1, (int64_t)2, (int64_t)3, (int64_t)7, (int64_t)1000000, (int64_t)999983, (int64_t)((1ll << 31) - 1)}) {
    for (int64_t q : {(int64_t)0, (int64_t)1, (int64_t)12345, std::min((int64_t)((1ll << 51) / d - 2), (int64_t)((1ll << 47) - 1))}) {
      for (int64_t r : {(int64_t)0, d - 1}) {
        const int64_t t = q * d + r;
        if (t >= (1ll << 51)) continue;
        int st = ST_OK;
        CHECK((int64_t)trunc_div_d((double)t, (double)d, recip_lo((double)d)) == (int64_t)idiv(t, d, st));
        CHECK((int64_t)trunc_div_d(-(double)t, (double)d, recip_lo((double)d)) == (int64_t)idiv(-t, d, st));
      }
    }
  }
  CHECK(bad == 0);
}

// The half-offset forms (wsad_fast.hpp: no remainder test) against the i128 routines: random operands
// over the whole stated ranges, plus dividends whose remainder is 0 or d - 1 at the largest quotients
// (the two fractional parts closest to an integer, where a product error would show).
static void wsad_half_paths() {
  std::mt19937_64 rng(777);
  auto uni = [&](int64_t lo, int64_t hi) { return lo + (int64_t)(rng() % (uint64_t)(hi - lo + 1)); };
  int bad = 0;
  for (int it = 0; it < 4000000 && bad < 10; ++it) {
    int st = ST_OK;
    // quadratic deviation: |d| up to 4.7e7 (quotients to 2.2e9)
    const int64_t d = it & 1 ? uni(-1000000, 1000000) : uni(-47000000, 47000000);
    const int64_t qd = (int64_t)qdev(d, 0, st);
    if ((int64_t)qdev_h((double)d) != qd) ++bad;
    if (qd < (1ll << 32) && (int64_t)qdev_u((double)d) != qd) ++bad;
    // z^2, z^2 * z, z^2 * z^2 of the z-power loop (z2 < 2^25, |z| < 5.8e6)
    const int64_t z = uni(-5800000, 5800000), z2 = uni(0, (1 << 25) - 1);
    if ((int64_t)wmul_pos_h((double)z, (double)z) != (int64_t)wmul(z, z, st)) ++bad;
    if ((int64_t)wmul_h((double)z2, (double)z, z < 0) != (int64_t)wmul(z2, z, st)) ++bad;
    if ((int64_t)wmul_t((double)z2, (double)z) != (int64_t)wmul(z2, z, st)) ++bad;
    if ((int64_t)wmul_pos_h((double)z2, (double)z2) != (int64_t)wmul(z2, z2, st)) ++bad;
    // small products of either sign (a b + 500000 changes sign)
    const int64_t a = uni(-2000, 2000), b = uni(-2000, 2000);
    if ((int64_t)wmul_h((double)a, (double)b, a * b < 0) != (int64_t)wmul(a, b, st)) ++bad;
    if ((int64_t)wmul_t((double)a, (double)b) != (int64_t)wmul(a, b, st)) ++bad;
    // wsad_div by a standard deviation, |a| < 2^26, b up to 2^31
    const int64_t num = it & 2 ? uni(-1000000, 1000000) : uni(-(1 << 26), 1 << 26);
    const int64_t sd = it & 4 ? uni(1, 2000000) : uni(1, (1ll << 31) - 1);
    if ((int64_t)wdiv_h((double)num, (double)sd) != (int64_t)wdiv(num, sd, st)) ++bad;
    CHECK(st == ST_OK);
  }
  CHECK(bad == 0);
  // remainders 0 and d - 1 (and their negatives) at the largest quotients each form takes
  for (int64_t dv : {(int64_t)1, (int64_t)2, (int64_t)3, (int64_t)1414, (int64_t)999983, (int64_t)1000000,
                     (int64_t)46341000, (int64_t)((1ll << 31) - 1)}) {
    const double ib = 1.0 / (double)dv;
    for (int64_t q : {(int64_t)0, (int64_t)1, (int64_t)777, (int64_t)((1ll << 51) / dv - 2), (int64_t)((1ll << 51) / dv / 3)}) {
      for (int64_t r : {(int64_t)0, (int64_t)1, dv - 1}) {
        const int64_t t = q * dv + r;
        if (t >= (1ll << 51) || t < 0) continue;
        int st = ST_OK;
        CHECK((int64_t)tdiv_h((double)t, ib, 0.5 * ib) == (int64_t)idiv(t, dv, st));
        CHECK((int64_t)tdiv_h(-(double)t, ib, 0.5 * ib) == (int64_t)idiv(-t, dv, st));
      }
    }
  }
  // wsad_mul quotients next to 2.25e9 with remainders 0 / 999999 (a b + 500000 = q 1e6 + r)
  for (int64_t q : {(int64_t)2249999999ll, (int64_t)1125899906ll, (int64_t)33554431, (int64_t)1}) {
    for (int64_t r : {(int64_t)0, (int64_t)1, (int64_t)999999}) {
      const int64_t t = q * 1000000 + r - 500000;   // = a * b with b = 1
      int st = ST_OK;
      CHECK((int64_t)wmul_pos_h((double)t, 1.0) == (int64_t)wmul(t, 1, st));
      CHECK((int64_t)wmul_h((double)-t, 1.0, true) == (int64_t)wmul(-t, 1, st));
      CHECK((int64_t)wmul_t((double)-t, 1.0) == (int64_t)wmul(-t, 1, st));
      CHECK((int64_t)wmul_t((double)t, 1.0) == (int64_t)wmul(t, 1, st));
    }
  }
}

// The wide forms (wsad_fast.hpp: unconstrained price-like columns) against the i128 routines.
static void wsad_wide_paths() {
  std::mt19937_64 rng(4242);
  auto uni = [&](int64_t lo, int64_t hi) { return lo + (int64_t)(rng() % (uint64_t)(hi - lo + 1)); };
  int bad = 0;
  for (int it = 0; it < 2000000 && bad < 10; ++it) {
    int st = ST_OK;
    const int64_t d = it & 1 ? uni(-(1ll << 31) + 1, (1ll << 31) - 1) : uni(-3000000, 3000000);
    if ((int64_t)qdev_wide((double)d) != (int64_t)qdev(d, 0, st)) ++bad;
    // relative truncated quotients: k = 2 (smooth median) and k = R (mean)
    const int64_t B = uni(-(1ll << 52), 1ll << 52), k = it % 3 == 0 ? 2 : uni(1, 1024);   // |k B| < 2^62
    const int64_t S = uni(-(1ll << 40), 1ll << 40);
    const int64_t want = (int64_t)idiv((i128)S + (i128)k * B, (i128)k, st) - B;
    if (tdiv_rel(S, B, k) != want) ++bad;
    if (tdiv_rel_fix(S / k, S % k == 0, S < 0, B) != want) ++bad;
    if (it % 8 == 0) {
      const int64_t v = it % 16 == 0 ? uni(0, 1ll << 31) : uni(0, (1ll << 43) - 1);
      int st2 = ST_OK;
      const int64_t ref = (int64_t)wsqrt(v, st2);
      int64_t out = -1;
      const bool ok = wsqrt_wide(v, out);
      if (ok != (st2 == ST_OK) || (ok && out != ref)) ++bad;
    }
    CHECK(st == ST_OK);
  }
  CHECK(bad == 0);
  for (int64_t v : {(int64_t)0, (int64_t)1, (int64_t)2, (int64_t)3, (int64_t)1000000, (int64_t)((1ll << 43) - 1), (int64_t)4000000000ll}) {
    int st2 = ST_OK;
    const int64_t ref = (int64_t)wsqrt(v, st2);
    int64_t out = -1;
    const bool ok = wsqrt_wide(v, out);
    CHECK(ok == (st2 == ST_OK) && (!ok || out == ref));
  }
  // exact multiples and neighbours of 1e6 in d^2 + 500000
  for (int64_t d : {(int64_t)1000, (int64_t)999, (int64_t)1001, (int64_t)2147483647, (int64_t)-2147483647, (int64_t)46340950}) {
    int st = ST_OK;
    CHECK((int64_t)qdev_wide((double)d) == (int64_t)qdev(d, 0, st));
  }
}

int main(int argc, char** argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 8;
  golden_fixture();
  wsad_fast_paths();
  wsad_half_paths();
  wsad_wide_paths();
  batch_vs_single(threads);
  governance_flow();
  io_roundtrip();
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("engine selftest OK (threads=%d)\n", threads);
  return 0;
}
