// wsad fixed point (i128 scaled by 1e6), bit-exact with contract/src/signed_decimal.cairo and the
// sqrt of contract/src/math.cairo:271-292.  Host and device: the CPU golden engine and the HIP exact
// kernel include this same header, so both produce the same integers and the same first-error
// status.  Panics become a sticky status word (first error wins) instead of a revert.
#pragma once

#include <stdint.h>

#include "status.hpp"

#if defined(__HIPCC__)
#define SVOC_HD __host__ __device__ __forceinline__
#else
#define SVOC_HD inline
#endif

namespace svoc {

typedef __int128 i128;
typedef unsigned __int128 u128;

constexpr int64_t WSAD = 1000000;
constexpr int64_t HALF_WSAD = 500000;
constexpr int MAX_SQRT_ITERATIONS = 50;

SVOC_HD void fail(int& st, int code) {
  if (st == ST_OK) st = code;
}

SVOC_HD i128 i128_min() { return (i128)((u128)1 << 127); }

SVOC_HD i128 add(i128 a, i128 b, int& st) {
  i128 r;
  if (__builtin_add_overflow(a, b, &r)) { fail(st, ST_OVERFLOW); return 0; }
  return r;
}

SVOC_HD i128 sub(i128 a, i128 b, int& st) {
  i128 r;
  if (__builtin_sub_overflow(a, b, &r)) { fail(st, ST_OVERFLOW); return 0; }
  return r;
}

SVOC_HD i128 mul(i128 a, i128 b, int& st) {
  i128 r;
  if (__builtin_mul_overflow(a, b, &r)) { fail(st, ST_OVERFLOW); return 0; }
  return r;
}

// I128Div (signed_decimal.cairo:52-63): |a| / |b| truncated, negated when the signs differ.
// as_unsigned() of i128::MIN multiplies by -1 and overflows in Cairo -> OVERFLOW.
SVOC_HD i128 idiv(i128 a, i128 b, int& st) {
  if (b == 0) { fail(st, ST_DIV_BY_ZERO); return 0; }
  if (a == i128_min() || b == i128_min()) { fail(st, ST_OVERFLOW); return 0; }
  u128 ua = a < 0 ? (u128)(-a) : (u128)a;
  u128 ub = b < 0 ? (u128)(-b) : (u128)b;
  // 64-bit operands (the common case: wsad values and their products below 2^64) take the much
  // cheaper 64-bit division; same truncated quotient
  const i128 q = ((ua | ub) >> 64) == 0 ? (i128)((uint64_t)ua / (uint64_t)ub) : (i128)(ua / ub);
  return ((a >= 0) == (b >= 0)) ? q : -q;
}

// Fast path for a positive 64-bit divisor that fits (the common case: W, 2, n, D).
SVOC_HD i128 idiv_pos64(i128 a, int64_t b, int& st) {
  if (b == 0) { fail(st, ST_DIV_BY_ZERO); return 0; }
  if (a >= 0) {
    if (a <= (i128)INT64_MAX) return (i128)((uint64_t)a / (uint64_t)b);
    return (i128)((u128)a / (u128)b);
  }
  if (a == i128_min()) { fail(st, ST_OVERFLOW); return 0; }
  i128 na = -a;
  if (na <= (i128)INT64_MAX) return -(i128)((uint64_t)na / (uint64_t)b);
  return -(i128)((u128)na / (u128)b);
}

// wsad_mul (signed_decimal.cairo:110-112): (a*b + HALF_WSAD) / WSAD, HALF added whatever the sign.
SVOC_HD i128 wmul(i128 a, i128 b, int& st) {
  return idiv_pos64(add(mul(a, b, st), HALF_WSAD, st), WSAD, st);
}

// wsad_div (signed_decimal.cairo:114-116): (a*WSAD + b/2) / b.
SVOC_HD i128 wdiv(i128 a, i128 b, int& st) {
  return idiv(add(mul(a, WSAD, st), idiv(b, 2, st), st), b, st);
}

// math.cairo:271-292.  sqrt(0) = 0; sqrt(1): g = 0 -> wdiv(.., 0) -> DIV_BY_ZERO.
SVOC_HD i128 wsqrt(i128 v, int& st) {
  if (v == 0) return 0;
  i128 g = idiv_pos64(v, 2, st);
  i128 g2 = add(g, WSAD, st);
  for (int i = 0; i < MAX_SQRT_ITERATIONS; ++i) {
    if (g == g2 || st != ST_OK) break;
    i128 n = wdiv(v, g, st);
    g2 = g;
    g = idiv_pos64(add(g, n, st), 2, st);
  }
  return g;
}

SVOC_HD i128 qdev(i128 a, i128 b, int& st) {  // quadratic_deviation (math.cairo:170-173)
  i128 x = sub(a, b, st);
  return wmul(x, x, st);
}

SVOC_HD i128 constrained_reliability(i128 mean_qr, int64_t dim, int& st) {  // contract.cairo:436-439
  return sub(WSAD, mul(wsqrt(idiv_pos64(mean_qr, dim, st), st), 2, st), st);
}

SVOC_HD i128 unconstrained_reliability(i128 sd, i128 max_spread, int& st) {  // contract.cairo:365-368
  i128 m = max_spread < sd ? max_spread : sd;
  return sub(WSAD, wdiv(m, max_spread, st), st);
}

SVOC_HD bool in_unit_interval(i128 v) { return v >= 0 && v <= WSAD; }

// skewness / kurtosis tails (math.cairo:336-337, 359-362), from the z-score sums.
SVOC_HD i128 skew_from_sum(i128 s3, int64_t n, int& st) {
  return idiv(mul(s3, n, st), mul(n - 1, n - 2, st), st);
}

SVOC_HD i128 kurt_from_sum(i128 s4, int64_t n, int& st) {
  i128 term1 = idiv(mul(mul(s4, n, st), n + 1, st), n - 1, st);
  i128 term2 = mul(mul(mul(3, WSAD, st), n - 1, st), n - 1, st);
  return idiv(sub(term1, term2, st), mul(n - 2, n - 3, st), st);
}

}  // namespace svoc
