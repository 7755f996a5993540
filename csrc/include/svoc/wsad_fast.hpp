// Exact fast paths of the wsad operations (signed_decimal.cairo:52-116, math.cairo:170-173,
// 271-292, 320-363) for BOUNDED operands -- the constrained domain [0, 1e6] of the column-parallel
// exact kernel (consensus_wsad.hip).  fp64 arithmetic on integral values instead of i128: every
// routine returns the identical integer that wsad.hpp computes, under the precondition stated on it
// (the kernel checks the preconditions and hands any instance that violates one to the i128 kernel).
//
// Why fp64 is exact here: integers below 2^53 are exact doubles, fma(a, b, c) rounds the exact
// a*b + c once (exact when that result is an integer below 2^53), and a quotient estimated through a
// reciprocal is within 1 of the truth whenever the dividend is below 2^51 -- one remainder test then
// fixes it.  CDNA4 runs fp64 VALU at half the fp32 rate; a 64-bit integer division is ~40 instructions.
#pragma once

#include <math.h>
#include <stdint.h>

#include "wsad.hpp"

namespace svoc {

// The reciprocal floor_div_d takes: 1 / d (rounded to nearest) scaled by (1 - 2^-48).  It lies below 1 / d
// by more than 2^-49 relative -- so t * inv, rounded, stays below t / d and its floor is never too large --
// and by less than 2^-47.8 -- so it falls short of t / d by less than 1 while t / d < 2^47.
SVOC_HD double recip_lo(double d) { return (1.0 / d) * (1.0 - 0x1p-48); }

// floor(t / d) for integral 0 <= t < 2^51, integral 1 <= d < 2^31 and quotient below 2^47 (every use in
// the exact kernel: qdev and wsad_mul quotients < 2^31, wsad_div's < 2^47 for divisors >= 16 or inside
// wsqrt's Newton steps, means / variances < 2^39), given inv = recip_lo(d).  The estimate is the quotient
// or one less, so a single one-sided remainder test fixes it (one compare and one add fewer than a
// two-sided test around a rounded-to-nearest reciprocal).
SVOC_HD double floor_div_d(double t, double d, double inv) {
  const double q = floor(t * inv);    // floor(t / d) or one less
  const double r = fma(-q, d, t);     // exact remainder (an integer in [0, 2d))
  return r >= d ? q + 1.0 : q;
}

// I128Div(a, d) = trunc(a / d) toward zero (signed_decimal.cairo:52-63) for |a| < 2^51, 1 <= d < 2^31, a
// quotient below 2^47; inv = recip_lo(d).
SVOC_HD double trunc_div_d(double a, double d, double inv) {
  // the same one-sided estimate on the signed dividend: trunc(a * inv) is the quotient or one step short
  // toward zero, and the remainder (same sign as a) says which -- no absolute value / sign restore
  const double q = trunc(a * inv);
  const double r = fma(-q, d, a);     // exact, |r| < 2d
  return fabs(r) >= d ? q + copysign(1.0, a) : q;
}

constexpr double kW = 1e6, kInvW = (1.0 / 1e6) * (1.0 - 0x1p-48), kHalfW = 5e5;   // kInvW = recip_lo(1e6)

// wsad_mul(a, b) = I128Div(a * b + HALF_WSAD, WSAD) for |a * b| < 2^50 (signed_decimal.cairo:110-112).
SVOC_HD double wmul_d(double a, double b) { return trunc_div_d(fma(a, b, kHalfW), kW, kInvW); }

// quadratic_deviation(a, b) = wsad_mul(a - b, a - b) for |a - b| < 2^25 (math.cairo:170-173).
SVOC_HD double qdev_d(double a, double b) {
  const double d = a - b;
  return floor_div_d(fma(d, d, kHalfW), kW, kInvW);
}

// wsad_div(a, b) = I128Div(a * WSAD + I128Div(b, 2), b) for 1 <= b < 2^31, |a| < 2^31 and a quotient below
// 2^47 (signed_decimal.cairo:114-116); inv = recip_lo(b).
SVOC_HD double wdiv_d(double a, double b, double inv) {
  return trunc_div_d(fma(a, kW, floor(b * 0.5)), b, inv);
}

// ---- Half-offset forms (no remainder test) -------------------------------------------------------
// For an integer t and an integer divisor d >= 1, (t + 1/2) / d lies at least 1 / (2d) away from every
// integer, and floor((t + 1/2) / d) = floor(t / d).  A product with a reciprocal correctly rounded to
// nearest (the fp64 1e-6 is 0.41 ulp off; 1.0 / d is IEEE division) carries at most 2^-52 relative error
// in total, which moves (t + 1/2) / d by less than 1 / (2d) while |t| < 2^51 (for d = 1e6: while the
// quotient is below 2.25e9) -- so the floor (trunc, for negative t - 1/2) is the exact quotient with no
// remainder correction: 3-4 fp64 instructions per wsad operation instead of 8-10.  The half is folded
// into the fma's addend (exact: every fma result below is a half-integer below 2^52).
constexpr double kInv6 = 1e-6;   // nearest double to 10^-6 (relative error 0.41 * 2^-53)

// quadratic_deviation(a, b) = floor((d^2 + 500000) / 1e6) for d = a - b, |d| < 4.7e7 (math.cairo:170-173)
SVOC_HD double qdev_h(double d) { return floor(fma(d, d, 500000.5) * kInv6); }
// the same as an unsigned word (v_cvt_u32_f64 truncates, which is the floor of a positive value)
SVOC_HD uint32_t qdev_u(double d) { return (uint32_t)(fma(d, d, 500000.5) * kInv6); }

// wsad_mul(a, b) = trunc((a b + 500000) / 1e6) (signed_decimal.cairo:110-112) for integral a, b with
// |a b| < 2.25e15, given neg = (a b < 0): the half goes away from zero.  (a b < 0 but a b + 500000 >= 0:
// both offsets give 0.)
SVOC_HD double wmul_h(double a, double b, bool neg) {
  return trunc(fma(a, b, neg ? 499999.5 : 500000.5) * kInv6);
}
// wsad_mul(a, b) for a b >= 0 (a square, a product of two non-negative values)
SVOC_HD double wmul_pos_h(double a, double b) { return floor(fma(a, b, 500000.5) * kInv6); }

// I128Div(A, b) = trunc(A / b) for integral |A| < 2^51, integral b >= 1, given ib = 1.0 / b (IEEE) and
// hb = 0.5 * ib: trunc((A + sign(A) / 2) / b).  wsad_div(a, b) is this with A = a * 1e6 + floor(b / 2)
// (signed_decimal.cairo:114-116).
// (Written on |A|: round-to-nearest is symmetric, so trunc(fma(-|A|, ib, -hb)) = -trunc(fma(|A|, ib, hb)) -- the
// absolute value is a free source modifier of v_fma_f64 and the sign goes back with one in-place v_bfi_b32,
// where copysign(hb, A) as the addend needed a v_bfi_b32 plus a v_mov_b32 for the pair's low word.)
SVOC_HD double tdiv_h(double A, double ib, double hb) { return copysign(trunc(fma(fabs(A), ib, hb)), A); }
// wsad_mul(a, b) of either sign without the caller's sign test: I128Div(t, 1e6) of the exact t = a b + 500000 by
// tdiv_h (the half offset follows t's sign, which is what truncation toward zero needs) -- for |a b| < 2^51 - 2^19.
// One fma more, but no compare / select / register copy per product (wmul_h's offset pair).
SVOC_HD double wmul_t(double a, double b) { return tdiv_h(fma(a, b, 500000.0), kInv6, 0.5 * kInv6); }
SVOC_HD double wdiv_h(double a, double b) {
  const double ib = 1.0 / b;
  return tdiv_h(fma(a, kW, floor(b * 0.5)), ib, 0.5 * ib);
}

// ---- Wide forms (unconstrained values far from each other: price-like columns) ------------------------
// quadratic_deviation(a, b) for |d| = |a - b| < 2^31 (d^2 < 2^62, quotient < 2^43): the square as the exact
// double-double p + e, the quotient estimated from p (within 2 of the truth), then corrected with the exact
// remainder p - q0 1e6 (an fma: the difference is a small integer) plus e + 500000, floored by the half-offset form.
SVOC_HD double qdev_wide(double d) {
  const double p = d * d;
  const double e = fma(d, d, -p);                      // d^2 = p + e exactly
  const double q0 = floor(p * kInv6);
  const double r = fma(-q0, kW, p) + (e + 500000.0);   // exact: |r| < 2^23
  return q0 + floor((r + 0.5) * kInv6);
}

// floor(A / g) for 0 <= A < 2^63, 1 <= g < 2^53 in int64 (fp64 estimate, exact remainder correction)
SVOC_HD int64_t floor_div_i64(int64_t A, int64_t g) {
  int64_t q = (int64_t)((double)A / (double)g);
  int64_t r = A - q * g;
  while (r < 0) { --q; r += g; }
  while (r >= g) { ++q; r -= g; }
  return q;
}

// sqrt (math.cairo:271-292) for integral 0 <= v < 2^43: wsad_div(v, g) = trunc((v 1e6 + g / 2) / g) in int64
// (the dividend passes 2^53).  Same Newton steps and stop rule as wsqrt; false where the contract divides by 0.
SVOC_HD bool wsqrt_wide(int64_t v, int64_t& out) {
  if (v == 0) {
    out = 0;
    return true;
  }
  int64_t g = v / 2, g2 = g + 1000000;
  for (int i = 0; i < MAX_SQRT_ITERATIONS; ++i) {
    if (g == g2) break;
    if (g == 0) return false;
    const int64_t n = floor_div_i64(v * 1000000 + g / 2, g);
    g2 = g;
    g = (g + n) / 2;
  }
  out = g;
  return true;
}

// trunc((S + k B) / k) - B for k >= 1, |S| < 2^51, |k B + S| < 2^63: the truncated quotient of a sum taken
// relative to a base B (the smooth median and the mean of a column stored relative to its first row,
// math.cairo:113-126, 240-254, with I128Div's truncation toward zero, signed_decimal.cairo:52-63).
SVOC_HD int64_t tdiv_rel(int64_t S, int64_t B, int64_t k) {
  int64_t q = S / k;                                     // trunc(S / k)
  if (q * k != S) {
    const int64_t T = k * B + S;                         // sign of the absolute quotient (never 0 here)
    if (S < 0 && T > 0) q -= 1;                          // floor instead of trunc
    else if (S > 0 && T < 0) q += 1;                     // ceil instead of trunc
  }
  return q;
}

// tdiv_rel from q = trunc(S / k) computed elsewhere (e.g. trunc_div_d with a per-instance reciprocal):
// `exact` = k divides S, `neg` = S < 0.  B + y > 0 (y = S / k, not integral) <=> B + q > 0 for y < 0, and
// B + y < 0 <=> B + q < 0 for y > 0: no multiplication by k.
SVOC_HD int64_t tdiv_rel_fix(int64_t q, bool exact, bool neg, int64_t B) {
  if (exact) return q;
  if (neg && B + q > 0) return q - 1;
  if (!neg && B + q < 0) return q + 1;
  return q;
}

// sqrt (math.cairo:271-292) for integral 0 <= v < 2^31: the same Newton steps and stop rule
// (g == previous g, at most 50 iterations).  Returns false where the contract reverts: a zero
// divisor (sqrt(1) -- g = 0 after the first halving).
SVOC_HD bool wsqrt_d(double v, double& out) {
  if (v == 0.0) {
    out = 0.0;
    return true;
  }
  double g = floor(v * 0.5);
  double g2 = g + kW;
  for (int i = 0; i < MAX_SQRT_ITERATIONS; ++i) {
    if (g == g2) break;
    if (g == 0.0) return false;
    const double n = wdiv_d(v, g, recip_lo(g));   // (quotient <= max(2e6, sqrt(v * 1e6)): Newton from above)
    g2 = g;
    g = floor((g + n) * 0.5);
  }
  out = g;
  return true;
}

}  // namespace svoc
