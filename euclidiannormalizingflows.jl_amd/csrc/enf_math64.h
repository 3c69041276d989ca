// enf_math64.h -- fp64 asinh / log (JohnsonTrafo, johnson_trafo.jl:31,41-57) and sinh / log1p
// (JohnsonTrafoInv, :36,103-104) on the hardware reciprocal / reciprocal-square-root seeds,
// branch-free.
//
// Why: ocml's double asinh carries its argument in double-double through an extended-precision log
// (~193 VALU instructions per element, PMC ~255 per element and layer at config 2), which makes the
// fp64 flows fp64-VALU bound. The reference evaluates Julia's Base.Math asinh (the FreeBSD msun
// algorithm, ~1 ulp) and Base log; these restate the same algorithms at ~1 ulp with three
// hardware seeds (v_rsq_f64, v_rcp_f64) refined by Newton steps instead of IEEE division / sqrt:
//
//   asinh |x| = log1p(a + a^2/(1 + sqrt(1 + a^2)))    a <= 2      (msun s_asinh.c, case 4)
//             = log(a + sqrt(1 + a^2))                2 < a < 2^28 (case 3; sqrt within 1 ulp, so
//                                                      the sum is within ~1 ulp and its log within
//                                                      1 ulp of a value >= log 4)
//             = log(a) + ln 2                         a >= 2^28   (case 2)
//   (a < 2^-28 comes out as x itself: u = 1 and the carried rounding c = a.)
//
// log1p(f) = log(u) + c/u with u = 1 + f rounded and c its exact rounding error (TwoSum), the same
// correction msun's log1p applies. log(u), u >= 1 finite, is msun's e_log.c reduction: u = 2^k m,
// m in [sqrt(1/2), sqrt(2)), f = m - 1, s = f/(2 + f), log m = f - (f^2/2 - s (f^2/2 + R(s^2)))
// with its degree-14 minimax R (coefficients Lg1..Lg7, a published constant set).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "enf_logtab.h"

namespace enf {

// n / d for d > 0 normal: v_rcp_f64 seed (relative error < 2^-22), one Newton step, and one
// residual correction of the quotient (error ~ 0.5 ulp + 2^-90 relative)
__device__ __forceinline__ double div64(double n, double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  const double q = n * r;
  return fma(fma(-d, q, n), r, q);
}

// sqrt(q) for 1 <= q < 2^1000: v_rsq_f64 seed, one Goldschmidt step on (g, h) = (sqrt, 1/(2 sqrt)),
// one residual correction of g (within 1 ulp)
__device__ __forceinline__ double sqrt64_ge1(double q) {
  const double y = __builtin_amdgcn_rsq(q);
  double g = q * y;
  const double h = 0.5 * y;
  const double r = fma(-g, h, 0.5);
  g = fma(g, r, g);
  // the residual q - g^2 is ~2^-44 g, so the seed's h (relative error ~2^-22) suffices for its correction
  // (2^-66 g); the Goldschmidt update of h is not needed (round 4)
  return fma(fma(-g, g, q), h, g);
}

// log(u) for u >= 1 finite (msun e_log.c restated); u = +Inf gives +Inf, NaN gives NaN
__device__ __forceinline__ double log64_ge1(double u) {
  constexpr double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                   Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                   Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                   Lg7 = 1.479819860511658591e-01;
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  double m = __builtin_amdgcn_frexp_mant(u);  // [0.5, 1)
  int k = __builtin_amdgcn_frexp_exp(u);
  const bool lo = m < 0.70710678118654752440;
  m = lo ? m + m : m;
  k = lo ? k - 1 : k;
  const double f = m - 1.0;
  const double s = div64(f, 2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * fma(w, fma(w, Lg6, Lg4), Lg2);
  const double t2 = z * fma(w, fma(w, fma(w, Lg7, Lg5), Lg3), Lg1);
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)k;
  const double r = fma(dk, ln2_hi, -((hfsq - fma(s, hfsq + R, dk * ln2_lo)) - f));
  return u < __builtin_huge_val() ? r : u;
}

// asinh(x) over the whole double range, odd (asinh(-0) = -0), +-Inf -> +-Inf, NaN -> NaN
__device__ __forceinline__ double asinh64(double x) {
  const double a = __builtin_fabs(x);
  const bool huge = a >= 268435456.0;  // 2^28
  const bool small = a <= 2.0;
  const double s = sqrt64_ge1(fma(a, a, 1.0));  // unused when huge (may be Inf there)
  // small: f = a + a^2/(1+s); u = 1 + f. Mid: u = a + s. Both with their TwoSum error c.
  const double t = div64(a * a, 1.0 + s);
  const double f = a + t;
  const double p = small ? 1.0 : a;
  const double qv = small ? f : s;
  const double u0 = p + qv;
  const double bv = u0 - p;
  const double c0 = (p - (u0 - bv)) + (qv - bv);
  const double u = huge ? a : u0;
  const double c = huge ? 0.0 : c0;
  double r = log64_ge1(u) + c * __builtin_amdgcn_rcp(u);
  r = huge ? r + 6.93147180559945309417e-01 : r;
  r = a < __builtin_huge_val() ? r : a;  // Inf stays Inf, NaN stays NaN
  return __builtin_copysign(r, x);
}

// log(1 + t) for t >= 0 (t = +Inf gives +Inf): u = 1 + t rounded, c its TwoSum error, log(u) + c/u
__device__ __forceinline__ double log1p64_ge0(double t) {
  const double u = 1.0 + t;
  const double bv = u - 1.0;
  const double c = (1.0 - (u - bv)) + (t - bv);
  const double r = log64_ge1(u) + c * __builtin_amdgcn_rcp(u);
  return u < __builtin_huge_val() ? r : u;
}

// ---------------------------------------------------------------------------------------------
// Table logarithm and asinh for the fused flow kernels (frag interpreter, fp64 JohnsonTrafo): no
// division, no reciprocal, one hardware seed (v_rsq_f64) per asinh. On gfx950 every fp64 VALU
// instruction issues at half the fp32 rate and v_rcp/v_rsq/v_sqrt_f64 cost ~3.6 of them
// (profiles/r02_microbench15_fp64_costs.txt); msun's reduction above needs a division per log
// (rcp + 4 FMAs) and asinh64 three reciprocals, the forms below none.
//
// log64_tab(u, kadd) = log(u * 2^kadd) for u >= 1 finite: u = 2^k m, m in [1, 2); j = the top B
// fraction bits of m rounded (0..2^B), c_j = 1 + j/2^B; r = fma(m, 1/c_j, -1) (|r| <= ~2^-(B+1), one
// rounding); log m = -log(1/c_j) + log1p(r) with the table's -log(1/c_j) in hi + lo (enf_logtab.h,
// exact to 2^-106 for the stored 1/c_j) and log1p(r) = r + r^2 P(r) (truncation < 2^-53 r). log64_tab:
// B = 5 (33 entries) everywhere: few distinct LDS addresses per wave, so the per-lane lookups mostly
// broadcast. B = 7 / 8 (kLogTabB7 / B8: two / three FMAs fewer per log) were measured in config 2's kernel
// and lost that in LDS bank conflicts (profiles/r03_c2_table_bits_nt.txt);
// j = 0 has 1/c = 1 exactly, so log(1 + tiny) keeps full relative accuracy. tab: the table in LDS
// (3 doubles per entry), filled by the kernel prologue.
// FOLD (round 4, measured variant): k ln2 as one fma with the double nearest ln2 into the table's hi part, the
// table's lo part added directly (one fma fewer; error k (ln2 - RN(ln2)) ~ k 2.3e-17 more)
template <int B, bool FOLD = false>
__device__ __forceinline__ double log64_tab_b(double u, int kadd, const double* __restrict__ tab) {
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const uint64_t b = __builtin_bit_cast(uint64_t, u);
  const uint32_t hi = (uint32_t)(b >> 32), frac = hi & 0xFFFFFu;
  const int k = (int)(hi >> 20) - 1023 + kadd;
  const uint32_t j = (frac + (1u << (19 - B))) >> (20 - B);
  const double m = __builtin_bit_cast(double, ((uint64_t)(frac | 0x3FF00000u) << 32) | (uint32_t)b);
  const double* t = tab + 3 * j;
  const double r = fma(m, t[0], -1.0);
  const double kd = (double)k;
  const double lhi = FOLD ? fma(kd, 6.93147180559945286227e-01, t[1]) : fma(kd, ln2_hi, t[1]);
  const double llo = FOLD ? t[2] : fma(kd, ln2_lo, t[2]);
  double p;
  if constexpr (B == 5) {
    // log1p(r) = r + r^2 P(r) with P the degree-6 Chebyshev economisation of (log1p(r) - r)/r^2 on
    // the reduced range [-0.01515, 2^-6] widened by 2 % (tools/gen_logtab.py --poly; round 4): relative error
    // 2^-57.1 of log1p, as the Taylor form to r^9 it replaces (2^-57.4), with one FMA fewer
    p = fma(-0.12485538735806584, r, 0.14290490248495968);
    p = fma(p, r, -0.16666671910057598);
    p = fma(p, r, 0.19999999413011174);
    p = fma(p, r, -0.24999999999589934);
    p = fma(p, r, 0.33333333333351384);
    p = fma(p, r, -0.5);
  } else if constexpr (B == 6) {
    // the B = 6 table (round 4, measured and not taken: in flow_hj64_kernel 2.374-2.385 vs 2.400-2.418 ms, -1.3 %,
    // for asinh max 1.97 vs 1.50 ulp; profiles/r04_hj64_tb_ab.jsonl, tools/asinh64_tab_check.hip): degree 5 on
    // |r| <= 2^-7 (--poly 6 5: 2^-56.9)
    p = fma(0.14282159536610894, r, -0.16667838296658544);
    p = fma(p, r, 0.20000000262923848);
    p = fma(p, r, -0.2499999997254017);
    p = fma(p, r, 0.3333333333333005);
    p = fma(p, r, -0.500000000000001);
  } else {
    // log1p(r) = r + r^2 P(r), P to r^(NP-2): |r| <= 2^-(B+1), truncation r^NP/NP < 2^-53 r
    constexpr int NP = B >= 8 ? 7 : B >= 7 ? 8 : 12;
    p = ((NP - 1) & 1 ? 1.0 : -1.0) / (NP - 1);
#pragma unroll
    for (int n = NP - 2; n >= 2; --n) p = fma(p, r, (n & 1 ? 1.0 : -1.0) / n);
  }
  return lhi + (r + fma(r * r, p, llo));
}

__device__ __forceinline__ double log64_tab(double u, int kadd, const double* __restrict__ tab) {
  return log64_tab_b<kLogTabBits>(u, kadd, tab);
}

// asinh(x) over the whole double range, odd, +-Inf -> +-Inf, NaN -> NaN, with the table log:
//   a = |x| < 2^26: s = sqrt(1 + a^2) as s1 + corr (rsq seed, one Goldschmidt step on s1 only; corr carries
//     the residual q - s1^2 AND the rounding of q = fl(1 + a^2), e_q = fma(a, a, 1 - q) exactly);
//     u = fl(a + s1) and c its exact error (Fast2Sum) plus corr: a + sqrt(1 + a^2) = u + c, so
//     asinh a = log(u) + c/u, and 1/u = s - a exactly (math), computed as (s1 - a) + corr (s1 - a
//     is exact; c itself carries the Goldschmidt step's error of s1, up to 2^-44 s). For small a this is
//     msun's log1p form without the log1p: u = 1 + (the rounded part) and c the rest.
//   a >= 2^26: asinh a = log(2a) + 1/(4a^2) - ... = log(a) + ln2 within 2^-54 (kadd = 1).
template <int B = kLogTabBits>
__device__ __forceinline__ double asinh64_tab(double x, const double* __restrict__ tab) {
  const double a = __builtin_fabs(x);
  const bool big = a >= 67108864.0;
  const double q = fma(a, a, 1.0);
  const double y = __builtin_amdgcn_rsq(q);
  double g = q * y;
  const double h = 0.5 * y;  // the seed's 1/(2 s): enough for corr (~2^-44 s, so its error is ~2^-66 s)
  const double rr = fma(-g, h, 0.5);
  g = fma(g, rr, g);
  const double eq = fma(a, a, 1.0 - q);
  const double corr = (fma(-g, g, q) + eq) * h;
  const double u0 = a + g;
  const double c0 = (a - (u0 - g)) + corr;
  const double cu = c0 * ((g - a) + corr);  // 1/u = s - a: g - a is exact (Sterbenz), corr completes s
  double r = log64_tab_b<B>(big ? a : u0, big ? 1 : 0, tab);
  r += big ? 0.0 : cu;
  r = a < __builtin_huge_val() ? r : a;  // Inf stays Inf, NaN stays NaN
  return __builtin_copysign(r, x);
}

// asinh64_tab for |x| < 2^26 and finite only (no range selects): the fused kernels take it for a wave whose
// arguments are all in that range (a wave-uniform vote), asinh64_tab otherwise. Same operations and
// roundings as asinh64_tab's a < 2^26 branch, so the same results there.
template <int B = kLogTabBits, bool FOLD = false>
__device__ __forceinline__ double asinh64_tab_fin(double x, const double* __restrict__ tab) {
  const double a = __builtin_fabs(x);
  const double q = fma(a, a, 1.0);
  const double y = __builtin_amdgcn_rsq(q);
  double g = q * y;
  const double h = 0.5 * y;  // the seed's 1/(2 s): enough for corr (~2^-44 s, so its error is ~2^-66 s)
  const double rr = fma(-g, h, 0.5);
  g = fma(g, rr, g);
  const double eq = fma(a, a, 1.0 - q);
  const double corr = (fma(-g, g, q) + eq) * h;
  const double u0 = a + g;
  const double c0 = (a - (u0 - g)) + corr;
  const double cu = c0 * ((g - a) + corr);
  return __builtin_copysign(log64_tab_b<B, FOLD>(u0, 0, tab) + cu, x);
}
// true when asinh64_tab_fin applies to x (|x| < 2^26; false for Inf and NaN)
__device__ __forceinline__ bool asinh64_fin_ok(double x) { return __builtin_fabs(x) < 67108864.0; }

// log(q_1 q_2 ... q_n) for n values q_i >= 1 (a fragment column segment's 1 + z^2): the exponents
// are summed as integers and the mantissas multiplied (< 2^n), so no product overflows; +Inf if a
// factor is +Inf, NaN if one is NaN (the reference's log(1/sqrt(Inf)) = -Inf, NaN propagation).
template <int NQ, int B = kLogTabBits>
__device__ __forceinline__ double logprod64_tab(const double (&q)[NQ], const double* __restrict__ tab) {
  int ks = 0;
  double mp = 1.0, qs = 0.0;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const uint64_t b = __builtin_bit_cast(uint64_t, q[i]);
    const uint32_t hi = (uint32_t)(b >> 32);
    ks += (int)(hi >> 20) - 1023;
    mp *= __builtin_bit_cast(double, ((uint64_t)((hi & 0xFFFFFu) | 0x3FF00000u) << 32) | (uint32_t)b);
    qs += q[i];
  }
  const double l = log64_tab_b<B>(mp, ks, tab);
  return qs < __builtin_huge_val() ? l : qs;
}

// ---------------------------------------------------------------------------------------------
// Round 4: the fp64 CenterStretch / CenterContract steps (center_stretch.jl:4-22, enf_steps.h) run on
// exp64_in, sqrt64_ge1, div64 and the table log instead of ocml's exp / log (42 / 98 VALU instructions each
// in the gfx950 ISA, log alone 76 of them fp64; an element of the literal CenterContract took 4 exp + 3 log
// + 3 divisions, ~510 instructions), and JohnsonTrafoInv's ladj on log1p64_tab.

// e^w for |w| <= 1000: n = rint(w log2e), r = w - n ln2 (hi + lo, |r| <= ln2/2), e^r by its Taylor series to
// r^13 (truncation < 2^-57, as sinh64), then one ldexp (the fp64 Center steps' in-range path, |w| <= 200)
__device__ __forceinline__ double exp64_in(double w) {
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double kd = __builtin_rint(w * 1.44269504088896340736);
  const double r = fma(-kd, ln2_lo, fma(-kd, ln2_hi, w));
  double p = 1.6059043836821614599e-10;
  p = fma(p, r, 2.0876756987868098979e-09);
  p = fma(p, r, 2.5052108385441718775e-08);
  p = fma(p, r, 2.7557319223985890653e-07);
  p = fma(p, r, 2.7557319223985890653e-06);
  p = fma(p, r, 2.4801587301587301587e-05);
  p = fma(p, r, 1.9841269841269841270e-04);
  p = fma(p, r, 1.3888888888888888889e-03);
  p = fma(p, r, 8.3333333333333333333e-03);
  p = fma(p, r, 4.1666666666666666667e-02);
  p = fma(p, r, 1.6666666666666666667e-01);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return __builtin_amdgcn_ldexp(p, (int)kd);
}

// log(1 + t) for t >= 0 (t = +Inf gives +Inf) with the table log: log1p64_ge0's TwoSum correction
__device__ __forceinline__ double log1p64_tab(double t, const double* __restrict__ tab) {
  const double u = 1.0 + t;
  const double bv = u - 1.0;
  const double c = (1.0 - (u - bv)) + (t - bv);
  const double r = log64_tab(u, 0, tab) + c * __builtin_amdgcn_rcp(u);
  return u < __builtin_huge_val() ? r : u;
}

// sinh(w) over the whole double range (johnson_trafo.jl:36), odd, +-Inf -> +-Inf, NaN -> NaN:
//   |w| < 1: the odd Taylor series to w^17 (truncation < 1e-17 relative);
//   else e^|w|/2 - e^-|w|/2 with e^|w| = 2^k e^r (msun e_exp.c reduction, |r| <= ln2/2, e^r by its
//   Taylor series to r^13, truncation < 2^-57) and both halves scaled by ldexp, so sinh stays finite
//   up to its own overflow (|w| ~ 710.48) although e^|w| overflows first.
__device__ __forceinline__ double sinh64(double w) {
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double a = __builtin_fabs(w);
  // series: a + a^3 (1/3! + a^2 (1/5! + ...))
  const double a2 = a * a;
  double sp = 2.8114572543455207632e-15;                 // 1/17!
  sp = fma(sp, a2, 7.6471637318198164759e-13);            // 1/15!
  sp = fma(sp, a2, 1.6059043836821614599e-10);            // 1/13!
  sp = fma(sp, a2, 2.5052108385441718775e-08);            // 1/11!
  sp = fma(sp, a2, 2.7557319223985890653e-06);            // 1/9!
  sp = fma(sp, a2, 1.9841269841269841270e-04);            // 1/7!
  sp = fma(sp, a2, 8.3333333333333333333e-03);            // 1/5!
  sp = fma(sp, a2, 1.6666666666666666667e-01);            // 1/3!
  const double small = fma(a * a2, sp, a);
  // exponential form
  const double am = a < 1000.0 ? a : 1000.0;              // keeps k finite; Inf/NaN handled below
  const double kd = __builtin_rint(am * 1.44269504088896340736);
  const double r = fma(-kd, ln2_lo, fma(-kd, ln2_hi, am));
  double p = 1.6059043836821614599e-10;                    // 1/13!
  p = fma(p, r, 2.0876756987868098979e-09);                // 1/12!
  p = fma(p, r, 2.5052108385441718775e-08);                // 1/11!
  p = fma(p, r, 2.7557319223985890653e-07);                // 1/10!
  p = fma(p, r, 2.7557319223985890653e-06);                // 1/9!
  p = fma(p, r, 2.4801587301587301587e-05);                // 1/8!
  p = fma(p, r, 1.9841269841269841270e-04);                // 1/7!
  p = fma(p, r, 1.3888888888888888889e-03);                // 1/6!
  p = fma(p, r, 8.3333333333333333333e-03);                // 1/5!
  p = fma(p, r, 4.1666666666666666667e-02);                // 1/4!
  p = fma(p, r, 1.6666666666666666667e-01);                // 1/3!
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);                                      // e^r in [0.70, 1.42]
  double q = __builtin_amdgcn_rcp(p);                      // e^-r: seed + two Newton steps
  q = fma(q, fma(-p, q, 1.0), q);
  q = fma(q, fma(-p, q, 1.0), q);
  const int k = (int)kd;
  const double big = __builtin_amdgcn_ldexp(p, k - 1) - __builtin_amdgcn_ldexp(q, -k - 1);
  double res = a < 1.0 ? small : big;
  res = a < __builtin_huge_val() ? res : a;  // Inf stays Inf, NaN stays NaN
  return __builtin_copysign(res, w);
}

// sinh(w) for |w| < ~709 (the compiled fp64 inverse program's in-range path, round 4; its range check admits
// |w| < ~347), branch-free, with msun's expm1 form (s_sinh.c): t = expm1(|w|), sinh = (t + t/(t + 1))/2 (an
// identity for every w; both terms >= 0, so no cancellation). expm1(a) = 2^k (1 + em) - 1 = fma(2^k, em,
// 2^k - 1) with k = rint(a/ln2), r = a - k ln2 (hi + lo), em = expm1(r) = r + r^2 P(r), P the degree-10
// Chebyshev economisation on |r| <= ln2/2 (tools/gen_logtab.py --poly-expm1: relative error 2^-60.7); 2^k - 1 is
// exact (k <= 53; beyond it the 1 no longer matters). t/(t + 1) as div64. One v_rcp_f64, ~28 fp64 instructions,
// against sinh64's two exp-form evaluations plus the Taylor series. expm1_64_in (a >= 0) is shared with the fp64
// CenterContract's in-range path (enf_steps.h).
__device__ __forceinline__ double expm1_64_in(double a) {
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double kd = __builtin_rint(a * 1.44269504088896340736);
  const double r = fma(-kd, ln2_lo, fma(-kd, ln2_hi, a));
  double p = fma(2.0914686968086876e-09, r, 2.5105217004720745e-08);
  p = fma(p, r, 2.75572736431103e-07);
  p = fma(p, r, 2.7557255400206422e-06);
  p = fma(p, r, 2.4801587325547743e-05);
  p = fma(p, r, 0.00019841269874820627);
  p = fma(p, r, 0.0013888888888883748);
  p = fma(p, r, 0.008333333333326136);
  p = fma(p, r, 0.04166666666666667);
  p = fma(p, r, 0.1666666666666667);
  p = fma(p, r, 0.5);
  const double em = fma(r * r, p, r);
  const double S = __builtin_amdgcn_ldexp(1.0, (int)kd);
  return fma(S, em, S - 1.0);
}

__device__ __forceinline__ double sinh64_in(double w) {
  const double t = expm1_64_in(__builtin_fabs(w));
  const double d = div64(t, t + 1.0);
  // (t + d for every |w|: max 2.3 ulp, mean 0.31 (sinh64: 1.6 / 0.26), tools/asinh64_tab_check.hip. msun's
  // 2t - t d below |w| = 1 would take ~1 ulp off the small-|w| side for a select per element: +5 VALU per
  // element of the inverse program, not taken.)
  return __builtin_copysign(0.5 * (t + d), w);
}

}  // namespace enf
