/* enf_oracle_jsu.c -- CPU restatement of the reference's JohnsonSU distribution functions
 * (TEST INFRASTRUCTURE ONLY; see enf_oracle.h for the contract).
 *
 * src/johnson_trafo.jl:120-129 define, for d = JohnsonSU(gamma, delta, xi, lambda):
 *   pdf(d, x)      = deriv_johnsontrafo(x, ...) * pdf(Normal(), johnsontrafo(x, ...))      :120
 *   cdf(d, x)      = cdf(Normal(), johnsontrafo(x, ...))                                    :121
 *   logpdf(d, x)   = log(deriv_johnsontrafo(x, ...) * pdf(Normal(), johnsontrafo(x, ...)))  :123
 *   logcdf(d, x)   = logcdf(Normal(), johnsontrafo(x, ...))                                 :124
 *   ccdf(d, x)     = 1 - cdf(d, x);  logccdf(d, x) = log(1 - cdf(d, x))                     :125-126
 *   quantile(d, p) = johnsontrafo_inv(quantile(Normal(), p), ...)                           :129
 * and rand(d) falls back to quantile(d, rand()) (Distributions' univariate inverse-CDF sampler).
 * The Normal() functions are StatsFuns' (a dependency of Distributions 0.21-0.25, Project.toml:33,
 * not vendored under /root/reference): normpdf(z) = exp(-z^2/2)/sqrt(2 pi),
 * normcdf(z) = erfc(-z/sqrt2)/2, normlogcdf(z) = log(erfcx(-z/sqrt2)/2) - z^2/2 for z < -1 else
 * log1p(-erfc(z/sqrt2)/2), norminvcdf(p) = -sqrt2 erfcinv(2p). C99 has erfc but neither erfcx nor
 * erfcinv: erfcx is restated from its definition (exp(t^2) erfc(t), asymptotic series beyond
 * t = 26) and norminvcdf by Newton iteration on log Phi in the lower tail (the upper half by
 * symmetry: q = 1 - p is exact for p >= 1/2), converged to the last bit. Evaluated in double;
 * golden values (mpmath, 50 digits) pin it in tests/golden/johnsonsu.npz.
 *
 * Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11; Random123's philox4x32 with R = 10) is restated
 * for the device sampler's uniform stream (enf_johnsonsu_sample in include/enf.h).
 */
#include <math.h>
#include <stdint.h>

#include "enf_oracle.h"

static const double kSqrt2 = 1.41421356237309504880;
static const double kInvSqrt2Pi = 0.39894228040143267794;

/* erfcx(t) = exp(t^2) erfc(t), t >= 0 */
static double or_erfcx(double t) {
  if (t < 26.0) return exp(t * t) * erfc(t);
  /* 1/(t sqrt(pi)) * sum_k (-1)^k (2k-1)!! / (2 t^2)^k */
  const double r = 1.0 / (2.0 * t * t);
  double term = 1.0, s = 1.0;
  for (int k = 1; k < 8; ++k) {
    term *= -(2.0 * k - 1.0) * r;
    s += term;
  }
  return s / (t * 1.77245385090551602730);
}

static double or_normlogcdf(double z) {
  if (z < -1.0) return log(or_erfcx(-z / kSqrt2) / 2.0) - z * z / 2.0;
  return log1p(-erfc(z / kSqrt2) / 2.0);
}

/* Phi^-1(p) for 0 < p < 1/2: Newton on log Phi(y) - log p, d/dy log Phi = phi/Phi =
 * sqrt(2/pi) / erfcx(-y/sqrt2). Start: Abramowitz & Stegun 26.2.23 (|error| < 4.5e-4). */
static double or_norminvcdf_lower(double p) {
  const double t = sqrt(-2.0 * log(p));
  double y = -(t - (2.515517 + 0.802853 * t + 0.010328 * t * t) /
                       (1.0 + 1.432788 * t + 0.189269 * t * t + 0.001308 * t * t * t));
  const double lp = log(p);
  for (int it = 0; it < 50; ++it) {
    const double g = or_normlogcdf(y) - lp;
    const double dg = 0.79788456080286535588 / or_erfcx(-y / kSqrt2);
    const double step = g / dg;
    y -= step;
    if (fabs(step) <= 1e-17 * fabs(y)) break;
  }
  return y;
}

double or_norminvcdf_f64(double p) {
  if (!(p > 0.0)) return p == 0.0 ? -INFINITY : NAN;
  if (!(p < 1.0)) return p == 1.0 ? INFINITY : NAN;
  if (p == 0.5) return 0.0;
  if (p < 0.5) return or_norminvcdf_lower(p);
  return -or_norminvcdf_lower(1.0 - p); /* exact complement (Sterbenz) */
}

double or_jsu_eval_f64(int fn, double x, double g, double d, double xi, double l) {
  if (fn == OR_JSU_QUANTILE) {
    const double z = or_norminvcdf_f64(x);
    return l * sinh((z - g) / d) + xi; /* johnsontrafo_inv, johnson_trafo.jl:34-37 */
  }
  const double u = (x - xi) / l;
  const double y = g + d * asinh(u); /* johnsontrafo, johnson_trafo.jl:29-32 */
  switch (fn) {
    case OR_JSU_PDF:
    case OR_JSU_LOGPDF: {
      const double deriv = (d / l) * (1.0 / sqrt(1.0 + u * u)); /* johnson_trafo.jl:39-42 */
      const double pdf = deriv * (exp(-(y * y) / 2.0) * kInvSqrt2Pi);
      return fn == OR_JSU_PDF ? pdf : log(pdf);
    }
    case OR_JSU_CDF: return erfc(-y / kSqrt2) / 2.0;
    case OR_JSU_LOGCDF: return or_normlogcdf(y);
    case OR_JSU_CCDF: return 1.0 - erfc(-y / kSqrt2) / 2.0;
    case OR_JSU_LOGCCDF: return log(1.0 - erfc(-y / kSqrt2) / 2.0);
    default: return NAN;
  }
}

void or_jsu_eval_vec_f64(int fn, int64_t n, const double* x, double* out, double g, double d, double xi,
                         double l) {
  for (int64_t i = 0; i < n; ++i) out[i] = or_jsu_eval_f64(fn, x[i], g, d, xi, l);
}

static uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

void or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

/* The device sampler's uniforms: call c = offset + i/4 (fp32) or offset + i/2 (fp64), key = seed. */
void or_jsu_uniforms(int is_f64, int64_t n, double* u, uint64_t seed, uint64_t offset) {
  const int per = is_f64 ? 2 : 4;
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  for (int64_t c = 0; c * per < n; ++c) {
    const uint64_t ctr64 = offset + (uint64_t)c;
    const uint32_t ctr[4] = {(uint32_t)ctr64, (uint32_t)(ctr64 >> 32), 0u, 0u};
    uint32_t w[4];
    or_philox4x32_10(ctr, key, w);
    for (int k = 0; k < per && c * per + k < n; ++k) {
      if (is_f64) {
        const uint64_t m = (((uint64_t)w[2 * k] << 32) | w[2 * k + 1]) >> 12;
        u[c * per + k] = ((double)m + 0.5) * 0x1p-52;
      } else {
        u[c * per + k] = (double)(((float)(w[k] >> 9) + 0.5f) * 0x1p-23f);
      }
    }
  }
}
