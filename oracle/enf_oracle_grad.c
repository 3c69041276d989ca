/* enf_oracle_grad.c -- CPU restatement of mvnormal_negll_trafograd and optimize_whitening
 * (TEST INFRASTRUCTURE ONLY: the checker of the device gradient and the timed CPU baseline of the examples'
 * training loops; the product path never links or calls it).
 *
 * The reference differentiates mvnormal_negll_trafo (src/optimize_whitening.jl:7-22) with Zygote: the
 * Householder reflections through their own rrules (src/householder_trafo.jl:22-54, chained :88-124), every
 * elementwise transform and the column sums by Zygote's broadcast AD of the formulas (third-party, absent here:
 * "parity unpinned" beyond central differences). This file restates that reverse pass in the structure a tape
 * gives it: the forward pass keeps every layer's input (D x N), the backward pass walks the layers in reverse
 * with the output cotangent dS/dy and the ladj cotangent -1/N of every column, and accumulates the parameter
 * cotangents summed over the columns:
 *   S = -(sum std_normal_logpdf.(Y) + sum(ladj)) / N      (dS/dY = Y / N, dS/dladj_j = -1 / N)
 * Elementwise derivatives (x input, y output, z = (x - xi)/lambda, s = sqrt(1 + z^2), w = (x - gamma)/delta):
 *   ScaleShift   y = x a + b, ladj = sum_d log|a_d|
 *   Johnson      y = gamma + delta asinh z, ladj_e = log|delta/lambda| - log(1 + z^2)/2
 *   JohnsonInv   y = lambda sinh w + xi,    ladj_e = log|lambda/delta| + log cosh w
 *   Contract     y = (softplus(t1) - softplus(t2))/b, t1 = b(x - c - a), t2 = -b(x - c + a),
 *                ladj_e = log(sigma(t1) + sigma(t2))
 *   Stretch      the inverse of Contract: dy/dx = 1/cc'(y), dy/dth = -dcc/dth(y) / cc'(y), ladj_e = -lcc(y)
 * Householder (householder_trafo.jl:22-40, pullback_v with w = v/|v|):
 *   dv = sum_j inrm (-2 (w'x dY + w'dY x) - inrm (sum_d -2 v_d (w'dY x_d + w'x dY_d)) v / |v| ... (the reference's
 *   expression, restated below), dx = dY - 2 v (v'dY)/(v'v); a chained V re-reflects its output to recover
 *   each column's input (chained_householder_trafo_pullback_V).
 * Gradient layout: include/enf.h enf_flow_param_count (per layer, per field, length-D vectors; V as D x k).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "enf_oracle.h"

#define ORACLE_GRAD_IMPL(T, S, EXP, LOG, SQRT, ASINH, SINH, COSH, TANH, FABS, FMA)                      \
  static T sigm_##S(T t) { return (T)1 / ((T)1 + EXP(-t)); }                                           \
  /* Contract at input x: y, dy/dx, dy/d(a,b,c), L = log(s1 + s2) and dL/dx, dL/d(a,b,c) */              \
  static void contract_d_##S(T x, T a, T b, T c, T* y, T* dydx, T* dyp, T* L, T* dLdx, T* dLp) {       \
    const T xu = x - c, t1 = b * (xu - a), t2 = -b * (xu + a);                                       \
    const T s1 = sigm_##S(t1), s2 = sigm_##S(t2), ss = s1 + s2;                                       \
    const T q1 = s1 * ((T)1 - s1), q2 = s2 * ((T)1 - s2);                                             \
    *y = (LOG((T)1 + EXP(t1)) - LOG((T)1 + EXP(t2))) / b;                                             \
    *dydx = ss;                                                                                        \
    dyp[0] = s2 - s1;                                                                                  \
    dyp[1] = (s1 * (xu - a) + s2 * (xu + a)) / b - *y / b;                                             \
    dyp[2] = -ss;                                                                                      \
    *L = LOG(ss);                                                                                      \
    *dLdx = b * (q1 - q2) / ss;                                                                        \
    dLp[0] = -b * (q1 + q2) / ss;                                                                      \
    dLp[1] = (q1 * (xu - a) - q2 * (xu + a)) / ss;                                                     \
    dLp[2] = -*dLdx;                                                                                   \
  }                                                                                                    \
  /* one elementwise layer's backward for one element: gy (dS/dy), cl (dS/dladj of the column); adds    */ \
  /* the parameter cotangents into dp[0..], returns dS/dx                                              */ \
  static T elem_back_##S(int op, T x, T gy, T cl, const T* p, T* dp) {                                  \
    switch (op) {                                                                                      \
      case OR_SCALESHIFT:                                                                              \
        dp[0] += gy * x + cl / p[0];                                                                   \
        dp[1] += gy;                                                                                   \
        return gy * p[0];                                                                              \
      case OR_JOHNSON: {                                                                               \
        const T g = p[0], d = p[1], xi = p[2], l = p[3];                                               \
        (void)g;                                                                                       \
        const T z = (x - xi) / l, s2 = (T)1 + z * z, s = SQRT(s2);                                     \
        dp[0] += gy;                                                                                   \
        dp[1] += gy * ASINH(z) + cl / d;                                                               \
        dp[2] += -gy * d / (l * s) + cl * z / (l * s2);                                                \
        dp[3] += -gy * d * z / (l * s) + cl * (-(T)1 / l + z * z / (l * s2));                          \
        return gy * d / (l * s) - cl * z / (l * s2);                                                   \
      }                                                                                                \
      case OR_JOHNSON_INV: {                                                                           \
        const T g = p[0], d = p[1], l = p[3];                                                          \
        const T w = (x - g) / d, ch = COSH(w), th = TANH(w);                                           \
        dp[0] += -gy * l * ch / d - cl * th / d;                                                       \
        dp[1] += -gy * l * ch * w / d + cl * (-(T)1 / d - th * w / d);                                 \
        dp[2] += gy;                                                                                   \
        dp[3] += gy * SINH(w) + cl / l;                                                                \
        return gy * l * ch / d + cl * th / d;                                                          \
      }                                                                                                \
      case OR_CENTER_CONTRACT: {                                                                       \
        T y, dydx, dyp[3], L, dLdx, dLp[3];                                                            \
        contract_d_##S(x, p[0], p[1], p[2], &y, &dydx, dyp, &L, &dLdx, dLp);                           \
        for (int q = 0; q < 3; ++q) dp[q] += gy * dyp[q] + cl * dLp[q];                                \
        return gy * dydx + cl * dLdx;                                                                  \
      }                                                                                                \
      case OR_CENTER_STRETCH: {                                                                        \
        const T y = or_center_stretch_##S(x, p[0], p[1], p[2]);                                        \
        T ccy, ccx, ccp[3], L, Ly, Lp[3];                                                              \
        contract_d_##S(y, p[0], p[1], p[2], &ccy, &ccx, ccp, &L, &Ly, Lp);                             \
        const T dydx = (T)1 / ccx;                                                                     \
        for (int q = 0; q < 3; ++q) {                                                                  \
          const T dyq = -ccp[q] / ccx;                                                                 \
          dp[q] += gy * dyq + cl * (-(Ly * dyq + Lp[q]));                                              \
        }                                                                                              \
        return gy * dydx + cl * (-Ly * dydx);                                                          \
      }                                                                                                \
      default:                                                                                         \
        return gy;                                                                                     \
    }                                                                                                  \
  }                                                                                                    \
  /* householder_trafo_pullback_v (householder_trafo.jl:22-40), summed over the N columns of x / dY     */ \
  static void hh_pullback_v_##S(int64_t D, int64_t N, const T* v, const T* X, const T* G, T* dv) {      \
    T vv = 0;                                                                                          \
    for (int64_t d = 0; d < D; ++d) vv += v[d] * v[d];                                                 \
    const T inrm = (T)1 / SQRT(vv), inrm2 = inrm * inrm;                                               \
    for (int64_t d = 0; d < D; ++d) dv[d] = 0;                                                         \
    for (int64_t j = 0; j < N; ++j) {                                                                  \
      const T* x = X + j * D;                                                                          \
      const T* g = G + j * D;                                                                          \
      T vx = 0, vg = 0;                                                                                \
      for (int64_t d = 0; d < D; ++d) {                                                                \
        vx += v[d] * x[d];                                                                             \
        vg += v[d] * g[d];                                                                             \
      }                                                                                                \
      const T w_x = inrm * vx, w_g = inrm * vg;                                                        \
      T dw_v = 0;                                                                                      \
      for (int64_t d = 0; d < D; ++d) dw_v += (T)-2 * v[d] * (w_g * x[d] + w_x * g[d]);                \
      for (int64_t d = 0; d < D; ++d)                                                                  \
        dv[d] += inrm * ((T)-2 * (w_x * g[d] + w_g * x[d]) - inrm2 * dw_v * v[d]);                     \
    }                                                                                                  \
  }                                                                                                    \
  int64_t or_param_count_##S(int64_t D, const oracle_layer* layers, int32_t nlayers) {                 \
    static const int np[6] = {2, 3, 3, 4, 4, 1};                                                       \
    int64_t n = 0;                                                                                     \
    for (int32_t l = 0; l < nlayers; ++l)                                                              \
      n += D * (layers[l].op == OR_HOUSEHOLDER ? layers[l].k : np[layers[l].op]);                      \
    return n;                                                                                          \
  }                                                                                                    \
  /* mvnormal_negll_trafograd: out[0] = negll, out[1 + i] = d negll / d theta_i (enf layout). 0 / -1 */   \
  int or_negll_grad_##S(int64_t D, int64_t N, const T* X, int64_t ldx, const oracle_layer* layers,     \
                        int32_t nlayers, T* out) {                                                     \
    const size_t DN = (size_t)D * (size_t)(N > 0 ? N : 1);                                             \
    T** ins = (T**)calloc((size_t)nlayers + 1, sizeof(T*));                                            \
    T* ladj = (T*)calloc((size_t)(N > 0 ? N : 1), sizeof(T));                                         \
    T* lt = (T*)calloc((size_t)(N > 0 ? N : 1), sizeof(T));                                           \
    int rc = 0;                                                                                        \
    ins[0] = (T*)malloc(DN * sizeof(T));                                                               \
    for (int64_t j = 0; j < N; ++j) memcpy(ins[0] + j * D, X + j * ldx, (size_t)D * sizeof(T));        \
    for (int32_t l = 0; l < nlayers && rc == 0; ++l) { /* forward: the tape keeps every layer input */ \
      const T* p[4] = {(const T*)layers[l].p[0], (const T*)layers[l].p[1], (const T*)layers[l].p[2],   \
                       (const T*)layers[l].p[3]};                                                      \
      ins[l + 1] = (T*)malloc(DN * sizeof(T));                                                         \
      rc = or_trafo_apply_##S(layers[l].op, D, N, p, layers[l].k, ins[l], D, ins[l + 1], D, lt);       \
      for (int64_t j = 0; j < N; ++j) ladj[j] = l == 0 ? lt[j] : ladj[j] + lt[j];                      \
    }                                                                                                  \
    if (rc == 0) {                                                                                     \
      const T* Y = ins[nlayers];                                                                       \
      out[0] = or_mvnormal_negll_##S(D, N, Y, ladj);                                                   \
      T* g = (T*)malloc(DN * sizeof(T)); /* dS/dY = Y / N */                                           \
      T* gn = (T*)malloc(DN * sizeof(T));                                                              \
      for (size_t i = 0; i < (size_t)D * (size_t)N; ++i) g[i] = Y[i] / (T)N;                           \
      const T cl = (T)-1 / (T)N;                                                                       \
      int64_t off = or_param_count_##S(D, layers, nlayers);                                            \
      for (int32_t l = nlayers - 1; l >= 0; --l) {                                                     \
        const oracle_layer* L = &layers[l];                                                            \
        const T* x = ins[l];                                                                           \
        if (L->op == OR_HOUSEHOLDER) {                                                                 \
          const T* V = (const T*)L->p[0];                                                              \
          off -= D * L->k;                                                                             \
          /* chained_householder_trafo_pullback_V / _x: z = the output, re-reflected column by     */    \
          /* column in reverse to each reflection's input; the cotangent reflected the same way    */    \
          T* z = (T*)malloc(DN * sizeof(T));                                                           \
          memcpy(z, ins[l + 1], DN * sizeof(T));                                                       \
          for (int32_t i = L->k - 1; i >= 0; --i) {                                                    \
            const T* v = V + (int64_t)i * D;                                                           \
            or_householder_##S(D, N, v, z, D, z, D);                                                   \
            hh_pullback_v_##S(D, N, v, z, g, out + 1 + off + (int64_t)i * D);                          \
            or_householder_##S(D, N, v, g, D, g, D);                                                   \
          }                                                                                            \
          free(z);                                                                                     \
          (void)x;                                                                                     \
          continue;                                                                                    \
        }                                                                                              \
        static const int np[6] = {2, 3, 3, 4, 4, 1};                                                   \
        const int npl = np[L->op];                                                                     \
        off -= D * npl;                                                                                \
        T* dpo = out + 1 + off;                                                                        \
        for (int64_t q = 0; q < D * npl; ++q) dpo[q] = 0;                                              \
        for (int64_t j = 0; j < N; ++j)                                                                \
          for (int64_t d = 0; d < D; ++d) {                                                            \
            T pv[4], dq[4] = {0, 0, 0, 0};                                                             \
            for (int q = 0; q < npl; ++q) pv[q] = ((const T*)L->p[q])[d];                              \
            gn[d + j * D] = elem_back_##S(L->op, x[d + j * D], g[d + j * D], cl, pv, dq);              \
            for (int q = 0; q < npl; ++q) dpo[q * D + d] += dq[q];                                     \
          }                                                                                            \
        T* t = g;                                                                                      \
        g = gn;                                                                                        \
        gn = t;                                                                                        \
      }                                                                                                \
      free(g);                                                                                         \
      free(gn);                                                                                        \
    }                                                                                                  \
    for (int32_t l = 0; l <= nlayers; ++l) free(ins[l]);                                               \
    free(ins);                                                                                         \
    free(ladj);                                                                                        \
    free(lt);                                                                                          \
    return rc;                                                                                         \
  }                                                                                                    \
  /* optimize_whitening (optimize_whitening.jl:25-45) over Ntot columns X in nbatches minibatches of        */ \
  /* round(Ntot / nbatches), ties to even (Julia round(Int, x), optimize_whitening.jl:31; Iterators.partition: the last one shorter), nepochs epochs: per minibatch   */ \
  /* the gradient above, Optimisers.update with ADAGrad(eta, epsilon) (acc += g^2; theta -= eta g /      */ \
  /* (sqrt(acc) + epsilon), acc starting at epsilon) on every parameter, then the HouseholderTrafo        */ \
  /* functor's normalize! of each V column (householder_trafo.jl:134-146). The layers' parameter         */ \
  /* pointers must point into theta (enf layout, nparams = or_param_count); acc has nparams entries.     */ \
  /* hist receives nepochs * nbatches_actual losses: with zygote != 0 the loss the reference RECORDS,     */ \
  /* i.e. under Zygote.pullback, where rrule(similar_fill) makes every ScaleShiftTrafo's primal ladj zero */ \
  /* (abstract_trafo.jl:30-33): + sum_d log|a_d| at the step's parameters. Returns the number of steps,  */ \
  /* or -1.                                                                                              */ \
  int64_t or_optimize_whitening_##S(int64_t D, int64_t Ntot, const T* X, const oracle_layer* layers,     \
                                    int32_t nlayers, T* theta, T* acc, int64_t nbatches, int64_t nepochs, \
                                    T eta, T eps, T* hist, int32_t zygote) {                           \
    const int64_t np = or_param_count_##S(D, layers, nlayers);                                          \
    int64_t bs = (int64_t)nearbyint((double)Ntot / (double)nbatches); /* ties to even, as round(Int, .) */ \
    if (bs < 1) bs = 1;                                                                                \
    T* out = (T*)malloc((size_t)(1 + np) * sizeof(T));                                                 \
    int64_t step = 0;                                                                                  \
    for (int64_t e = 0; e < nepochs; ++e)                                                              \
      for (int64_t b0 = 0; b0 < Ntot; b0 += bs) {                                                      \
        const int64_t B = Ntot - b0 < bs ? Ntot - b0 : bs;                                             \
        if (or_negll_grad_##S(D, B, X + b0 * D, D, layers, nlayers, out) != 0) {                       \
          free(out);                                                                                   \
          return -1;                                                                                   \
        }                                                                                              \
        T rec = out[0];                                                                                \
        for (int32_t l = 0; zygote && l < nlayers; ++l)                                                \
          if (layers[l].op == OR_SCALESHIFT)                                                           \
            for (int64_t d = 0; d < D; ++d) rec += LOG(FABS(((const T*)layers[l].p[0])[d]));             \
        hist[step++] = rec;                                                                            \
        for (int64_t i = 0; i < np; ++i) {                                                             \
          const T g = out[1 + i];                                                                      \
          acc[i] = acc[i] + g * g;                                                                     \
          theta[i] = theta[i] - eta * g / (SQRT(acc[i]) + eps);                                        \
        }                                                                                              \
        int64_t off = 0;                                                                               \
        static const int npt[6] = {2, 3, 3, 4, 4, 1};                                                  \
        for (int32_t l = 0; l < nlayers; ++l) {                                                        \
          if (layers[l].op == OR_HOUSEHOLDER) {                                                        \
            for (int32_t c = 0; c < layers[l].k; ++c) {                                                \
              T* v = theta + off + (int64_t)c * D;                                                     \
              T ss = 0;                                                                                \
              for (int64_t d = 0; d < D; ++d) ss += v[d] * v[d];                                       \
              const T nrm = SQRT(ss);                                                                  \
              for (int64_t d = 0; d < D; ++d) v[d] = v[d] / nrm;                                       \
            }                                                                                          \
            off += D * layers[l].k;                                                                    \
          } else {                                                                                     \
            off += D * npt[layers[l].op];                                                              \
          }                                                                                            \
        }                                                                                              \
      }                                                                                                \
    free(out);                                                                                         \
    return step;                                                                                       \
  }

ORACLE_GRAD_IMPL(double, f64, exp, log, sqrt, asinh, sinh, cosh, tanh, fabs, fma)
ORACLE_GRAD_IMPL(long double, f80, expl, logl, sqrtl, asinhl, sinhl, coshl, tanhl, fabsl, fmal)
