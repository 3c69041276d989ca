/* enf_oracle.c -- CPU restatement of the reference bijector math (TEST INFRASTRUCTURE ONLY).
 *
 * See enf_oracle.h for the contract. Every function follows the cited line of
 * /root/reference (bat/EuclidianNormalizingFlows.jl v0.1.0) with the same operation order,
 * evaluated in the precision T of the inputs (Julia's float(promote_type(...)) rule).
 * Julia's `muladd` is taken as a fused multiply-add (what LLVM emits for it on x86-64 with
 * FMA); Julia's `sum` over a column (reducedim along dim 1) is a left-to-right sum.
 *
 * The flow driver (or_flow_apply_*) is "reference-structured": it applies one transform at a
 * time over the whole D x N batch, materialising Y and the D x N elementwise-ladj temporary and
 * reducing it with sum(dims=1), as the Julia broadcasts do (src/johnson_trafo.jl:76-80,
 * src/abstract_trafo.jl:9), then adds per-layer ladj rows in composition order
 * (ChangesOfVariables 0.1 with_logabsdet_jacobian(::ComposedFunction): inner first).
 */
#include "enf_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* Julia sign(): -1, 0, +1 (NaN stays NaN) */
#define SIGN_OF(T, x) ((x) > (T)0 ? (T)1 : ((x) < (T)0 ? (T)-1 : (x)))

#define ORACLE_IMPL(T, S, EXP, LOG, SQRT, ASINH, SINH, COSH, FABS, FMA)                             \
  /* src/center_stretch.jl:4-8 */                                                                  \
  T or_center_stretch_##S(T x, T a, T b, T c) {                                                    \
    T e = EXP(FABS(b * x));                                                                        \
    T ome = (T)1 - e;                                                                              \
    T inner = (SQRT(ome * ome * EXP((T)2 * b * a) + (T)4 * e) - ome * EXP(b * a)) / (T)2;          \
    return SIGN_OF(T, x) * LOG(inner) / b + c;                                                     \
  }                                                                                                \
  /* src/center_stretch.jl:11-15 */                                                                \
  T or_center_contract_##S(T x, T a, T b, T c) {                                                   \
    T xu = x - c;                                                                                  \
    return (LOG((T)1 + EXP(b * (xu - a))) - LOG((T)1 + EXP(-b * (xu + a)))) / b;                   \
  }                                                                                                \
  /* src/center_stretch.jl:17-22 */                                                                \
  T or_center_contract_ladj_##S(T x, T a, T b, T c) {                                              \
    T xu = x - c;                                                                                  \
    T dy = (T)1 / ((T)1 + EXP(-b * (xu - a))) + (T)1 / ((T)1 + EXP(b * (xu + a)));                 \
    return LOG(FABS(dy));                                                                          \
  }                                                                                                \
  /* src/johnson_trafo.jl:29-32 */                                                                 \
  T or_johnsontrafo_##S(T x, T g, T d, T xi, T l) { return g + d * ASINH((x - xi) / l); }          \
  /* src/johnson_trafo.jl:34-37 */                                                                 \
  T or_johnsontrafo_inv_##S(T x, T g, T d, T xi, T l) { return l * SINH((x - g) / d) + xi; }       \
  /* src/johnson_trafo.jl:39-42 */                                                                 \
  T or_deriv_johnsontrafo_##S(T x, T g, T d, T xi, T l) {                                          \
    T z = (x - xi) / l;                                                                            \
    (void)g;                                                                                       \
    return (d / l) * ((T)1 / SQRT((T)1 + z * z));                                                  \
  }                                                                                                \
  /* src/johnson_trafo.jl:44-47 */                                                                 \
  T or_deriv_johnsontrafo_inv_##S(T x, T g, T d, T xi, T l) {                                      \
    (void)xi;                                                                                      \
    return l * COSH((x - g) / d) / d;                                                              \
  }                                                                                                \
  /* src/johnson_trafo.jl:49-52 */                                                                 \
  T or_johnsontrafo_ladj_##S(T x, T g, T d, T xi, T l) {                                           \
    return LOG(FABS(or_deriv_johnsontrafo_##S(x, g, d, xi, l)));                                   \
  }                                                                                                \
  /* src/johnson_trafo.jl:54-57 */                                                                 \
  T or_johnsontrafo_inv_ladj_##S(T x, T g, T d, T xi, T l) {                                       \
    return LOG(FABS(or_deriv_johnsontrafo_inv_##S(x, g, d, xi, l)));                               \
  }                                                                                                \
  /* src/householder_trafo.jl:4-11: k = (v'x)/(v'v); y .= muladd.(-2 .* k, v, x). x, y may    */  \
  /* alias: k is formed from the whole column before any element is written.                  */  \
  void or_householder_##S(int64_t D, int64_t N, const T* v, const T* X, int64_t ldx, T* Y,         \
                          int64_t ldy) {                                                           \
    T vv = 0;                                                                                      \
    for (int64_t d = 0; d < D; ++d) vv += v[d] * v[d];                                             \
    for (int64_t j = 0; j < N; ++j) {                                                              \
      const T* x = X + j * ldx;                                                                    \
      T* y = Y + j * ldy;                                                                          \
      T vx = 0;                                                                                    \
      for (int64_t d = 0; d < D; ++d) vx += v[d] * x[d];                                           \
      T m2k = (T)-2 * (vx / vv);                                                                   \
      for (int64_t d = 0; d < D; ++d) y[d] = FMA(m2k, v[d], x[d]);                                 \
    }                                                                                              \
  }                                                                                                \
  /* src/householder_trafo.jl:71-85: y .= x; reflect by V[:,1], ..., V[:,K] in column order */    \
  void or_chained_householder_##S(int64_t D, int64_t K, int64_t N, const T* V, const T* X,         \
                                  int64_t ldx, T* Y, int64_t ldy) {                                \
    for (int64_t j = 0; j < N; ++j)                                                                \
      if (Y + j * ldy != X + j * ldx) memmove(Y + j * ldy, X + j * ldx, (size_t)D * sizeof(T));    \
    for (int64_t i = 0; i < K; ++i) or_householder_##S(D, N, V + i * D, Y, ldy, Y, ldy);           \
  }                                                                                                \
  /* One transform over the batch: returns 0 on success, -1 on an unknown op.                 */  \
  /* ladj (length N) is OVERWRITTEN with the transform's per-sample ladj.                     */  \
  int or_trafo_apply_##S(int op, int64_t D, int64_t N, const T* const* p, int32_t k, const T* X,   \
                         int64_t ldx, T* Y, int64_t ldy, T* ladj) {                                \
    T* tmp = NULL;                                                                                 \
    if (op == OR_CENTER_STRETCH || op == OR_CENTER_CONTRACT || op == OR_JOHNSON ||                 \
        op == OR_JOHNSON_INV)                                                                      \
      tmp = (T*)malloc((size_t)D * (size_t)(N > 0 ? N : 1) * sizeof(T)); /* D x N ladj temp */     \
    switch (op) {                                                                                  \
      case OR_SCALESHIFT: { /* src/scale_shift_trafo.jl:15-24 */                                   \
        T l = 0;                                                                                   \
        for (int64_t d = 0; d < D; ++d) l += LOG(FABS(p[0][d]));                                   \
        for (int64_t j = 0; j < N; ++j) {                                                          \
          for (int64_t d = 0; d < D; ++d)                                                          \
            Y[d + j * ldy] = FMA(X[d + j * ldx], p[0][d], p[1][d]);                                \
          if (ladj) ladj[j] = l;                                                                   \
        }                                                                                          \
        break;                                                                                     \
      }                                                                                            \
      case OR_CENTER_STRETCH: /* src/center_stretch.jl:37-43: ladj from the OUTPUT */              \
        for (int64_t j = 0; j < N; ++j)                                                            \
          for (int64_t d = 0; d < D; ++d)                                                          \
            Y[d + j * ldy] = or_center_stretch_##S(X[d + j * ldx], p[0][d], p[1][d], p[2][d]);     \
        for (int64_t j = 0; j < N; ++j)                                                            \
          for (int64_t d = 0; d < D; ++d)                                                          \
            tmp[d + j * D] =                                                                       \
                or_center_contract_ladj_##S(Y[d + j * ldy], p[0][d], p[1][d], p[2][d]);            \
        break;                                                                                     \
      case OR_CENTER_CONTRACT: /* src/center_stretch.jl:61-67: ladj from the INPUT */              \
        for (int64_t j = 0; j < N; ++j)                                                            \
          for (int64_t d = 0; d < D; ++d)                                                          \
            tmp[d + j * D] =                                                                       \
                or_center_contract_ladj_##S(X[d + j * ldx], p[0][d], p[1][d], p[2][d]);            \
        for (int64_t j = 0; j < N; ++j)                                                            \
          for (int64_t d = 0; d < D; ++d)                                                          \
            Y[d + j * ldy] = or_center_contract_##S(X[d + j * ldx], p[0][d], p[1][d], p[2][d]);    \
        break;                                                                                     \
      case OR_JOHNSON: /* src/johnson_trafo.jl:74-80: ladj from the INPUT */                       \
        for (int64_t j = 0; j < N; ++j)                                                            \
          for (int64_t d = 0; d < D; ++d)                                                          \
            tmp[d + j * D] = or_johnsontrafo_ladj_##S(X[d + j * ldx], p[0][d], p[1][d], p[2][d],   \
                                                      p[3][d]);                                    \
        for (int64_t j = 0; j < N; ++j)                                                            \
          for (int64_t d = 0; d < D; ++d)                                                          \
            Y[d + j * ldy] =                                                                       \
                or_johnsontrafo_##S(X[d + j * ldx], p[0][d], p[1][d], p[2][d], p[3][d]);           \
        break;                                                                                     \
      case OR_JOHNSON_INV: /* src/johnson_trafo.jl:99-105: ladj from the OUTPUT */                 \
        for (int64_t j = 0; j < N; ++j)                                                            \
          for (int64_t d = 0; d < D; ++d)                                                          \
            Y[d + j * ldy] =                                                                       \
                or_johnsontrafo_inv_##S(X[d + j * ldx], p[0][d], p[1][d], p[2][d], p[3][d]);       \
        for (int64_t j = 0; j < N; ++j)                                                            \
          for (int64_t d = 0; d < D; ++d)                                                          \
            tmp[d + j * D] = or_johnsontrafo_ladj_##S(Y[d + j * ldy], p[0][d], p[1][d], p[2][d],   \
                                                      p[3][d]);                                    \
        break;                                                                                     \
      case OR_HOUSEHOLDER: /* src/householder_trafo.jl:156-160: ladj = 0 */                        \
        or_chained_householder_##S(D, k, N, p[0], X, ldx, Y, ldy);                                 \
        if (ladj)                                                                                  \
          for (int64_t j = 0; j < N; ++j) ladj[j] = 0;                                             \
        break;                                                                                     \
      default:                                                                                     \
        free(tmp);                                                                                 \
        return -1;                                                                                 \
    }                                                                                              \
    if (tmp) {                                                                                     \
      /* sum_ladjs, src/abstract_trafo.jl:9: column sums; the forward CenterStretch and       */  \
      /* JohnsonTrafoInv negate the summed row (center_stretch.jl:42, johnson_trafo.jl:104) */    \
      const T sgn = (op == OR_CENTER_STRETCH || op == OR_JOHNSON_INV) ? (T)-1 : (T)1;              \
      if (ladj)                                                                                    \
        for (int64_t j = 0; j < N; ++j) {                                                          \
          T s = 0;                                                                                 \
          for (int64_t d = 0; d < D; ++d) s += tmp[d + j * D];                                     \
          ladj[j] = sgn * s;                                                                       \
        }                                                                                          \
      free(tmp);                                                                                   \
    }                                                                                              \
    return 0;                                                                                      \
  }                                                                                                \
  /* Composed flow, layers[0] innermost. ladj (length N, may be NULL) = sum of layer ladjs,   */  \
  /* added in application order (ChangesOfVariables: ladj_inner + ladj_outer).               */  \
  int or_flow_apply_##S(int64_t D, int64_t N, const T* X, int64_t ldx, T* Y, int64_t ldy,          \
                        T* ladj, const oracle_layer* layers, int32_t nlayers) {                    \
    T* lt = (T*)malloc((size_t)(N > 0 ? N : 1) * sizeof(T));                                       \
    T* cur = (T*)malloc((size_t)D * (size_t)(N > 0 ? N : 1) * sizeof(T));                          \
    for (int64_t j = 0; j < N; ++j) memcpy(cur + j * D, X + j * ldx, (size_t)D * sizeof(T));       \
    if (ladj)                                                                                      \
      for (int64_t j = 0; j < N; ++j) ladj[j] = 0;                                                 \
    int rc = 0;                                                                                    \
    for (int32_t l = 0; l < nlayers && rc == 0; ++l) {                                             \
      const T* p[4] = {(const T*)layers[l].p[0], (const T*)layers[l].p[1],                         \
                       (const T*)layers[l].p[2], (const T*)layers[l].p[3]};                        \
      T* nxt = (T*)malloc((size_t)D * (size_t)(N > 0 ? N : 1) * sizeof(T));                        \
      rc = or_trafo_apply_##S(layers[l].op, D, N, p, layers[l].k, cur, D, nxt, D, lt);             \
      free(cur);                                                                                   \
      cur = nxt;                                                                                   \
      if (ladj && rc == 0)                                                                         \
        for (int64_t j = 0; j < N; ++j) ladj[j] = (l == 0) ? lt[j] : ladj[j] + lt[j];              \
    }                                                                                              \
    for (int64_t j = 0; j < N; ++j) memcpy(Y + j * ldy, cur + j * D, (size_t)D * sizeof(T));      \
    free(cur);                                                                                     \
    free(lt);                                                                                      \
    return rc;                                                                                     \
  }                                                                                                \
  /* Same computation, column blocks spread over nthreads OpenMP threads (CPU baseline #2). Blocks */ \
  /* of 256 columns keep every temporary below glibc's mmap threshold (128 KiB at D = 32 fp32), so */ \
  /* the per-block malloc/free stays in the threads' arenas instead of mmap/munmap + page zeroing   */ \
  /* serialised on the address-space lock (4096-column blocks scaled 10x on 256 threads).          */ \
  int or_flow_apply_mt_##S(int64_t D, int64_t N, const T* X, int64_t ldx, T* Y, int64_t ldy,       \
                           T* ladj, const oracle_layer* layers, int32_t nlayers, int nthreads) {   \
    const int64_t B = 256;                                                                         \
    const int64_t nb = (N + B - 1) / B;                                                            \
    int rc = 0;                                                                                    \
    _Pragma("omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(|: rc)")        \
    for (int64_t b = 0; b < nb; ++b) {                                                             \
      int64_t j0 = b * B, n = (N - j0 < B) ? N - j0 : B;                                           \
      rc |= or_flow_apply_##S(D, n, X + j0 * ldx, ldx, Y + j0 * ldy, ldy, ladj ? ladj + j0 : NULL, \
                              layers, nlayers);                                                    \
    }                                                                                              \
    (void)nthreads;                                                                                \
    return rc;                                                                                     \
  }                                                                                                \
  /* src/optimize_whitening.jl:4-15: -(sum(std_normal_logpdf.(Y)) + sum(ladj)) / N,            */  \
  /* with Julia's pairwise summation (blocks of 1024) for the D x N sum.                       */  \
  static T pairwise_##S(const T* a, int64_t n, int sq) {                                           \
    if (n <= 1024) {                                                                               \
      T s = 0;                                                                                     \
      for (int64_t i = 0; i < n; ++i) s += sq ? -(a[i] * a[i] + (T)1.8378770664093453) / (T)2     \
                                              : a[i];                                              \
      return s;                                                                                    \
    }                                                                                              \
    int64_t h = n >> 1;                                                                            \
    return pairwise_##S(a, h, sq) + pairwise_##S(a + h, n - h, sq);                                \
  }                                                                                                \
  T or_mvnormal_negll_##S(int64_t D, int64_t N, const T* Y, const T* ladj) {                       \
    T ll = (pairwise_##S(Y, D * N, 1) + pairwise_##S(ladj, N, 0)) / (T)N;                          \
    return -ll;                                                                                    \
  }

ORACLE_IMPL(double, f64, exp, log, sqrt, asinh, sinh, cosh, fabs, fma)
ORACLE_IMPL(float, f32, expf, logf, sqrtf, asinhf, sinhf, coshf, fabsf, fmaf)
ORACLE_IMPL(long double, f80, expl, logl, sqrtl, asinhl, sinhl, coshl, fabsl, fmal)
