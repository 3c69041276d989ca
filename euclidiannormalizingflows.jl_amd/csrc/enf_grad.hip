// enf_grad.hip -- fused forward + backward of the whitening loss (config 5, optimize_whitening).
//
// For the N local samples (columns) of X and the composed flow y = f_L o ... o f_1 (x):
//   S      = sum_j [ sum_d (y_dj^2 + log 2pi)/2 - ladj_j ]            (= B * mvnormal_negll_trafo,
//                                                                    src/optimize_whitening.jl:7-15)
//   dS/dth for every flow parameter                                   (mvnormal_negll_trafograd, :18-22)
// out[0] += S, out[1 + i] += dS/dth_i (layout: include/enf.h enf_flow_param_count).
//
// Kernel structure: fragment layout as the forward kernel (enf_flow.hip), one fragment (16 B) per
// lane per tile. The forward pass stores every step's input in LDS (the reference's chained
// Householder pullback instead recomputes inputs by re-reflection, householder_trafo.jl:88-103;
// storing is exact and costs 1 KiB of LDS per step per wave). The backward pass walks the steps
// in reverse with the cotangent g = dS/du (starting at g = y), accumulating per-row parameter
// gradients into LDS (double LDS atomics, summed per block), and writes one partial gradient
// vector per block; a second kernel sums the block partials in double, in block order, applies
// the Householder direction projection (householder_trafo.jl:22-40) and adds into out.
//
// The arithmetic here is the accurate library form (ocml asinh/log/exp/... in T); it is not the
// headline path.
//
// enf_flow_vjp runs the same kernel with general cotangents (VJP = true): the backward pass starts
// from g = dY and weights every step's ladj derivative by the sample's dladj (the negll loss is the
// special case dY = Y, dladj = -1), writes the input cotangent dX = g after the last step, and the
// block partials hold the parameter VJP summed over the samples (householder_trafo.jl:22-54,88-124:
// the rrules of householder_trafo / chained_householder_trafo; Zygote's broadcast AD of the
// elementwise maps).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <algorithm>
#include <cstring>
#include <initializer_list>
#include <string>
#include <type_traits>
#include <vector>

#include "enf_grad_hj.h"
#include "enf_grad_tail.h"
#include "enf_internal.h"
#include "enf_math64.h"
#include "enf_train.h"

namespace enf {

constexpr int kMaxGradLayers = 16;

struct GradArgs {
  const void* X;
  int64_t N;
  int64_t ldx;
  int32_t D;        // rows of the flow
  int32_t Dp;       // kernel rows: D rounded up to a power of two (padded rows are inert)
  int32_t nsteps;
  int32_t nlayers;
  int32_t nparams;  // gradient entries of this flow
  void* partial;    // [gridDim.x][1 + nparams] of double (loss first)
  LayerDesc layers[kMaxGradLayers];
  int32_t op[kMaxGradSteps];
  int32_t layer[kMaxGradSteps];
  int32_t col[kMaxGradSteps];     // Householder column
  int32_t roff[kMaxGradSteps];    // record offset (elements of T) in LDS
  int32_t goff[kMaxGradSteps];    // gradient offset of the step's first parameter vector
  // enf_flow_vjp only: the cotangents of Y (D x N, ld lddy) and of ladj (length N, may be NULL) and
  // the output dX (D x N, ld lddx)
  const void* dY;
  int64_t lddy;
  const void* dl;
  void* dX;
  int64_t lddx;
  int32_t diag_ts;  // diagnostics build (ENF_SMALL_TS): the one-block step's thread 0 prints its phase clocks
  int32_t zq;       // ENF_NEGLL_ZYGOTE: block 0 adds N sum log|a| of the ScaleShiftTrafos back to the loss
};

// sum_d log|a_d| of the flow's ScaleShiftTrafos (src/scale_shift_trafo.jl:22: over a's own length -- a length-1 a
// broadcast over the rows counts once), this lane's share (d = lane, lane + 64, ...), in double
template <typename T>
__device__ __forceinline__ double scaleshift_ladj_lane(const GradArgs& a, int lane) {
  double s = 0.0;
  for (int l = 0; l < a.nlayers; ++l) {
    if (a.layers[l].op != OP_SCALESHIFT) continue;
    const T* p = (const T*)a.layers[l].p[0];
    const int n = a.layers[l].k == 1 ? 1 : a.D;
    for (int d = lane; d < n; d += 64) s += log(fabs((double)p[d]));
  }
  return s;
}

// values per lane of the generic gradient kernel at kernel rows D: a 16-byte fragment, or D/64 rows
template <typename T>
__host__ __device__ constexpr int grad_lane_values(int D) {
  return D > 64 * (16 / (int)sizeof(T)) ? D / 64 : 16 / (int)sizeof(T);
}

__host__ __device__ constexpr int grad_nparams(int op) {
  return op == OP_HOUSEHOLDER ? 1 : op == OP_SCALESHIFT ? 2 : (op == OP_JOHNSON || op == OP_JOHNSON_INV) ? 4 : 3;
}

typedef unsigned int u32x4g __attribute__((ext_vector_type(4)));

template <int CTRL, typename T>
__device__ __forceinline__ T gdpp(T x) {
  if constexpr (std::is_same_v<T, float>) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  }
}
template <int G, typename T>
__device__ __forceinline__ T gsum(T x) {
  if constexpr (G >= 2) x += gdpp<0xB1>(x);
  if constexpr (G >= 4) x += gdpp<0x4E>(x);
  if constexpr (G >= 8) x += gdpp<0x141>(x);
  if constexpr (G >= 16) x += gdpp<0x140>(x);
  if constexpr (G >= 32) x = add_xor_swap<16>(x);
  if constexpr (G >= 64) x = add_xor_swap<32>(x);
  return x;
}

// Add a per-lane contribution to the wave's double accumulator of row `row`: the lanes holding the
// same row (all column slots of the wave) are summed with cross-lane shuffles first, then one lane
// per row does a plain (non-atomic) read-modify-write -- every address has exactly one writer.
// D >= V (CPF == 1): lanes with equal lane % G share rows; D < V: every lane holds all D rows.
// Round 5: the stages within a 16-lane row are DPP moves (quad_perm xor 1 / xor 2, row_ror 4 / 8 -- shifts by a
// multiple of the class size keep lanes in their class), only the two cross-row stages are ds_bpermute; a
// bpermute round trip is several times a DPP move's latency and the examples' one-block steps are chains of these.
template <int CTRL, typename T>
__device__ __forceinline__ T wdpp(T x) {
  if constexpr (std::is_same_v<T, float>) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, true);
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  }
}
template <int G, int CPF, int SEG, typename T>
__device__ __forceinline__ void wave_accumulate(double* __restrict__ acc, int row, T v, int lane, int nrows) {
  (void)CPF;
  (void)SEG;
  if constexpr (G < 2) v += wdpp<0xB1>(v);   // quad_perm(1,0,3,2): lane ^ 1
  if constexpr (G < 4) v += wdpp<0x4E>(v);   // quad_perm(2,3,0,1): lane ^ 2
  if constexpr (G < 8) v += wdpp<0x124>(v);  // row_ror:4
  if constexpr (G < 16) v += wdpp<0x128>(v); // row_ror:8
  if constexpr (G < 32) v = add_xor_swap<16>(v);
  if constexpr (G < 64) v = add_xor_swap<32>(v);
  if (lane < G && row < nrows) acc[row] += (double)v;  // padded rows (row >= D) have no parameter
}

template <typename T>
__device__ __forceinline__ T sigm(T t) { return (T)1 / ((T)1 + exp(-t)); }

// ---- fp64 in-range forms of the elementwise steps (round 5; VERDICT r04 item 4, the reference examples'
// optimize_whitening steps at D <= 2 are one dependent chain per column through these steps). ocml's fp64 exp /
// log are ~42 / ~98 VALU instructions and a division ~12: the literal CenterContract forward + backward took 8
// exp, 5 log and ~10 divisions per element, the Johnson step two asinh / log1p and ~8 divisions. Here, with the
// row constants the block prologue derives once (rec_extra below) and enf_math64.h's table log / expm1 / div64
// (as the flow kernels' fp64 steps, enf_steps.h): a wave whose elements are all in range (grad_fast_ok, a
// wave vote) takes these forms, any other wave the literal ones (fwd_elem / bwd_elem).
// Row constants after the np parameters (fp64, kernel rows <= 64):
//   ScaleShift   {log|a|, 1/a}
//   Johnson      {1/lambda, 1/delta, log|delta/lambda|}
//   Center*      {exp(b a), exp(-b a), exp(2 b a), 1/b}
__host__ __device__ constexpr int rec_extra(int op) {
  return op == OP_SCALESHIFT ? 2 : op == OP_JOHNSON ? 3 : (op == OP_CENTER_STRETCH || op == OP_CENTER_CONTRACT) ? 4 : 0;
}
constexpr int kFastMaxD = 64;
template <typename T, int D>
__host__ __device__ constexpr bool grad_fast_rows() { return std::is_same_v<T, double> && D <= kFastMaxD; }
// record values per row of a step: the parameters, then (fast rows) the constants
__host__ __device__ constexpr int rec_nparams(int op, bool fast) {
  return (op == OP_HOUSEHOLDER ? 1 : op == OP_SCALESHIFT ? 2 : (op == OP_JOHNSON || op == OP_JOHNSON_INV) ? 4 : 3) +
         (fast ? rec_extra(op) : 0);
}

// the row constants of a step, from its parameters just written to the record r (value q of the row at r[q V]).
// Round 5: on the table log / exp64_in / div64 of the in-range forms where their arguments allow (ocml's exp and log
// otherwise): the ocml forms made this pass ~40 % of the examples' block prologue (profiles/r05/small_ts_v5.txt).
__device__ __forceinline__ double gx_log_abs(double v, const double* __restrict__ tab) {
  const double a = fabs(v);
  return (a >= 1e-300 && a <= 1e300) ? log64_tab(a, 0, tab) : log(a);
}
__device__ __forceinline__ double gx_exp(double w) { return fabs(w) <= 700.0 ? exp64_in(w) : exp(w); }
__device__ __forceinline__ double gx_rcp(double d) {
  return (fabs(d) >= 1e-300 && fabs(d) <= 1e300) ? div64(1.0, d) : 1.0 / d;
}
template <int V>
__device__ __forceinline__ void rec_extra_store(int op, double* r, const double* __restrict__ tab) {
  if (op == OP_SCALESHIFT) {
    const double a = r[0];
    r[2 * V] = gx_log_abs(a, tab);
    r[3 * V] = gx_rcp(a);
  } else if (op == OP_JOHNSON) {
    const double dl = r[V], lm = r[3 * V];
    const double il = gx_rcp(lm);
    r[4 * V] = il;
    r[5 * V] = gx_rcp(dl);
    r[6 * V] = gx_log_abs(dl / lm, tab);
  } else if (op == OP_CENTER_STRETCH || op == OP_CENTER_CONTRACT) {
    const double a = r[0], b = r[V];
    r[3 * V] = gx_exp(b * a);
    r[4 * V] = gx_exp(-b * a);
    r[5 * V] = gx_exp(2.0 * b * a);
    r[6 * V] = gx_rcp(b);
  }
}

__device__ __forceinline__ bool center_moderate(double b, double E1) {
  return fabs(b) >= 1e-100 && fabs(b) <= 1e100 && E1 >= 1e-50 && E1 <= 1e50;
}

// Does the in-range form apply to this element (forward: x the step's input; backward also y its output)?
__device__ __forceinline__ bool grad_fast_ok(int op, double x, double y, const double* p, const double* xr, bool bwd) {
  switch (op) {
    case OP_SCALESHIFT: return true;
    case OP_JOHNSON: {
      // |z| < 2^26 with margin (asinh64_tab_fin), the parameters and their reciprocals normal and finite
      const double zq = (x - p[2]) * xr[0];
      return fabs(zq) < 3.0e7 && fabs(p[3]) >= 1e-300 && fabs(p[3]) <= 1e300 && fabs(p[1]) >= 1e-300 &&
             fabs(p[1]) <= 1e300 && fabs(xr[2]) < 1e300;
    }
    case OP_CENTER_CONTRACT: return center_moderate(p[1], xr[0]) && fabs(p[1] * (x - p[2])) <= 200.0;
    case OP_CENTER_STRETCH:
      return center_moderate(p[1], xr[0]) && fabs(p[1] * x) <= 200.0 && (!bwd || fabs(p[1] * (y - p[2])) <= 200.0);
    default: return false;
  }
}

// the logistic pair of t = b xu, u = |t|: with P = e^u, D1 = P + E1, D2 = 1 + P E1 (E1 = e^(b a)) and ONE
// division, sigmoid(t - b a) and sigmoid(-t - b a) with their complements (s1, 1 - s1, s2, 1 - s2), each a
// product of positive terms (no cancellation): P/D1, E1/D1 and 1/D2, P E1/D2, swapped for t < 0.
struct Logistic2 {
  double s1, c1, s2, c2;
};
__device__ __forceinline__ Logistic2 logistic2(double t, double E1) {
  const double P = 1.0 + expm1_64_in(fabs(t));
  const double D1 = P + E1, D2 = fma(P, E1, 1.0);
  const double rr = div64(1.0, D1 * D2);
  const double sa = P * D2 * rr, ca = E1 * D2 * rr, sb = D1 * rr, cb = P * E1 * D1 * rr;
  const bool neg = t < 0.0;
  return {neg ? sb : sa, neg ? cb : ca, neg ? sa : sb, neg ? ca : cb};
}

// forward of one element, in-range form; adds the ladj term (natural log) to lad. tab: the log table (LDS).
__device__ __forceinline__ double fwd_fast(int op, double x, const double* p, const double* xr, double& lad,
                                           const double* __restrict__ tab) {
  switch (op) {
    case OP_SCALESHIFT: lad += xr[0]; return fma(x, p[0], p[1]);  // scale_shift_trafo.jl:15-22
    case OP_JOHNSON: {  // johnson_trafo.jl:29-32, 39-42
      const double z = div64(x - p[2], p[3]);
      lad += xr[2] - 0.5 * log1p64_tab(z * z, tab);
      return fma(p[1], asinh64_tab_fin(z, tab), p[0]);
    }
    case OP_CENTER_CONTRACT: {  // center_stretch.jl:11-15, 17-22 (enf_steps.h step_center_contract's form)
      const double E1 = xr[0], Ei = xr[1], ib = xr[3];
      const double t = p[1] * (x - p[2]);
      const double em = expm1_64_in(fabs(t));
      const double P = 1.0 + em;
      const double arg = div64(Ei * (em * (2.0 + em)), P + Ei);
      const double pe = fma(P, E1, 1.0), pi = P + E1;
      lad += log64_tab(div64(fma(P, pe, pi), pi * pe), 0, tab);
      return (__builtin_copysign(log1p64_tab(arg, tab), t) + 0.0) * ib;
    }
    default: {  // OP_CENTER_STRETCH, center_stretch.jl:4-8, 41-42 (enf_steps.h step_center_stretch's form)
      const double bv = p[1], c = p[2], E1 = xr[0], E2 = xr[2], ib = xr[3];
      const double ex = exp64_in(fabs(bv * x));
      const double ome = 1.0 - ex;
      const double inner = (sqrt64_ge1(ome * ome * E2 + 4.0 * ex) - ome * E1) / 2.0;
      const double pe = fma(E1, inner, 1.0), ie = inner + E1;
      lad -= log64_tab(div64(fma(inner, pe, ie), ie * pe), 0, tab);
      return fma(__builtin_copysign(log64_tab(inner, 0, tab), x), ib, c);
    }
  }
}

// backward of one element, in-range form (bwd_elem's derivatives): x the step's input, y its output (the next
// step's stored input, or the flow's output), g = dS/dy, cl = dS/dladj; adds dS/dparam into dp, returns dS/dx
__device__ __forceinline__ double bwd_fast(int op, double x, double y, double g, const double* p, const double* xr,
                                           double* dp, double cl, const double* __restrict__ tab) {
  switch (op) {
    case OP_SCALESHIFT:
      dp[0] += g * x + cl * xr[1];
      dp[1] += g;
      return g * p[0];
    case OP_JOHNSON: {
      const double dl = p[1], il = xr[0];
      const double z = div64(x - p[2], p[3]);
      const double s2 = fma(z, z, 1.0);
      double rs = __builtin_amdgcn_rsq(s2);  // 1/sqrt(1 + z^2): seed + two Newton steps
      rs = fma(0.5 * rs, fma(-s2 * rs, rs, 1.0), rs);
      rs = fma(0.5 * rs, fma(-s2 * rs, rs, 1.0), rs);
      const double A = dl * il * rs;       // dl / (lm s)
      const double Bc = z * il * rs * rs;  // z / (lm s2)
      dp[0] += g;
      dp[1] += fma(g, asinh64_tab_fin(z, tab), cl * xr[1]);
      dp[2] += -g * A + cl * Bc;
      dp[3] += (-g * A * z - cl * il) + cl * (Bc * z);
      return g * A - cl * Bc;
    }
    case OP_CENTER_CONTRACT: {
      const double a = p[0], b = p[1], xu = x - p[2], ib = xr[3];
      const Logistic2 L = logistic2(b * xu, xr[0]);
      const double ss = L.s1 + L.s2, iss = div64(1.0, ss);
      const double q1 = L.s1 * L.c1, q2 = L.s2 * L.c2;
      const double dyda = L.s2 - L.s1, dydb = (L.s1 * (xu - a) + L.s2 * (xu + a) - y) * ib;
      const double dldx = (q1 * b - q2 * b) * iss, dlda = -(q1 + q2) * b * iss, dldb = (q1 * (xu - a) - q2 * (xu + a)) * iss;
      dp[0] += g * dyda + cl * dlda;
      dp[1] += g * dydb + cl * dldb;
      dp[2] += -(g * ss + cl * dldx);
      return g * ss + cl * dldx;
    }
    default: {  // OP_CENTER_STRETCH: y = cs(x) = s(x) + c and cc(y) = f(y - c) = x (bwd_elem's derivation, its ccv = x)
      const double a = p[0], b = p[1], c = p[2], ib = xr[3];
      const double yu = y - c;
      const Logistic2 L = logistic2(b * yu, xr[0]);
      const double ss = L.s1 + L.s2, iss = div64(1.0, ss);
      const double q1 = L.s1 * L.c1, q2 = L.s2 * L.c2;
      const double cc_a = L.s2 - L.s1, cc_b = (L.s1 * (yu - a) + L.s2 * (yu + a) - x) * ib;
      const double lcc_y = (q1 * b - q2 * b) * iss, lcc_a = -(q1 + q2) * b * iss,
                   lcc_b = (q1 * (yu - a) - q2 * (yu + a)) * iss;
      const double dyda = -cc_a * iss, dydb = -cc_b * iss;
      const double dlda = -(lcc_y * dyda + lcc_a), dldb = -(lcc_y * dydb + lcc_b);
      dp[0] += g * dyda + cl * dlda;
      dp[1] += g * dydb + cl * dldb;
      dp[2] += g;  // dy/dc = 1, dl/dc = 0
      return g * iss - cl * (lcc_y * iss);
    }
  }
}

// Per-element forward of one step (accurate form). Returns the output; adds the element's ladj
// term (natural log) to lad.
template <typename T>
__device__ __forceinline__ T fwd_elem(int op, T x, const T* p, T& lad) {
  switch (op) {
    case OP_SCALESHIFT: lad += log(fabs(p[0])); return fma(x, p[0], p[1]);
    case OP_JOHNSON: {
      const T z = (x - p[2]) / p[3];
      lad += log(fabs(p[1] / p[3])) - (T)0.5 * log1p(z * z);
      return p[0] + p[1] * asinh(z);
    }
    case OP_JOHNSON_INV: {
      const T w = (x - p[0]) / p[1];
      const T y = p[3] * sinh(w) + p[2];
      const T z = (y - p[2]) / p[3];
      lad -= log(fabs(p[1] / p[3])) - (T)0.5 * log1p(z * z);
      return y;
    }
    case OP_CENTER_CONTRACT: {
      const T a = p[0], b = p[1], xu = x - p[2];
      lad += log(fabs(sigm(b * (xu - a)) + sigm(-b * (xu + a))));
      return (log1p(exp(b * (xu - a))) - log1p(exp(-b * (xu + a)))) / b;
    }
    case OP_CENTER_STRETCH: {
      const T a = p[0], b = p[1], c = p[2];
      const T e = exp(fabs(b * x));
      const T ome = (T)1 - e;
      const T inner = (sqrt(ome * ome * exp((T)2 * b * a) + (T)4 * e) - ome * exp(b * a)) / (T)2;
      const T sg = x > (T)0 ? (T)1 : (x < (T)0 ? (T)-1 : x);
      const T y = sg * log(inner) / b + c;
      const T yu = y - c;
      lad -= log(fabs(sigm(b * (yu - a)) + sigm(-b * (yu + a))));
      return y;
    }
    default: return x;
  }
}

// Backward of one elementwise step for one element: input x, output cotangent g (dS/dy), ladj
// cotangent cl (dS/dladj: -1 for the loss S, which contains -ladj). Adds dS/dparam into dp[0..np)
// and returns dS/dx. The negll kernel passes the literal cl = -1, for which every "+ cl*t" /
// "- cl*t" below is exactly the subtraction / addition of t.
template <typename T>
__device__ __forceinline__ T bwd_elem(int op, T x, T g, const T* p, T* dp, T cl) {
  switch (op) {
    case OP_SCALESHIFT: {  // y = x a + b ; l = log|a|
      dp[0] += g * x + cl * ((T)1 / p[0]);
      dp[1] += g;
      return g * p[0];
    }
    case OP_JOHNSON: {  // y = gm + dl*asinh(z), z = (x - xi)/lm ; l = log|dl/lm| - log(1+z^2)/2
      const T dl = p[1], lm = p[3];
      const T z = (x - p[2]) / lm;
      const T s2 = (T)1 + z * z, s = sqrt(s2);
      dp[0] += g;
      dp[1] += g * asinh(z) + cl * ((T)1 / dl);
      dp[2] += -g * dl / (lm * s) + cl * (z / (lm * s2));
      dp[3] += (-g * dl * z / (lm * s) - cl * ((T)1 / lm)) + cl * (z * z / (lm * s2));
      return g * dl / (lm * s) - cl * (z / (lm * s2));
    }
    case OP_JOHNSON_INV: {  // y = lm*sinh(w) + xi, w = (x - gm)/dl ; l = log|lm/dl| + log cosh w
      const T dl = p[1], lm = p[3];
      const T w = (x - p[0]) / dl;
      const T ch = cosh(w), th = tanh(w);
      dp[0] += -g * lm * ch / dl - cl * (th / dl);
      dp[1] += (-g * lm * ch * w / dl - cl * ((T)1 / dl)) - cl * (th * w / dl);
      dp[2] += g;
      dp[3] += g * sinh(w) + cl * ((T)1 / lm);
      return g * lm * ch / dl + cl * (th / dl);
    }
    case OP_CENTER_CONTRACT: {
      // y = (softplus(t1) - softplus(t2))/b, t1 = b(xu - a), t2 = -b(xu + a), xu = x - c
      // l = log(s1 + s2), s_i = sigmoid(t_i); dy/dx = s1 + s2
      const T a = p[0], b = p[1], xu = x - p[2];
      const T t1 = b * (xu - a), t2 = -b * (xu + a);
      const T s1 = sigm(t1), s2 = sigm(t2), ss = s1 + s2;
      const T y = (log1p(exp(t1)) - log1p(exp(t2))) / b;
      const T q1 = s1 * ((T)1 - s1), q2 = s2 * ((T)1 - s2);
      const T dydx = ss, dyda = s2 - s1, dydb = (s1 * (xu - a) + s2 * (xu + a)) / b - y / b;
      const T dldx = (q1 * b - q2 * b) / ss, dlda = -(q1 + q2) * b / ss, dldb = (q1 * (xu - a) - q2 * (xu + a)) / ss;
      dp[0] += g * dyda + cl * dlda;
      dp[1] += g * dydb + cl * dldb;
      dp[2] += -(g * dydx + cl * dldx);  // d/dc = -d/dx
      return g * dydx + cl * dldx;
    }
    case OP_CENTER_STRETCH: {
      // y = cs(x) with cc(y) = x: dy/dx = 1/cc'(y), dy/dth = -dcc/dth(y)/cc'(y);
      // l = -lcc(y): dl/dth = -(dlcc/dy dy/dth + dlcc/dth), dl/dx = -dlcc/dy dy/dx
      const T a = p[0], b = p[1], c = p[2];
      T lad = 0;
      const T y = fwd_elem<T>(OP_CENTER_STRETCH, x, p, lad);
      const T yu = y - c;
      const T t1 = b * (yu - a), t2 = -b * (yu + a);
      const T s1 = sigm(t1), s2 = sigm(t2), ss = s1 + s2;
      const T ccv = (log1p(exp(t1)) - log1p(exp(t2))) / b;  // = x (up to rounding)
      const T q1 = s1 * ((T)1 - s1), q2 = s2 * ((T)1 - s2);
      const T cc_a = s2 - s1, cc_b = (s1 * (yu - a) + s2 * (yu + a)) / b - ccv / b, cc_c = -ss;
      const T lcc_y = (q1 * b - q2 * b) / ss, lcc_a = -(q1 + q2) * b / ss, lcc_b = (q1 * (yu - a) - q2 * (yu + a)) / ss,
              lcc_c = -lcc_y;
      const T dydx = (T)1 / ss;
      const T dyda = -cc_a / ss, dydb = -cc_b / ss, dydc = -cc_c / ss;
      const T dlda = -(lcc_y * dyda + lcc_a), dldb = -(lcc_y * dydb + lcc_b), dldc = -(lcc_y * dydc + lcc_c);
      const T dldx = -lcc_y * dydx;
      dp[0] += g * dyda + cl * dlda;
      dp[1] += g * dydb + cl * dldb;
      dp[2] += g * dydc + cl * dldc;
      return g * dydx + cl * dldx;
    }
    default: return g;
  }
}

// The in-range forms of one step over the lane's V values (FAST rows): loads the step's records with compile-time
// offsets, votes over the wave, and returns false (nothing done) when some element is out of range.
template <int OP, int V>
__device__ __forceinline__ void fast_rec(const double* __restrict__ r, int e, double (&p)[4], double (&xr)[4]) {
  constexpr int np = grad_nparams(OP), nx = rec_extra(OP);
#pragma unroll
  for (int q = 0; q < 4; ++q) p[q] = q < np ? r[q * V + e] : 0.0;
#pragma unroll
  for (int q = 0; q < 4; ++q) xr[q] = q < nx ? r[(np + q) * V + e] : 0.0;
}

template <int OP, int V, int SEG, int CPF>
__device__ __forceinline__ bool fwd_fast_step(double (&x)[V], double (&lad)[CPF], const double* __restrict__ r, bool ss1,
                                              int r0, const double* __restrict__ tab) {
  bool ok = true;
#pragma unroll
  for (int e = 0; e < V; ++e) {
    double p[4], xr[4];
    fast_rec<OP, V>(r, e, p, xr);
    ok = ok && grad_fast_ok(OP, x[e], 0.0, p, xr, false);
  }
  if (!__all(ok)) return false;
#pragma unroll
  for (int e = 0; e < V; ++e) {
    double p[4], xr[4];
    fast_rec<OP, V>(r, e, p, xr);
    double l = 0.0;
    x[e] = fwd_fast(OP, x[e], p, xr, l, tab);
    if (!ss1 || r0 + e % SEG == 0) lad[e / SEG] += l;
  }
  return true;
}

template <int OP, int V, int SEG, int G, int CPF>
__device__ __forceinline__ bool bwd_fast_step(const double (&xin)[V], const double (&yout)[V], double (&g)[V],
                                              const bool (&valid)[V], const double (&clv)[V], const double* __restrict__ r,
                                              double* __restrict__ gacc, int r0, int lane, int Dr,
                                              const double* __restrict__ tab) {
  constexpr int np = grad_nparams(OP);
  bool ok = true;
#pragma unroll
  for (int e = 0; e < V; ++e) {
    double p[4], xr[4];
    fast_rec<OP, V>(r, e, p, xr);
    ok = ok && grad_fast_ok(OP, xin[e], yout[e], p, xr, true);
  }
  if (!__all(ok)) return false;
  // the lane's contributions per (parameter, row): its CPF columns summed in the lane first, then one wave sum each
  double dsum[4][SEG];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int k = 0; k < SEG; ++k) dsum[q][k] = 0.0;
#pragma unroll
  for (int e = 0; e < V; ++e) {
    double p[4], xr[4], dp[4] = {0, 0, 0, 0};
    fast_rec<OP, V>(r, e, p, xr);
    const double gx = bwd_fast(OP, xin[e], yout[e], g[e], p, xr, dp, clv[e], tab);
#pragma unroll
    for (int q = 0; q < np; ++q) dsum[q][e % SEG] += valid[e] ? dp[q] : 0.0;
    g[e] = valid[e] ? gx : 0.0;
  }
#pragma unroll
  for (int q = 0; q < np; ++q)
#pragma unroll
    for (int k = 0; k < SEG; ++k) wave_accumulate<G, CPF, SEG>(gacc + q * Dr, r0 + k, dsum[q][k], lane, Dr);
  return true;
}

// STEP (round 5): the single-block fused optimize_whitening step -- the grid is one block, and instead of writing
// its partial row the block sums its waves into LDS and runs the update itself (block_step_update): one launch per
// minibatch step where the two-launch path costs two kernel boundaries (the examples' B = 100 / 1000 steps).
// VL (round 5): values per lane other than the default -- VL = 1 for fp64 D = 2 batches of at most 256 columns (the
// 2-D example's B = 100): one row per lane, so a column's two elements run on two lanes instead of one after the
// other in a single lane, and the batch's one block has twice the waves (make_plan grad_vl).
// A compiled step sequence (round 5): the op of every step known at compile time, so the step loops unroll, each
// step's op-dependent code is selected at compile time and its descriptors (offsets, parameter pointers) are loaded
// once instead of per step. OpProg<> is the step-table interpreter (ops read from GradArgs at run time). Used for the
// reference examples' flows at their dimension (make_plan grad_prog).
template <int... Ops>
struct OpProg {
  static constexpr int n = (int)sizeof...(Ops);
  __host__ __device__ static constexpr int at(int s) {
    constexpr int ops[] = {Ops..., -1};
    return ops[s];
  }
};
using ProgInterp = OpProg<>;
using ProgExample1d = OpProg<OP_CENTER_CONTRACT, OP_JOHNSON, OP_CENTER_CONTRACT, OP_JOHNSON>;  // nf_example_1d.jl:23-24
using ProgExample2d = OpProg<OP_SCALESHIFT, OP_HOUSEHOLDER, OP_CENTER_CONTRACT>;                // nf_example_2d.jl:25-27
// parameter items (step, parameter vector) of a compiled program
template <class Prog>
__host__ __device__ constexpr int prog_items() {
  int n = 0;
  for (int s = 0; s < Prog::n; ++s) n += grad_nparams(Prog::at(s));
  return n;
}

// The minibatch a launch of negll_grad_impl processes: its columns (X, N) and, for the one-block step, where its
// loss goes and its ADAGrad gradient scale 1/B (the GradArgs / StepArgs values, or the epoch kernel's j-th batch).
struct BatchCtx {
  const void* X;
  int64_t N;
  double* loss_out;
  int64_t nsamp;
  double scale;
  bool fill_ltab;  // false: the table log is already in LDS (the epoch kernel's steps after its first)
};

template <typename T, int D, bool VJP, bool STEP = false, int VL = 0, class Prog = ProgInterp>
__device__ __forceinline__ void negll_grad_impl(const GradArgs& a, const ReduceArgs* rs, const StepArgs* ss,
                                                const BatchCtx& bc) {
  // values per lane: one 16-byte fragment, or D/64 rows when a column needs more than 64 fragments (round 4:
  // kernel rows up to 1024, a column then spans the whole wave)
  constexpr int V = VL ? VL : grad_lane_values<T>(D);
  constexpr int G = D >= V ? D / V : 1;
  constexpr int CPF = D >= V ? 1 : V / D;
  constexpr int SEG = D >= V ? V : D;
  constexpr int COLS = 64 / G * CPF;  // columns per wave tile (one fragment per lane)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // LDS: [grad accumulators: nw waves x nparams doubles][loss: nw (<= 8) waves x double][records][activations]
  // (nw = blockDim.x / 64: 4, fewer when D > 64 makes the per-wave accumulators large, 8 for a one-block batch)
  const int nw = blockDim.x >> 6;
  const int gbytes = ((a.nparams * 8 + 15) / 16) * 16;
  double* gacc = reinterpret_cast<double*>(smem + (threadIdx.x >> 6) * gbytes);  // this wave's
  double* lossw = reinterpret_cast<double*>(smem + nw * gbytes);
  T* rec = reinterpret_cast<T*>(smem + nw * gbytes + 64);
  constexpr bool FAST = grad_fast_rows<T, D>();  // (fp64, D <= 64: the row constants of rec_extra are recorded)
  int nrec = 0;
  for (int s = 0; s < a.nsteps; ++s) nrec += rec_nparams(a.op[s], FAST) * (D > V ? D : V);
  T* act = rec + ((nrec + 3) / 4) * 4 + (threadIdx.x >> 6) * (a.nsteps * 64 * V);
  // the table log of the in-range forms (after the activations of the block's waves)
  double* ltab = reinterpret_cast<double*>(rec + ((nrec + 3) / 4) * 4 + nw * (a.nsteps * 64 * V));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#if ENF_DIAG
  const long long ts0 = STEP && a.diag_ts ? (long long)clock64() : 0;
#endif
  for (int i = lane; i < a.nparams; i += 64) gacc[i] = 0.0;
  if constexpr (FAST)
    if (bc.fill_ltab)
      for (int i = tid; i < 3 * kLogTabN; i += blockDim.x) ltab[i] = kLogTab[i];
  // Records, layout [group][param][element] as the forward kernel (RV = V), in three passes (round 5: ONE round of
  // global loads, where the step-by-step loop waited for each step's parameters, and each thread of a reflection
  // loaded the whole column for its v'v):
  //   (A) every raw parameter value of every step: one (step, parameter) pair per wave at a time, lanes on the
  //       entries, up to four pairs per wave loaded before any is stored (a larger flow loops);
  //   (B) the reflections' v'v in double, one wave per Householder step (its lanes, then the xor tree);
  //   (C) vh = v sqrt(2/v'v) (householder_trafo.jl:9-10) and, FAST, the row constants (rec_extra).
  const int nent = D > V ? D : V;
  // the raw value of parameter q of entry i of step s, and its record index (s and q wave-uniform: the parameter
  // pointer is a scalar)
  auto raw_item = [&](int s, int i, int q, T& v) -> int {
    const int op = a.op[s], rn = rec_nparams(op, FAST);
    const int g = D >= V ? i / V : 0, e = i % V;
    const int row = D >= V ? i : e % D;
    if (row >= a.D) {
      // padded row (D not a power of two): parameters that map 0 to 0 with ladj 0 (ScaleShift
      // a = 1, b = 0; Johnson gamma = xi = 0, delta = lambda = 1; Center a = c = 0, b = 1;
      // reflection 0), so padded rows stay 0 and add nothing to the loss or the gradients
      v = op == OP_HOUSEHOLDER ? (T)0
          : op == OP_SCALESHIFT ? (q == 0 ? (T)1 : (T)0)
          : (op == OP_JOHNSON || op == OP_JOHNSON_INV) ? ((q == 1 || q == 3) ? (T)1 : (T)0)
          : (q == 1 ? (T)1 : (T)0);
    } else if (op == OP_HOUSEHOLDER) {
      v = ((const T*)a.layers[a.layer[s]].p[0])[(int64_t)a.col[s] * a.D + row];
    } else {
      v = ((const T*)a.layers[a.layer[s]].p[q])[row];
    }
    return a.roff[s] + (g * rn + q) * V + e;
  };
  // (A) item j = the j-th (step, parameter) pair: wave w takes items w, w + nw, ... with its lanes on the entries;
  // up to four items per wave are loaded before any is stored. A compiled program (one step per layer, column 0)
  // knows every item's step and parameter at compile time: its loads are independent (one scalar load of the
  // parameter pointer each, no walk over the step table and no layer indirection) and all are in flight before
  // the first store.
  if constexpr (Prog::n > 0) {
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    constexpr int NI = prog_items<Prog>();
    T vb[NI];
    int ib[NI];
    int j = 0;
#pragma unroll
    for (int s = 0; s < Prog::n; ++s) {
      const int op = Prog::at(s), rn = rec_nparams(op, FAST);
#pragma unroll
      for (int q = 0; q < grad_nparams(op); ++q, ++j) {
        ib[j] = -1;
        if (j % nw == wv && lane < nent) {
          const int g = D >= V ? lane / V : 0, e = lane % V;
          const int row = D >= V ? lane : e % D;
          vb[j] = ((const T*)a.layers[s].p[op == OP_HOUSEHOLDER ? 0 : q])[row];
          ib[j] = a.roff[s] + (g * rn + q) * V + e;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NI; ++k)
      if (ib[k] >= 0) rec[ib[k]] = vb[k];
  } else {
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    int nitems = 0;
    for (int s = 0; s < a.nsteps; ++s) nitems += grad_nparams(a.op[s]);
    if (nent <= 64 && nitems <= 4 * nw) {
      T vb[4];
      int ib[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        ib[m] = -1;
        const int j = wv + m * nw;
        if (j < nitems) {
          int s = 0, q = j;
          while (q >= grad_nparams(a.op[s])) {
            q -= grad_nparams(a.op[s]);
            ++s;
          }
          if (lane < nent) ib[m] = raw_item(s, lane, q, vb[m]);
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
        if (ib[m] >= 0) rec[ib[m]] = vb[m];
    } else {
      int j = 0;
      for (int s = 0; s < a.nsteps; ++s)
        for (int q = 0; q < grad_nparams(a.op[s]); ++q, ++j) {
          if (j % nw != wv) continue;
          for (int i = lane; i < nent; i += 64) {
            T v;
            const int ix = raw_item(s, i, q, v);
            rec[ix] = v;
          }
        }
    }
  }
  __syncthreads();
#if ENF_DIAG
  const long long tsA = STEP && a.diag_ts ? (long long)clock64() : 0;
#endif
  // (B) one step per wave (its op wave-uniform, so no lane runs another op's branch): a reflection's v'v in double
  // over its lanes, then vh = v sqrt(2/v'v) (householder_trafo.jl:9-10) written by the same wave; FAST, the other
  // steps' row constants (rec_extra) -- the reflections' chains and the exp / log chains run side by side, one
  // barrier for both
  // ENF_NEGLL_ZYGOTE: the reference's recorded loss (its ScaleShiftTrafo primal ladj is zero under Zygote,
  // src/abstract_trafo.jl:30-33): block 0 adds N sum log|a| back, at the parameters this step read. FAST, the wave
  // that writes a ScaleShift step's row constants sums the log|a| it just stored (the value the forward adds) and
  // adds it to its own loss partial; otherwise wave 0 sums them from the parameters in global memory
  double zq_lane = 0.0;
  auto step_consts = [&](const int s, const int op) {
    const int rn = rec_nparams(op, FAST);
    if (op == OP_HOUSEHOLDER) {
      double vv = 0.0;
      for (int d = lane; d < a.D; d += 64) {
        const int g = D >= V ? d / V : 0, e = D >= V ? d % V : d;  // (D < V: entry d holds row d)
        const double v = (double)rec[a.roff[s] + g * rn * V + e];
        vv += v * v;
      }
      vv = lane_sum(vv, a.D);
      // lane 0's sum for every lane (lane_sum leaves it in lanes < D; D < V has entries past D)
      const uint64_t vb = __builtin_bit_cast(uint64_t, vv);
      vv = __builtin_bit_cast(double, ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(vb >> 32)) << 32) |
                                          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)vb));
      const double hs = sqrt(2.0 / vv);
      for (int i = lane; i < nent; i += 64) {
        T* r = rec + a.roff[s] + (D >= V ? i / V : 0) * rn * V + i % V;
        r[0] = (T)((double)r[0] * hs);
      }
    } else if constexpr (FAST) {
      if (rec_extra(op) > 0)
        for (int i = lane; i < nent; i += 64)
          rec_extra_store<V>(op, (double*)(rec + a.roff[s] + (D >= V ? i / V : 0) * rn * V + i % V), ltab);
      if (op == OP_SCALESHIFT && a.zq && blockIdx.x == 0) {
        const int n = a.layers[a.layer[s]].k == 1 ? 1 : a.D;  // (a length-1 a counts once)
        for (int d = lane; d < n; d += 64)  // (the entries this lane just stored)
          zq_lane += (double)rec[a.roff[s] + (D >= V ? d / V : 0) * rn * V + d % V + 2 * V];
      }
    }
  };
  {
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    if constexpr (Prog::n > 0) {
#pragma unroll
      for (int s = 0; s < Prog::n; ++s)
        if (s % nw == wv) step_consts(s, Prog::at(s));
    } else {
      for (int s = wv; s < a.nsteps; s += nw) step_consts(s, a.op[s]);
    }
  }
  __syncthreads();
#if ENF_DIAG
  const long long tsB = tsA;
#endif
#if ENF_DIAG
  const long long ts1 = STEP && a.diag_ts ? (long long)clock64() : 0;
#endif

  // the one-block step: the update's own loads (theta, ADAGrad state, Householder columns) issued now, consumed after
  // the tiles (block_step_update)
  StepPre<T> pre;
  bool have_pre = false;
  if constexpr (STEP) {
    have_pre = a.nparams <= (int)blockDim.x;
    if (have_pre && tid < a.nparams) pre = step_prefetch<T>(tid, a.D, *rs, *ss);
  }
  const int r0 = D >= V ? V * (lane % G) : 0;
  const int grp = D >= V ? lane % G : 0;
  const int64_t ntiles = (bc.N + COLS - 1) / COLS;
  // (the ENF_NEGLL_ZYGOTE sum without the FAST records: started here, so its loads and logs overlap the tiles)
  if constexpr (!FAST)
    if (a.zq && blockIdx.x == 0 && wave == 0) zq_lane = scaleshift_ladj_lane<T>(a, lane);
  double lossp = 0.0;
#if ENF_DIAG
  long long tsF = 0, tsL = 0;  // the first tile's forward end and loss end (diagnostics)
#endif
  for (int64_t t = (int64_t)blockIdx.x * nw + wave; t < ntiles; t += (int64_t)gridDim.x * nw) {
    const int64_t c0 = t * COLS + (lane / G) * CPF;
    T x[V];
    bool valid[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int64_t c = c0 + e / SEG;
      valid[e] = c < bc.N;
      x[e] = (valid[e] && r0 + e % SEG < a.D) ? ((const T*)bc.X)[c * a.ldx + r0 + e % SEG] : (T)0;
    }
    // ---- forward, storing each step's input
    T lad[CPF];
#pragma unroll
    for (int c = 0; c < CPF; ++c) lad[c] = (T)0;
    auto fwd_step = [&](const int s, const int op) {
      T* as = act + s * 64 * V + lane * V;
#pragma unroll
      for (int e = 0; e < V; ++e) as[e] = x[e];
      const T* r = rec + a.roff[s] + grp * rec_nparams(op, FAST) * V;
      if (op == OP_HOUSEHOLDER) {
#pragma unroll
        for (int c = 0; c < CPF; ++c) {
          T dot = 0;
#pragma unroll
          for (int e = 0; e < SEG; ++e) dot = fma(r[c * SEG + e], x[c * SEG + e], dot);
          dot = gsum<G>(dot);
#pragma unroll
          for (int e = 0; e < SEG; ++e) x[c * SEG + e] = fma(-dot, r[c * SEG + e], x[c * SEG + e]);
        }
      } else {
        const int np = grad_nparams(op);
        // ScaleShiftTrafo with a length-1 `a` (layer k = 1): its ladj constant log|a| counts once, on row 0
        // (scale_shift_trafo.jl:22 sums over a's own length)
        const bool ss1 = op == OP_SCALESHIFT && a.layers[a.layer[s]].k == 1;
        bool done = false;
        if constexpr (FAST) {
          switch (op) {
            case OP_SCALESHIFT: done = fwd_fast_step<OP_SCALESHIFT, V, SEG, CPF>(x, lad, r, ss1, r0, ltab); break;
            case OP_JOHNSON: done = fwd_fast_step<OP_JOHNSON, V, SEG, CPF>(x, lad, r, ss1, r0, ltab); break;
            case OP_CENTER_CONTRACT: done = fwd_fast_step<OP_CENTER_CONTRACT, V, SEG, CPF>(x, lad, r, ss1, r0, ltab); break;
            case OP_CENTER_STRETCH: done = fwd_fast_step<OP_CENTER_STRETCH, V, SEG, CPF>(x, lad, r, ss1, r0, ltab); break;
            default: break;
          }
        }
        if (!done) {
#pragma unroll
          for (int e = 0; e < V; ++e) {
            T p[4];
            for (int q = 0; q < np; ++q) p[q] = r[q * V + e];
            T l = 0;
            x[e] = fwd_elem<T>(op, x[e], p, l);
            if (!ss1 || r0 + e % SEG == 0) lad[e / SEG] += l;
          }
        }
      }
    };
    if constexpr (Prog::n > 0) {
#pragma unroll
      for (int s = 0; s < Prog::n; ++s) fwd_step(s, Prog::at(s));
    } else {
      for (int s = 0; s < a.nsteps; ++s) fwd_step(s, a.op[s]);
    }
#if ENF_DIAG
    if (STEP && a.diag_ts && !tsF) tsF = (long long)clock64();
#endif
    T yfin[V];  // the flow's output (the last step's output for the backward's in-range forms)
#pragma unroll
    for (int e = 0; e < V; ++e) yfin[e] = x[e];
    // ---- loss: sum_d (y^2 + log 2pi)/2 - ladj (only valid columns)
    if constexpr (!VJP) {
      T part = 0;
#pragma unroll
      for (int e = 0; e < V; ++e)
        if (valid[e] && r0 + e % SEG < a.D) part += (x[e] * x[e] + (T)1.8378770664093454836) / (T)2;
#pragma unroll
      for (int c = 0; c < CPF; ++c) {
        const T tot = gsum<G>(lad[c]);  // all lanes active (DPP)
        if (valid[c * SEG] && (lane % G) == 0) part -= tot;
      }
      lossp += (double)part;
    }
#if ENF_DIAG
    if (STEP && a.diag_ts && !tsL) tsL = (long long)clock64();
#endif
    // ---- backward: g = dS/dy = y (invalid columns carry g = 0 and contribute nothing); VJP: g = dY,
    // the ladj cotangent of each column dladj (0 when absent)
    T g[V], cl[CPF];
    if constexpr (VJP) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const int64_t c = c0 + e / SEG;
        g[e] = (valid[e] && r0 + e % SEG < a.D) ? ((const T*)a.dY)[c * a.lddy + r0 + e % SEG] : (T)0;
      }
#pragma unroll
      for (int c = 0; c < CPF; ++c) cl[c] = (valid[c * SEG] && a.dl) ? ((const T*)a.dl)[c0 + c] : (T)0;
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) g[e] = valid[e] ? x[e] : (T)0;
    }
    const int nst = Prog::n > 0 ? Prog::n : a.nsteps;
    auto bwd_step = [&](const int s, const int op) {
      const T* as = act + s * 64 * V + lane * V;
      T xin[V];
#pragma unroll
      for (int e = 0; e < V; ++e) xin[e] = as[e];
      const int np = grad_nparams(op);
      const T* r = rec + a.roff[s] + grp * rec_nparams(op, FAST) * V;
      if (op == OP_HOUSEHOLDER) {
        // y = x - vh (vh'x): dS/dx = g - vh (vh'g); with w = vh/sqrt2 (unit), the direction
        // gradient dS/dw_d = -2 (g_d (w'x) + x_d (w'g)) = -sqrt2 (g_d (vh'x) + x_d (vh'g)); the
        // projection onto v (householder_trafo.jl:32,39) is applied after the sample sum.
#pragma unroll
        for (int c = 0; c < CPF; ++c) {
          T vx = 0, vg = 0;
#pragma unroll
          for (int e = 0; e < SEG; ++e) {
            vx = fma(r[c * SEG + e], xin[c * SEG + e], vx);
            vg = fma(r[c * SEG + e], g[c * SEG + e], vg);
          }
          vx = gsum<G>(vx);
          vg = gsum<G>(vg);
#pragma unroll
          for (int e = 0; e < SEG; ++e) {
            const T contrib = valid[c * SEG + e] ? g[c * SEG + e] * vx + xin[c * SEG + e] * vg : (T)0;
            wave_accumulate<G, CPF, SEG>(gacc + a.goff[s], r0 + e, contrib, lane, a.D);
            g[c * SEG + e] = fma(-vg, r[c * SEG + e], g[c * SEG + e]);
          }
        }
      } else {
        const bool ss1 = op == OP_SCALESHIFT && a.layers[a.layer[s]].k == 1;
        // the step's output: the next step's stored input, or the flow's output
        T yout[V];
        {
          const T* an = act + (s + 1) * 64 * V + lane * V;
#pragma unroll
          for (int e = 0; e < V; ++e) yout[e] = s + 1 < nst ? an[e] : yfin[e];
        }
        bool done = false;
        if constexpr (FAST) {
          double clv[V];
#pragma unroll
          for (int e = 0; e < V; ++e) clv[e] = (ss1 && r0 + e % SEG != 0) ? 0.0 : (VJP ? (double)cl[e / SEG] : -1.0);
          double* ga = gacc + a.goff[s];
          switch (op) {
            case OP_SCALESHIFT:
              done = bwd_fast_step<OP_SCALESHIFT, V, SEG, G, CPF>(xin, yout, g, valid, clv, r, ga, r0, lane, a.D, ltab);
              break;
            case OP_JOHNSON:
              done = bwd_fast_step<OP_JOHNSON, V, SEG, G, CPF>(xin, yout, g, valid, clv, r, ga, r0, lane, a.D, ltab);
              break;
            case OP_CENTER_CONTRACT:
              done = bwd_fast_step<OP_CENTER_CONTRACT, V, SEG, G, CPF>(xin, yout, g, valid, clv, r, ga, r0, lane, a.D, ltab);
              break;
            case OP_CENTER_STRETCH:
              done = bwd_fast_step<OP_CENTER_STRETCH, V, SEG, G, CPF>(xin, yout, g, valid, clv, r, ga, r0, lane, a.D, ltab);
              break;
            default: break;
          }
        }
        if (!done) {
#pragma unroll
          for (int e = 0; e < V; ++e) {
            T p[4], dp[4] = {0, 0, 0, 0};
            for (int q = 0; q < np; ++q) p[q] = r[q * V + e];
            const int row = r0 + e % SEG;
            // (ScaleShift's ladj cotangent only reaches its ladj term, which a length-1 `a` has on row 0 only)
            const T clw = (ss1 && row != 0) ? (T)0 : (VJP ? cl[e / SEG] : (T)-1);
            const T gx = bwd_elem<T>(op, xin[e], g[e], p, dp, clw);
            for (int q = 0; q < np; ++q)
              wave_accumulate<G, CPF, SEG>(gacc + a.goff[s] + q * a.D, row, valid[e] ? dp[q] : (T)0, lane, a.D);
            g[e] = valid[e] ? gx : (T)0;
          }
        }
      }
    };
    if constexpr (Prog::n > 0) {
#pragma unroll
      for (int s = Prog::n - 1; s >= 0; --s) bwd_step(s, Prog::at(s));
    } else {
      for (int s = a.nsteps - 1; s >= 0; --s) bwd_step(s, a.op[s]);
    }
    if constexpr (VJP) {  // dX = the cotangent after the first step
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const int64_t c = c0 + e / SEG;
        if (valid[e] && r0 + e % SEG < a.D) ((T*)a.dX)[c * a.lddx + r0 + e % SEG] = g[e];
      }
    }
  }
  // ---- block partials
#if ENF_DIAG
  const long long ts2 = STEP && a.diag_ts ? (long long)clock64() : 0;
#endif
  lossp = fma(zq_lane, (double)bc.N, lossp);
  lossp = xor_tree(lossp, 64);  // (the 64-lane xor butterfly)
  if (lane == 0) lossw[wave] = lossp;
  __syncthreads();
  if constexpr (STEP) {
    // the block's row into LDS past the activations (the same sums as the row below), then the update
    const size_t act_end = reinterpret_cast<size_t>(ltab + (FAST ? 3 * kLogTabN : 0));
    double* tot = reinterpret_cast<double*>((act_end + 15) / 16 * 16);
    unsigned char* scratch = reinterpret_cast<unsigned char*>(tot + ((1 + a.nparams + 1) / 2) * 2);
    if (tid == 0) {
      double l = lossw[0];
      for (int w = 1; w < nw; ++w) l += lossw[w];
      tot[0] = l;
    }
    const double* g0 = reinterpret_cast<const double*>(smem);
    const int w8 = gbytes / 8;
    if (step_update_lanes(have_pre, a.D)) {
      // thread i sums entry i over the waves itself and updates it: no row in LDS, no second barrier
      double v = 0.0;
      if (tid < a.nparams) {
        v = g0[tid];
        for (int w = 1; w < nw; ++w) v += g0[w * w8 + tid];
      }
      if (tid == 0) *bc.loss_out = (double)((T)tot[0] / (T)bc.nsamp);
#if ENF_DIAG
      const long long ts3 = a.diag_ts ? (long long)clock64() : 0;
#endif
      step_update_lane<T>(v, a.nparams, a.D, *rs, *ss, pre, bc.scale);
#if ENF_DIAG
      if (a.diag_ts) {  // (uniform)
        __syncthreads();
        const long long ts4 = (long long)clock64();
        if (tid == 0)
          printf("ENF_SMALL_TS prologue %lld (loads %lld, v'v %lld, records %lld) tiles %lld (to fwd end %lld, loss %lld) "
                 "partials %lld update %lld (shader clocks)\n", ts1 - ts0, tsA - ts0, tsB - tsA, ts1 - tsB, ts2 - ts1,
                 tsF ? tsF - ts1 : 0, tsL ? tsL - tsF : 0, ts3 - ts2, ts4 - ts3);
      }
#endif
      return;
    }
    for (int i = tid; i < a.nparams; i += blockDim.x) {
      double v = g0[i];
      for (int w = 1; w < nw; ++w) v += g0[w * w8 + i];
      tot[1 + i] = v;
    }
    __syncthreads();
#if ENF_DIAG
    const long long ts3 = a.diag_ts ? (long long)clock64() : 0;
#endif
    block_step_update<T>(tot, a.nparams, a.D, *rs, *ss, scratch, pre, have_pre, bc.loss_out, bc.nsamp, bc.scale);
#if ENF_DIAG
    if (a.diag_ts) {  // (uniform)
      __syncthreads();
      const long long ts4 = (long long)clock64();
      if (tid == 0)
        printf("ENF_SMALL_TS prologue %lld (loads %lld, v'v %lld, records %lld) tiles %lld partials %lld update %lld "
               "(shader clocks)\n", ts1 - ts0, tsA - ts0, tsB - tsA, ts1 - tsB, ts2 - ts1, ts3 - ts2, ts4 - ts3);
    }
#endif
    return;
  }
  if (!a.partial) return;  // enf_flow_vjp without parameter cotangents
  double* out = (double*)a.partial + (int64_t)blockIdx.x * (1 + a.nparams);
  if (tid == 0) {  // the waves' values in wave order (deterministic)
    double l = lossw[0];
    for (int w = 1; w < nw; ++w) l += lossw[w];
    out[0] = l;
  }
  const double* g0 = reinterpret_cast<const double*>(smem);
  const int w8 = gbytes / 8;
  for (int i = tid; i < a.nparams; i += blockDim.x) {
    double v = g0[i];
    for (int w = 1; w < nw; ++w) v += g0[w * w8 + i];
    out[1 + i] = v;
  }
}

template <typename T, int D, bool VJP, int VL = 0>
__global__ __launch_bounds__(512) void negll_grad_kernel(GradArgs a) {
  negll_grad_impl<T, D, VJP, false, VL>(a, nullptr, nullptr, BatchCtx{a.X, a.N, nullptr, 0, 0.0, true});
}

template <typename T, int D, int VL = 0, class Prog = ProgInterp>
__global__ __launch_bounds__(512) void whitening_step_small_kernel(GradArgs a, ReduceArgs r, StepArgs s) {
  negll_grad_impl<T, D, false, true, VL, Prog>(a, &r, &s, BatchCtx{a.X, a.N, s.loss_out, s.nsamp, s.scale, true});
}

// The single-rank steps of a whole epoch in ONE launch (round 5, enf_whitening_epoch): a minibatch that fits one
// block never needs a second block, so the block walks the minibatches [b0, b0 + bs) of the N columns in order
// (src/optimize_whitening.jl:31-42, Iterators.partition), each step exactly as whitening_step_small_kernel, with
// the parameters it updated visible to its next step's prologue after a workgroup fence and a barrier -- no launch
// per step (the examples' per-step boundary cost) and no device-wide synchronisation. Step j's loss to
// s.loss_out[j].
template <typename T, int D, int VL = 0, class Prog = ProgInterp>
__global__ __launch_bounds__(512) void whitening_epoch_small_kernel(GradArgs a, ReduceArgs r, StepArgs s, int64_t N,
                                                                    int64_t bs) {
  int64_t j = 0;
  for (int64_t b0 = 0; b0 < N; b0 += bs, ++j) {
    const int64_t B = N - b0 < bs ? N - b0 : bs;
    negll_grad_impl<T, D, false, true, VL, Prog>(
        a, &r, &s, BatchCtx{(const T*)a.X + b0 * a.ldx, B, s.loss_out + j, B, 1.0 / (double)B, j == 0});
    __threadfence_block();  // this step's theta / ADAGrad stores before the next step's prologue reads them
    __syncthreads();
  }
}
static_assert(sizeof(GradArgs) + sizeof(ReduceArgs) + sizeof(StepArgs) + 2 * sizeof(int64_t) <= 4096,
              "kernel arguments over 4 KB");

// The update half of a data-parallel step (enf_whitening_apply): the same loss / ADAGrad /
// re-normalisation as whitening_tail_kernel, reading the cross-rank sum g (1 + nparams values of T,
// the all-reduced enf_flow_negll_grad output) instead of the totals. Same operations and roundings
// as out[0:1] / B + enf_adagrad_step per run + enf_householder_normalize_strided per batch.
template <typename T>
__global__ __launch_bounds__(256) void whitening_apply_kernel(const T* __restrict__ g, StepArgs a) {
  T* th = (T*)a.theta;
  T* ac = (T*)a.acc;
  if (threadIdx.x == 0) *a.loss_out = (double)(g[0] / (T)a.nsamp);
  for (int q = 0; q < a.nruns; ++q)
    for (int64_t i = a.runs[q][0] + threadIdx.x; i < a.runs[q][1]; i += blockDim.x)
      adagrad_update<T>(th[i], ac[i], g[1 + i], (T)a.scale, (T)a.eta, (T)a.eps);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int q = 0; q < a.nhb; ++q)
    for (int64_t c = w; c < a.hb[q][1]; c += 4) normalize_column<T>(th + a.hb[q][0] + c * a.hb[q][2], a.D, lane);
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int kSmallMaxWaves = 8;  // the generic kernels' blocks have 4 waves, or 8 for a one-block batch

struct Plan {
  GradArgs ga;
  ReduceArgs ra;
  size_t lds = 0;
  size_t small_lds = 0;  // the single-block fused step's LDS (lds + the block's row and the update's scratch)
  int blocks = 0;   // blocks (partial rows) of the generic kernel
  int ws_rows = 0;  // partial rows the workspace reserves: the generic kernel's or the fused (J o H)^n kernel's
  int nw = 4;  // waves per block of the generic kernel
  int vl = 0;  // values per lane other than the default (negll_grad_impl VL): 1 for fp64 D = 2 batches of <= 256 columns
  int prog = 0;  // one-block steps: 0 = the step-table interpreter, 1 / 2 = the compiled ProgExample1d / 2d
};

// Kernel rows Dp (D rounded up to a power of two) up to 1024: up to 256 fp32 / 128 fp64 a column is a group of
// 16-byte fragments (the flow kernels' layout), above that a column spans the wave with Dp/64 rows per lane
// (round 4; round 3 stopped at 256 / 128).
constexpr int64_t kGradMaxD = 1024;
bool grad_D_supported(int64_t D, bool f64) {
  (void)f64;
  return D >= 1 && D <= kGradMaxD;
}
constexpr size_t kGradLdsMax = 160 * 1024;

// kernel rows: D rounded up to a power of two
int64_t grad_Dp(int64_t D) {
  int64_t p = 1;
  while (p < D) p <<= 1;
  return p;
}

enf_status make_plan(bool f64, int64_t D, int64_t N, const enf_layer* layers, int32_t nlayers, Plan& P) {
  std::memset(&P.ga, 0, sizeof P.ga);
  std::memset(&P.ra, 0, sizeof P.ra);
  if (!grad_D_supported(D, f64))
    return set_error(ENF_ERR_UNSUPPORTED, "enf_flow_negll_grad: D must be <= 1024");
  if (nlayers > kMaxGradLayers) return set_error(ENF_ERR_UNSUPPORTED, "enf_flow_negll_grad: more than 16 layers");
  const int64_t Dp = grad_Dp(D);
  // one row per lane for fp64 D = 2 batches that then still fit one block (<= kSmallMaxWaves tiles of 32 columns)
  P.vl = (f64 && Dp == 2 && N <= 32 * kSmallMaxWaves) ? 1 : 0;
  const int V = P.vl ? P.vl : f64 ? grad_lane_values<double>((int)Dp) : grad_lane_values<float>((int)Dp);
  const int nent = (int)(Dp > V ? Dp : V);
  const bool fast = f64 && Dp <= kFastMaxD;  // grad_fast_rows: the row constants in the records, the log table
  int s = 0, goff = 0, roff = 0;
  for (int l = 0; l < nlayers; ++l) {
    P.ga.layers[l].op = layers[l].op;
    P.ga.layers[l].k = layers[l].k;
    for (int q = 0; q < 4; ++q) P.ga.layers[l].p[q] = layers[l].p[q];
    const int ncol = layers[l].op == OP_HOUSEHOLDER ? layers[l].k : 1;
    for (int c = 0; c < ncol; ++c) {
      if (s >= kMaxGradSteps) return set_error(ENF_ERR_UNSUPPORTED, "enf_flow_negll_grad: more than 32 steps");
      P.ga.op[s] = layers[l].op;
      P.ga.layer[s] = l;
      P.ga.col[s] = c;
      P.ga.roff[s] = roff;
      P.ga.goff[s] = goff + (layers[l].op == OP_HOUSEHOLDER ? c * (int)D : 0);
      if (layers[l].op == OP_HOUSEHOLDER) {
        P.ra.hoff[P.ra.nh] = P.ga.goff[s];
        P.ra.hcol[P.ra.nh] = (const char*)layers[l].p[0] + (size_t)c * D * (f64 ? 8 : 4);
        ++P.ra.nh;
      }
      roff += rec_nparams(layers[l].op, fast) * nent;
      ++s;
    }
    goff += (int)D * (layers[l].op == OP_HOUSEHOLDER ? layers[l].k : grad_nparams(layers[l].op));
  }
  P.ga.D = (int32_t)D;
  P.ga.Dp = (int32_t)Dp;
  P.ga.N = N;
  P.ga.nsteps = s;
  // the reference examples' flows at their dimension run their one-block steps as compiled programs (OpProg)
  auto ops_are = [&](std::initializer_list<int> ops) {
    if ((int)ops.size() != s) return false;
    int i = 0;
    for (int op : ops)
      if (P.ga.op[i++] != op) return false;
    return true;
  };
  P.prog = 0;
  if (f64 && Dp == 1 && P.vl == 0 && ops_are({OP_CENTER_CONTRACT, OP_JOHNSON, OP_CENTER_CONTRACT, OP_JOHNSON})) P.prog = 1;
  if (f64 && Dp == 2 && P.vl == 1 && ops_are({OP_SCALESHIFT, OP_HOUSEHOLDER, OP_CENTER_CONTRACT})) P.prog = 2;
  P.ga.nlayers = nlayers;
  P.ga.nparams = goff;
  P.ga.zq = tl_negll_zygote;
  const size_t esz = f64 ? 8 : 4;
  const size_t gbytes = ((size_t)goff * 8 + 15) / 16 * 16;
  // records, and (fast) the log table after the waves' activations
  const size_t rbytes = ((size_t)(roff + 3) / 4) * 4 * esz + (fast ? 3 * kLogTabN * sizeof(double) : 0);
  const size_t abytes = (size_t)s * 64 * V * esz;  // per wave
  // 4 waves per block, fewer when their per-wave gradient accumulators and activations do not fit
  P.nw = 4;
  while (P.nw > 1 && P.nw * (gbytes + abytes) + 64 + rbytes > kGradLdsMax) P.nw >>= 1;
  P.lds = P.nw * (gbytes + abytes) + 64 + rbytes;  // generic kernel; checked where it is launched
  const int cols = (int)(64 / (Dp >= V ? Dp / V : 1) * (Dp >= V ? 1 : V / Dp));
  const int64_t tiles = (N + cols - 1) / cols;
  // a batch of at most kSmallMaxWaves tiles runs as ONE block with one tile per wave (8 waves when their LDS
  // fits): one partial row, and the single-rank step then runs its update in the same launch (round 5). Two
  // tiles per wave in one block lost to two blocks: a tile of an fp64 flow is a long dependent chain (the 1d
  // example's J o K o J o K, B = 1000: 16.4k against 26.8k steps/s, profiles/r05/example_1d_v2.json)
  if (tiles > P.nw && tiles <= kSmallMaxWaves && P.nw == 4 &&
      (size_t)kSmallMaxWaves * (gbytes + abytes) + 64 + rbytes <= kGradLdsMax) {
    P.nw = kSmallMaxWaves;
    P.lds = P.nw * (gbytes + abytes) + 64 + rbytes;
  }
  int64_t blocks = (tiles + P.nw - 1) / P.nw;
  P.small_lds = P.lds + 16 + ((size_t)goff + 2) * 8 + (size_t)goff * (8 + 2 * esz + 4) + 16;
  DeviceInfo dev;
  if (current_device_info(&dev) != ENF_OK) return ENF_ERR_HIP;
  // blocks per CU (2: what the fused kernel's LDS lets stay resident; measured best at config 5)
  static const int per_cu = ENF_KNOB("ENF_GRAD_BPC", 2);
  const int64_t cap = (int64_t)dev.num_cu * per_cu;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  P.blocks = (int)blocks;
  P.ws_rows = P.blocks;
  if (!f64 && hj_grad_shape_ok(D, layers, nlayers)) P.ws_rows = std::max(P.ws_rows, hj_grad_blocks(D, N, nlayers / 2));
  P.ra.nblocks = P.blocks;
  P.ra.nparams = goff;
  P.ra.D = (int32_t)D;
  P.ra.upb = reduce_units_per_block(D);
  P.ra.nloc = N;
  return ENF_OK;
}

#if ENF_DIAG
// diagnostics (ENF_RED_DBG): the reduction's launch floor -- 1: the same grid and arguments, returning at once;
// 2: one dependent round trip (the loss row's first value to loss_out / tot)
template <typename T, int MODE, int KIND>
__global__ __launch_bounds__(kRedThreads) void reduce_probe_kernel(ReduceArgs r, StepArgs s) {
  if (KIND == 2 && blockIdx.x == 0 && threadIdx.x == 0) {
    if (MODE == MODE_STEP) *s.loss_out = r.partial[0];
    else if (MODE == MODE_SUM) r.tot[0] = r.partial[0];
  }
}
// 3: the same grid with an 8-byte argument (does the ~2 KB argument block cost launch time?)
__global__ __launch_bounds__(kRedThreads) void reduce_probe_small_kernel(double* p) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && p) p[0] = 0.0;
}
#endif

template <typename T, int MODE>
hipError_t launch_reduce(const ReduceArgs& r, const StepArgs& s, hipStream_t st) {
#if ENF_DIAG
  static const int dbg = ENF_KNOB("ENF_RED_DBG", 0);
  if (dbg == 3) {
    hipLaunchKernelGGL(reduce_probe_small_kernel, dim3(reduce_grid(r.D, r.nparams)), dim3(kRedThreads), 0, st,
                       (double*)nullptr);
    return hipGetLastError();
  }
  if (dbg == 1 || dbg == 2) {
    if (dbg == 1) hipLaunchKernelGGL((reduce_probe_kernel<T, MODE, 1>), dim3(reduce_grid(r.D, r.nparams)), dim3(kRedThreads), 0, st, r, s);
    else hipLaunchKernelGGL((reduce_probe_kernel<T, MODE, 2>), dim3(reduce_grid(r.D, r.nparams)), dim3(kRedThreads), 0, st, r, s);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL((grad_reduce_kernel<T, MODE>), dim3(reduce_grid(r.D, r.nparams)), dim3(kRedThreads), 0, st, r, s);
  return hipGetLastError();
}
template <int MODE>
hipError_t launch_reduce(bool f64, const ReduceArgs& r, const StepArgs& s, hipStream_t st) {
  return f64 ? launch_reduce<double, MODE>(r, s, st) : launch_reduce<float, MODE>(r, s, st);
}

// workspace: [partial rows: ws_rows x (1 + nparams)][tot: 1 + nparams][the constant ladj: 1][...] (doubles)
size_t plan_workspace_bytes(const Plan& P) {
  return ((size_t)P.ws_rows + kSumSlices) * (1 + (size_t)P.ga.nparams) * sizeof(double);
}
void plan_bind_workspace(Plan& P, void* workspace) {
  const size_t n = 1 + (size_t)P.ga.nparams;
  P.ga.partial = workspace;
  P.ra.partial = (const double*)workspace;
  P.ra.tot = (double*)workspace + (size_t)P.ws_rows * n;
}
double* plan_ctot_slot(const Plan& P) { return P.ra.tot + 1 + P.ga.nparams; }

template <typename T, int DD, bool VJP, int VL = 0>
hipError_t launch_grad_D(const Plan& P, hipStream_t st) {
  if constexpr (VL == 0 && DD == 2 && std::is_same_v<T, double>) {
    if (P.vl == 1) return launch_grad_D<T, DD, VJP, 1>(P, st);
  }
  if (P.lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)negll_grad_kernel<T, DD, VJP, VL>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)P.lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((negll_grad_kernel<T, DD, VJP, VL>), dim3(P.blocks), dim3(64 * P.nw), P.lds, st, P.ga);
  return hipGetLastError();
}

template <typename T, int DD, int VL = 0, class Prog = ProgInterp>
hipError_t launch_step_small_D(const Plan& P, const StepArgs& sa, hipStream_t st) {
  if constexpr (VL == 0 && Prog::n == 0 && DD == 2 && std::is_same_v<T, double>) {
    if (P.vl == 1) {
      if (P.prog == 2) return launch_step_small_D<T, DD, 1, ProgExample2d>(P, sa, st);
      return launch_step_small_D<T, DD, 1>(P, sa, st);
    }
  }
  if constexpr (VL == 0 && Prog::n == 0 && DD == 1 && std::is_same_v<T, double>) {
    if (P.prog == 1) return launch_step_small_D<T, DD, 0, ProgExample1d>(P, sa, st);
  }
  if (P.small_lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)whitening_step_small_kernel<T, DD, VL, Prog>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)P.small_lds);
    if (e != hipSuccess) return e;
  }
#if ENF_DIAG
  static const int ts = ENF_KNOB("ENF_SMALL_TS", 0);
  if (ts) {
    GradArgs ga = P.ga;
    ga.diag_ts = 1;
    hipLaunchKernelGGL((whitening_step_small_kernel<T, DD, VL, Prog>), dim3(1), dim3(64 * P.nw), P.small_lds, st, ga, P.ra,
                       sa);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL((whitening_step_small_kernel<T, DD, VL, Prog>), dim3(1), dim3(64 * P.nw), P.small_lds, st, P.ga, P.ra,
                     sa);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_step_small(const Plan& P, const StepArgs& sa, hipStream_t st) {
  switch (P.ga.Dp) {
#define ENF_S(DD) case DD: return launch_step_small_D<T, DD>(P, sa, st);
    ENF_S(1) ENF_S(2) ENF_S(4) ENF_S(8) ENF_S(16) ENF_S(32) ENF_S(64) ENF_S(128) ENF_S(256) ENF_S(512) ENF_S(1024)
#undef ENF_S
    default: return hipErrorInvalidValue;
  }
}

template <typename T, int DD, int VL = 0, class Prog = ProgInterp>
hipError_t launch_epoch_small_D(const Plan& P, const StepArgs& sa, int64_t N, int64_t bs, hipStream_t st) {
  if constexpr (VL == 0 && Prog::n == 0 && DD == 2 && std::is_same_v<T, double>) {
    if (P.vl == 1) {
      if (P.prog == 2) return launch_epoch_small_D<T, DD, 1, ProgExample2d>(P, sa, N, bs, st);
      return launch_epoch_small_D<T, DD, 1>(P, sa, N, bs, st);
    }
  }
  if constexpr (VL == 0 && Prog::n == 0 && DD == 1 && std::is_same_v<T, double>) {
    if (P.prog == 1) return launch_epoch_small_D<T, DD, 0, ProgExample1d>(P, sa, N, bs, st);
  }
  if (P.small_lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)whitening_epoch_small_kernel<T, DD, VL, Prog>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)P.small_lds);
    if (e != hipSuccess) return e;
  }
#if ENF_DIAG
  static const int ts = ENF_KNOB("ENF_SMALL_TS", 0);
  if (ts) {
    GradArgs ga = P.ga;
    ga.diag_ts = 1;
    hipLaunchKernelGGL((whitening_epoch_small_kernel<T, DD, VL, Prog>), dim3(1), dim3(64 * P.nw), P.small_lds, st, ga,
                       P.ra, sa, N, bs);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL((whitening_epoch_small_kernel<T, DD, VL, Prog>), dim3(1), dim3(64 * P.nw), P.small_lds, st, P.ga, P.ra,
                     sa, N, bs);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_epoch_small(const Plan& P, const StepArgs& sa, int64_t N, int64_t bs, hipStream_t st) {
  switch (P.ga.Dp) {
#define ENF_E(DD) case DD: return launch_epoch_small_D<T, DD>(P, sa, N, bs, st);
    ENF_E(1) ENF_E(2) ENF_E(4) ENF_E(8) ENF_E(16) ENF_E(32) ENF_E(64) ENF_E(128) ENF_E(256) ENF_E(512) ENF_E(1024)
#undef ENF_E
    default: return hipErrorInvalidValue;
  }
}

template <typename T, bool VJP = false>
hipError_t launch_grad(const Plan& P, hipStream_t st) {
  hipError_t e0 = hipSuccess;
  switch (P.ga.Dp) {
#define ENF_G(DD) case DD: e0 = launch_grad_D<T, DD, VJP>(P, st); break;
    ENF_G(1) ENF_G(2) ENF_G(4) ENF_G(8) ENF_G(16) ENF_G(32) ENF_G(64) ENF_G(128) ENF_G(256) ENF_G(512)
    ENF_G(1024)
#undef ENF_G
    default: return hipErrorInvalidValue;
  }
  return e0;
}

}  // namespace

namespace {
enf_status single_workspace(bool f64, int64_t D, int64_t N, const enf_layer* layers, int32_t nlayers, size_t* bytes) {
  Plan P;
  enf_status s = make_plan(f64, D, N > 0 ? N : 1, layers, nlayers, P);
  if (s != ENF_OK) return s;
  *bytes = plan_workspace_bytes(P);
  return ENF_OK;
}

// The per-block partial rows (fused (J o H)^n kernel or the generic one) in the workspace; P.ra then describes
// them for grad_reduce_kernel (rows, the constant ladj the fused kernel computes once).
enf_status grad_parts(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                      int32_t nlayers, void* workspace, size_t workspace_bytes, hipStream_t st, Plan& P) {
  enf_status s = make_plan(f64, D, N, layers, nlayers, P);
  if (s != ENF_OK) return s;
  if (!workspace || workspace_bytes < plan_workspace_bytes(P))
    return set_error(ENF_ERR_INVALID, "enf_flow_negll_grad: workspace too small");
  P.ga.X = X;
  P.ga.ldx = ldx;
  plan_bind_workspace(P, workspace);
  hipError_t e;
  static const int generic = ENF_KNOB("ENF_GRAD_GENERIC", 0);
  if (!f64 && !generic && hj_grad_eligible(D, ldx, X, layers, nlayers)) {
    // (make_plan reserved hj_grad_blocks(D, N, n) rows for this shape: the launch writes that many)
    int rows = 0;
    e = launch_hj_grad(D, N, X, layers, nlayers, P.ga.nparams, (double*)workspace, plan_ctot_slot(P), &rows, st);
    P.ra.nblocks = rows;
    P.ra.ctot = plan_ctot_slot(P);
  } else {
    if (P.lds > kGradLdsMax) return set_error(ENF_ERR_UNSUPPORTED, "enf_flow_negll_grad: flow too large for LDS");
    e = f64 ? launch_grad<double>(P, st) : launch_grad<float>(P, st);
    P.ra.nblocks = P.blocks;
    P.ra.ctot = nullptr;
  }
  if (e != hipSuccess) return set_error(ENF_ERR_HIP, hipGetErrorString(e));
  return ENF_OK;
}

}  // namespace

enf_status negll_grad_single(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                             int32_t nlayers, void* out, void* workspace, size_t workspace_bytes, hipStream_t st) {
  Plan P;
  enf_status s = grad_parts(f64, D, N, X, ldx, layers, nlayers, workspace, workspace_bytes, st, P);
  if (s != ENF_OK) return s;
  P.ra.out = out;
  StepArgs none;
  std::memset(&none, 0, sizeof none);
  hipError_t e = launch_reduce<MODE_OUT>(f64, P.ra, none, st);
  return e == hipSuccess ? ENF_OK : set_error(ENF_ERR_HIP, hipGetErrorString(e));
}

enf_status flow_vjp_single(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const void* dY, int64_t lddy,
                           const void* dladj, const enf_layer* layers, int32_t nlayers, void* dX, int64_t lddx,
                           void* dparams, void* workspace, size_t workspace_bytes, hipStream_t st) {
  Plan P;
  enf_status s = make_plan(f64, D, N, layers, nlayers, P);
  if (s != ENF_OK) return s;
  if (P.lds > kGradLdsMax) return set_error(ENF_ERR_UNSUPPORTED, "enf_flow_vjp: flow too large for LDS");
  P.ga.X = X;
  P.ga.ldx = ldx;
  P.ga.dY = dY;
  P.ga.lddy = lddy;
  P.ga.dl = dladj;
  P.ga.dX = dX;
  P.ga.lddx = lddx;
  if (dparams) {
    if (!workspace || workspace_bytes < plan_workspace_bytes(P))
      return set_error(ENF_ERR_INVALID, "enf_flow_vjp: workspace too small");
    plan_bind_workspace(P, workspace);
  }
  hipError_t e = f64 ? launch_grad<double, true>(P, st) : launch_grad<float, true>(P, st);
  if (e == hipSuccess && dparams) {
    P.ra.nblocks = P.blocks;
    P.ra.ctot = nullptr;
    P.ra.out = dparams;
    P.ra.skip_loss = 1;
    StepArgs none;
    std::memset(&none, 0, sizeof none);
    e = launch_reduce<MODE_OUT>(f64, P.ra, none, st);
  }
  if (e != hipSuccess) return set_error(ENF_ERR_HIP, hipGetErrorString(e));
  return ENF_OK;
}

enf_status whitening_apply(bool f64, int64_t D, int64_t nparams, const void* g, int64_t B, void* theta, void* acc,
                           const int64_t* runs, int32_t nruns, const int64_t* hb, int32_t nhb, double eta,
                           double epsilon, double* loss_out, hipStream_t st) {
  if (nruns < 0 || nruns > kMaxStepRuns || nhb < 0 || nhb > kMaxStepHB)
    return set_error(ENF_ERR_UNSUPPORTED, "enf_whitening_apply: too many parameter runs or Householder batches");
  StepArgs a;
  std::memset(&a, 0, sizeof a);
  a.theta = theta;
  a.acc = acc;
  a.loss_out = loss_out;
  a.scale = 1.0 / (double)B;
  a.eta = eta;
  a.eps = epsilon;
  a.D = D;
  a.nsamp = B;
  a.nruns = nruns;
  a.nhb = nhb;
  for (int i = 0; i < nruns; ++i) {
    a.runs[i][0] = runs[2 * i];
    a.runs[i][1] = runs[2 * i + 1];
    if (a.runs[i][0] < 0 || a.runs[i][1] < a.runs[i][0] || a.runs[i][1] > nparams)
      return set_error(ENF_ERR_INVALID, "enf_whitening_apply: parameter run outside theta");
  }
  for (int i = 0; i < nhb; ++i) {
    for (int q = 0; q < 3; ++q) a.hb[i][q] = hb[3 * i + q];
    if (a.hb[i][0] < 0 || a.hb[i][1] < 0 || a.hb[i][2] < D ||
        (a.hb[i][1] > 0 && a.hb[i][0] + (a.hb[i][1] - 1) * a.hb[i][2] + D > nparams))
      return set_error(ENF_ERR_INVALID, "enf_whitening_apply: Householder batch outside theta");
  }
  if (f64) hipLaunchKernelGGL((whitening_apply_kernel<double>), dim3(1), dim3(256), 0, st, (const double*)g, a);
  else hipLaunchKernelGGL((whitening_apply_kernel<float>), dim3(1), dim3(256), 0, st, (const float*)g, a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ENF_OK : set_error(ENF_ERR_HIP, hipGetErrorString(e));
}

namespace {
// StepArgs of a single-rank step and their checks against the flow's parameter count np
enf_status step_args(int64_t D, void* theta, void* acc, const int64_t* runs, int32_t nruns, const int64_t* hb,
                     int32_t nhb, double eta, double epsilon, double* loss_out, int64_t B, int64_t np, StepArgs& a) {
  if (nruns < 0 || nruns > kMaxStepRuns || nhb < 0 || nhb > kMaxStepHB)
    return set_error(ENF_ERR_UNSUPPORTED, "enf_whitening_step: too many parameter runs or Householder batches");
  std::memset(&a, 0, sizeof a);
  a.theta = theta;
  a.acc = acc;
  a.loss_out = loss_out;
  a.scale = 1.0 / (double)B;
  a.eta = eta;
  a.eps = epsilon;
  a.D = D;
  a.nsamp = B;
  a.nruns = nruns;
  a.nhb = nhb;
  for (int i = 0; i < nruns; ++i) {
    a.runs[i][0] = runs[2 * i];
    a.runs[i][1] = runs[2 * i + 1];
    if (a.runs[i][0] < 0 || a.runs[i][1] < a.runs[i][0] || a.runs[i][1] > np)
      return set_error(ENF_ERR_INVALID, "enf_whitening_step: parameter run outside theta");
  }
  for (int i = 0; i < nhb; ++i) {
    for (int q = 0; q < 3; ++q) a.hb[i][q] = hb[3 * i + q];
    if (a.hb[i][0] < 0 || a.hb[i][1] < 0 || a.hb[i][2] < D ||
        (a.hb[i][1] > 0 && a.hb[i][0] + (a.hb[i][1] - 1) * a.hb[i][2] + D > np))
      return set_error(ENF_ERR_INVALID, "enf_whitening_step: Householder batch outside theta");
    // (each column is one D-entry vector of the parameter layout: the reduction re-normalises it where it updates it)
    if (a.hb[i][0] % D != 0 || a.hb[i][2] % D != 0)
      return set_error(ENF_ERR_INVALID, "enf_whitening_step: Householder batch columns must start at multiples of D");
  }
  return ENF_OK;
}

// the largest gradient-row payload the data-parallel step hands to the collective instead of reducing it first
constexpr size_t kRowsCollectiveMax = 64 << 10;

// B: the global batch size the update normalises by (N on one rank); ar: the cross-rank sum between the gradient
// and the update (enf_whitening_step_dp), or none; nranks: the ranks of that sum.
enf_status whitening_step_single(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                                 int32_t nlayers, void* theta, void* acc, const int64_t* runs, int32_t nruns,
                                 const int64_t* hb, int32_t nhb, double eta, double epsilon, double* loss_out,
                                 void* workspace, size_t workspace_bytes, hipStream_t st, int64_t B, AllreduceFn ar,
                                 void* ar_ctx, int nranks) {
  Plan P;
  enf_status s = make_plan(f64, D, N > 0 ? N : 1, layers, nlayers, P);
  if (s != ENF_OK) return s;
  StepArgs a;
  s = step_args(D, theta, acc, runs, nruns, hb, nhb, eta, epsilon, loss_out, B, P.ga.nparams, a);
  if (s != ENF_OK) return s;
  const size_t n1 = 1 + (size_t)P.ga.nparams;
  // Data-parallel step of the fused (J o H)^n fp32 kernel over a share of the minibatch (round 6, VERDICT r05 item
  // 5): the cross-rank sum carries the gradient kernel's partial rows themselves -- every rank launches the grid of
  // ceil(B / nranks) columns, and block 0 adds the row {-N ctot, 0...} -- and the update launch sums the summed rows
  // in its fixed order: no reduction launch between the gradient and the sum. The rows trade that launch (~4.4 us)
  // for R times the collective's bytes, so they are taken only while they stay small (kRowsCollectiveMax): config
  // 5's share has R = 197 rows of 641 doubles (1 MB), which an 8-rank ring all-reduce over xGMI moves far slower than
  // one row (the one-rank emulation's 18.2 us does not see that cost; no 8-GPU box to measure it). The choice
  // depends on the flow, B and nranks only, so every rank takes it (the rows of all ranks must line up); one rank
  // with its whole batch (N == B) keeps the path below, bit-identical to enf_whitening_step.
  const bool rows_ok = ar && !f64 && (nranks > 1 || N < B) && ldx == D && hj_grad_shape_ok(D, layers, nlayers);
  const int64_t Nplan = nranks > 1 ? (B + nranks - 1) / nranks : (N > 0 ? N : 1);
  const int R = rows_ok ? hj_grad_launch_rows(D, Nplan, nlayers / 2) + 1 : 0;  // (+ the ctot row)
  if (rows_ok && (size_t)R * n1 * sizeof(double) <= kRowsCollectiveMax) {
    if (N > 0 && (((uintptr_t)X) & 15) != 0)
      return set_error(ENF_ERR_UNSUPPORTED, "enf_whitening_step_dp: X must be 16-byte aligned on this flow");
    if (!workspace || workspace_bytes < ((size_t)R + 2) * n1 * sizeof(double))
      return set_error(ENF_ERR_INVALID, "enf_whitening_step_dp: workspace too small (enf_flow_negll_grad_workspace "
                                        "of ceil(B / ranks) columns)");
    double* rows = (double*)workspace;
    hipError_t e = hipSuccess;
    if (N > 0) {
      int nb = 0;
      e = launch_hj_grad(D, N, X, layers, nlayers, P.ga.nparams, rows, rows + (size_t)R * n1, &nb, st, Nplan, true);
      if (e != hipSuccess) return set_error(ENF_ERR_HIP, hipGetErrorString(e));
      if (nb != R) return set_error(ENF_ERR_HIP, "enf_whitening_step_dp: unexpected gradient grid");
    } else if (hipMemsetAsync(rows, 0, (size_t)R * n1 * sizeof(double), st) != hipSuccess) {
      return set_error(ENF_ERR_HIP, "hipMemsetAsync");
    }
    s = ar(ar_ctx, rows, (int64_t)R * (int64_t)n1, true, st);
    if (s != ENF_OK) return s;
    P.ra.partial = rows;
    P.ra.nblocks = R;
    P.ra.ctot = nullptr;
    P.ra.tot = rows + (size_t)R * n1;
    e = launch_reduce<MODE_STEP>(f64, P.ra, a, st);
    return e == hipSuccess ? ENF_OK : set_error(ENF_ERR_HIP, hipGetErrorString(e));
  }
  // one rank, a batch of one block, not the fused (J o H)^n kernel: gradient and update in ONE launch (round 5)
  static const int small_ok = ENF_KNOB("ENF_STEP_SMALL", 1);
  if (small_ok && !ar && N > 0 && P.blocks == 1 && P.small_lds <= kGradLdsMax &&
      (f64 || !hj_grad_eligible(D, ldx, X, layers, nlayers))) {
    P.ga.X = X;
    P.ga.ldx = ldx;
    P.ga.partial = nullptr;
    hipError_t e = f64 ? launch_step_small<double>(P, a, st) : launch_step_small<float>(P, a, st);
    return e == hipSuccess ? ENF_OK : set_error(ENF_ERR_HIP, hipGetErrorString(e));
  }
  if (N > 0) {
    s = grad_parts(f64, D, N, X, ldx, layers, nlayers, workspace, workspace_bytes, st, P);
    if (s != ENF_OK) return s;
  } else {  // an empty share (a rank without columns in this minibatch): zero totals
    if (!workspace || workspace_bytes < plan_workspace_bytes(P))
      return set_error(ENF_ERR_INVALID, "enf_whitening_step: workspace too small");
    plan_bind_workspace(P, workspace);
    if (hipMemsetAsync(P.ra.tot, 0, n1 * sizeof(double), st) != hipSuccess) return set_error(ENF_ERR_HIP, "hipMemsetAsync");
  }
  hipError_t e = hipSuccess;
  if (ar || N <= 0) {
    if (N > 0) {  // this rank's totals (MODE_SUM), the all-reduce, then the update reading the one summed row
      e = launch_reduce<MODE_SUM>(f64, P.ra, a, st);
      if (e != hipSuccess) return set_error(ENF_ERR_HIP, hipGetErrorString(e));
    }
    if (ar) {
      s = ar(ar_ctx, P.ra.tot, (int64_t)n1, true, st);
      if (s != ENF_OK) return s;
    }
    P.ra.partial = P.ra.tot;
    P.ra.nblocks = 1;
    P.ra.ctot = nullptr;
  }
  e = launch_reduce<MODE_STEP>(f64, P.ra, a, st);
  return e == hipSuccess ? ENF_OK : set_error(ENF_ERR_HIP, hipGetErrorString(e));
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Chunked gradient / VJP (round 4, VERDICT r03 missing item 1): a flow beyond one gradient launch's bounds
// (more than 16 layers or 32 steps, or parameter accumulators and activations that do not fit the LDS, as
// at large D) runs as consecutive chunks of layers (a chained HouseholderTrafo may be split between its
// columns), each within the bounds. The forward pass keeps each chunk's input (a checkpoint, D x N) --
// the reference's pullback recomputes layer inputs instead (householder_trafo.jl:91-101); a checkpoint per
// chunk is exact and costs one D x N buffer each --, the backward pass runs the chunks' VJP kernels in
// reverse, each from its checkpoint, the cotangent of the chunk's output and the ladj cotangent, writing the
// cotangent of its input in place and ACCUMULATING its parameter VJP at the chunk's offset of the flow's
// gradient layout (a chunk's entries are a contiguous range of it: layers in order, a chained
// Householder's columns in order). The loss is the device reduction of enf_flow_negll over the last chunk's
// output and the ladj accumulated over the chunks.
namespace {

struct GradChunk {
  std::vector<enf_layer> layers;
  int64_t goff = 0;     // first gradient entry of the chunk in the flow's layout
  int64_t nparams = 0;  // its gradient entries
};

bool fits_one_launch(bool f64, int64_t D, int64_t N, const enf_layer* layers, int32_t nlayers) {
  Plan P;
  return make_plan(f64, D, N > 0 ? N : 1, layers, nlayers, P) == ENF_OK && P.lds <= kGradLdsMax;
}

// Greedy chunks: units (one layer, or one column of a chained Householder) are appended while the chunk
// fits one launch.
enf_status plan_chunks(bool f64, int64_t D, int64_t N, const enf_layer* layers, int32_t nlayers,
                       std::vector<GradChunk>& out) {
  out.clear();
  const size_t esz = f64 ? 8 : 4;
  GradChunk cur;
  int64_t goff = 0;
  auto unit_layer = [&](int32_t l, int32_t c) {
    enf_layer u = layers[l];
    if (u.op == ENF_OP_HOUSEHOLDER) {
      u.k = 1;
      u.p[0] = (const char*)layers[l].p[0] + (size_t)c * (size_t)D * esz;
    }
    return u;
  };
  for (int32_t l = 0; l < nlayers; ++l) {
    const int32_t ncol = layers[l].op == ENF_OP_HOUSEHOLDER ? layers[l].k : 1;
    const int64_t per = layers[l].op == ENF_OP_HOUSEHOLDER ? D : D * grad_nparams(layers[l].op);
    for (int32_t c = 0; c < ncol; ++c) {
      const enf_layer u = unit_layer(l, c);
      std::vector<enf_layer> trial = cur.layers;
      // the next column of the same chained Householder extends the chunk's last sub-layer
      const bool merge = c > 0 && !trial.empty() && trial.back().op == ENF_OP_HOUSEHOLDER &&
                         (const char*)trial.back().p[0] + (size_t)trial.back().k * (size_t)D * esz == (const char*)u.p[0];
      if (merge) trial.back().k += 1;
      else trial.push_back(u);
      if (fits_one_launch(f64, D, N, trial.data(), (int32_t)trial.size())) {
        cur.layers.swap(trial);
        cur.nparams += per;
      } else {
        if (cur.layers.empty())
          return set_error(ENF_ERR_UNSUPPORTED, "enf_flow_negll_grad: one transform exceeds the gradient kernel's bounds");
        out.push_back(cur);
        cur = GradChunk();
        cur.goff = goff;
        cur.layers.push_back(u);
        cur.nparams = per;
        if (!fits_one_launch(f64, D, N, cur.layers.data(), 1))
          return set_error(ENF_ERR_UNSUPPORTED, "enf_flow_negll_grad: one transform exceeds the gradient kernel's bounds");
      }
      goff += per;
    }
  }
  if (!cur.layers.empty()) out.push_back(cur);
  set_error(ENF_OK, "");
  return ENF_OK;
}

size_t al256g(size_t b) { return (b + 255) / 256 * 256; }

struct ChunkWs {
  size_t ck = 0, y = 0, l = 0, m1 = 0, part = 0, g = 0, vws = 0, total = 0;  // byte offsets / sizes
  size_t vws_bytes = 0;
};

// Workspace layout of the chunked calls: [checkpoints (m - 1) x D x N][Y or the cotangent buffer: D x N]
// [ladj: N][-1 vector: N][loss partials][whitening: g (1 + nparams)][the chunks' VJP workspace (largest)]
enf_status chunk_ws(bool f64, int64_t D, int64_t N, const std::vector<GradChunk>& ch, int64_t nparams, ChunkWs& w) {
  const size_t e = f64 ? 8 : 4, DN = (size_t)D * (size_t)(N > 0 ? N : 1), Nn = (size_t)(N > 0 ? N : 1);
  size_t off = 0;
  w.ck = off;
  off += al256g((ch.size() - 1) * DN * e);
  w.y = off;
  off += al256g(DN * e);
  w.l = off;
  off += al256g(Nn * e);
  w.m1 = off;
  off += al256g(Nn * e);
  w.part = off;
  off += al256g(1025 * sizeof(double));
  w.g = off;
  off += al256g((size_t)(1 + nparams) * e);
  w.vws = off;
  w.vws_bytes = 0;
  for (const GradChunk& c : ch) {
    size_t b = 0;
    enf_status s = single_workspace(f64, D, N > 0 ? N : 1, c.layers.data(), (int32_t)c.layers.size(), &b);
    if (s != ENF_OK) return s;
    w.vws_bytes = std::max(w.vws_bytes, b);
  }
  w.total = off + al256g(w.vws_bytes);
  return ENF_OK;
}

template <typename T>
__global__ void fill_kernel(T* __restrict__ p, int64_t n, T v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

enf_status fill(bool f64, void* p, int64_t n, double v, hipStream_t st) {
  const unsigned nb = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
  if (f64) hipLaunchKernelGGL((fill_kernel<double>), dim3(nb > 0 ? nb : 1), dim3(256), 0, st, (double*)p, n, v);
  else hipLaunchKernelGGL((fill_kernel<float>), dim3(nb > 0 ? nb : 1), dim3(256), 0, st, (float*)p, n, (float)v);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? ENF_OK : set_error(ENF_ERR_HIP, hipGetErrorString(e));
}

int64_t total_params(int64_t D, const enf_layer* layers, int32_t nlayers) {
  int64_t n = 0;
  for (int32_t l = 0; l < nlayers; ++l) n += D * (layers[l].op == ENF_OP_HOUSEHOLDER ? layers[l].k : grad_nparams(layers[l].op));
  return n;
}

// forward over the chunks: checkpoints of chunks 1 .. m-1's inputs; with Yout, the last chunk's output and the
// ladj summed over all chunks (L)
enf_status chunk_forward(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const std::vector<GradChunk>& ch,
                         char* ws, const ChunkWs& w, bool want_y, hipStream_t st) {
  const size_t e = f64 ? 8 : 4, DN = (size_t)D * (size_t)N;
  const void* cur = X;
  int64_t ld = ldx;
  const size_t m = ch.size();
  for (size_t c = 0; c + (want_y ? 0 : 1) < m; ++c) {
    void* dst = c + 1 < m ? (void*)(ws + w.ck + c * DN * e) : (void*)(ws + w.y);
    enf_status s = enf_flow_apply(f64 ? ENF_F64 : ENF_F32, D, N, cur, ld, dst, D, want_y ? ws + w.l : nullptr,
                                  c > 0 ? 1 : 0, ch[c].layers.data(), (int32_t)ch[c].layers.size(), st);
    if (s != ENF_OK) return s;
    cur = dst;
    ld = D;
  }
  return ENF_OK;
}

// backward over the chunks from the cotangent in `cot` (D x N, ld D, overwritten): the last chunk reads dY
// (ld lddy; may be cot), the first writes dX (ld lddx; may be cot); parameter VJPs into dparams + offsets
enf_status chunk_backward(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const void* dY, int64_t lddy,
                          const void* dladj, const std::vector<GradChunk>& ch, void* dX, int64_t lddx, char* dparams,
                          char* ws, const ChunkWs& w, hipStream_t st) {
  const size_t e = f64 ? 8 : 4, DN = (size_t)D * (size_t)N;
  void* cot = ws + w.y;
  for (size_t c = ch.size(); c-- > 0;) {
    const void* in = c == 0 ? X : (const void*)(ws + w.ck + (c - 1) * DN * e);
    const int64_t ldin = c == 0 ? ldx : D;
    const void* gy = c + 1 == ch.size() ? dY : cot;
    const int64_t ldgy = c + 1 == ch.size() ? lddy : D;
    void* gx = c == 0 ? dX : cot;
    const int64_t ldgx = c == 0 ? lddx : D;
    enf_status s = flow_vjp_single(f64, D, N, in, ldin, gy, ldgy, dladj, ch[c].layers.data(), (int32_t)ch[c].layers.size(),
                                   gx, ldgx, dparams ? dparams + (size_t)ch[c].goff * e : nullptr, ws + w.vws,
                                   w.vws_bytes, st);
    if (s != ENF_OK) return s;
  }
  return ENF_OK;
}

// ENF_NEGLL_ZYGOTE on the chunked path: out[0] += N sum log|a| over the flow's ScaleShiftTrafos (one wave; the
// one-launch path adds the same inside the gradient kernel, scaleshift_ladj_lane)
constexpr int kZygoteMaxSS = 64;
struct ZygoteSS {
  const void* p[kZygoteMaxSS];
  int32_t n[kZygoteMaxSS];
  int32_t cnt;
};
template <typename T>
__global__ __launch_bounds__(64) void zygote_loss_kernel(T* out, ZygoteSS z, int64_t N) {
  double s = 0.0;
  for (int i = 0; i < z.cnt; ++i)
    for (int d = threadIdx.x; d < z.n[i]; d += 64) s += log(fabs((double)((const T*)z.p[i])[d]));
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  if (threadIdx.x == 0) out[0] += (T)((double)N * s);
}
enf_status zygote_loss_chunked(bool f64, int64_t D, int64_t N, const std::vector<GradChunk>& ch, void* out,
                               hipStream_t st) {
  ZygoteSS z;
  std::memset(&z, 0, sizeof z);
  for (const GradChunk& c : ch)
    for (const enf_layer& l : c.layers) {
      if (l.op != OP_SCALESHIFT) continue;
      if (z.cnt == kZygoteMaxSS) return set_error(ENF_ERR_UNSUPPORTED, "ENF_NEGLL_ZYGOTE: more than 64 ScaleShiftTrafos");
      z.p[z.cnt] = l.p[0];
      z.n[z.cnt++] = l.k == 1 ? 1 : (int32_t)D;
    }
  if (z.cnt == 0) return ENF_OK;
  if (f64) hipLaunchKernelGGL(zygote_loss_kernel<double>, dim3(1), dim3(64), 0, st, (double*)out, z, N);
  else hipLaunchKernelGGL(zygote_loss_kernel<float>, dim3(1), dim3(64), 0, st, (float*)out, z, N);
  const hipError_t h = hipGetLastError();
  return h == hipSuccess ? ENF_OK : set_error(ENF_ERR_HIP, hipGetErrorString(h));
}

// the whole negll + gradient through the chunks into out (1 + nparams of T, accumulated)
enf_status negll_grad_chunked(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx,
                              const std::vector<GradChunk>& ch, void* out, char* ws, const ChunkWs& w, hipStream_t st) {
  const size_t e = f64 ? 8 : 4;
  enf_status s = chunk_forward(f64, D, N, X, ldx, ch, ws, w, true, st);
  if (s != ENF_OK) return s;
  double* part = (double*)(ws + w.part);
  s = negll_reduce(f64, D, N, ws + w.y, ws + w.l, part, part + 1024, true, st);
  if (s == ENF_OK) s = negll_add_total(f64, part + 1024, out, st);
  if (s == ENF_OK && tl_negll_zygote) s = zygote_loss_chunked(f64, D, N, ch, out, st);
  if (s == ENF_OK) s = fill(f64, ws + w.m1, N, -1.0, st);  // d(loss)/d(ladj) = -1; d(loss)/dY = Y (in place)
  if (s != ENF_OK) return s;
  return chunk_backward(f64, D, N, X, ldx, ws + w.y, D, ws + w.m1, ch, ws + w.y, D, (char*)out + e, ws, w, st);
}

}  // namespace

enf_status negll_grad_workspace(bool f64, int64_t D, int64_t N, const enf_layer* layers, int32_t nlayers,
                                size_t* bytes) {
  if (fits_one_launch(f64, D, N, layers, nlayers)) return single_workspace(f64, D, N > 0 ? N : 1, layers, nlayers, bytes);
  std::vector<GradChunk> ch;
  enf_status s = plan_chunks(f64, D, N, layers, nlayers, ch);
  if (s != ENF_OK) return s;
  ChunkWs w;
  s = chunk_ws(f64, D, N, ch, total_params(D, layers, nlayers), w);
  if (s != ENF_OK) return s;
  *bytes = w.total;
  return ENF_OK;
}

namespace {
enf_status chunked_setup(bool f64, int64_t D, int64_t N, const enf_layer* layers, int32_t nlayers, void* workspace,
                         size_t workspace_bytes, std::vector<GradChunk>& ch, ChunkWs& w, const char* who) {
  enf_status s = plan_chunks(f64, D, N, layers, nlayers, ch);
  if (s != ENF_OK) return s;
  s = chunk_ws(f64, D, N, ch, total_params(D, layers, nlayers), w);
  if (s != ENF_OK) return s;
  if (!workspace || workspace_bytes < w.total)
    return set_error(ENF_ERR_INVALID, (std::string(who) + ": workspace too small (chunked flow: " +
                                       std::to_string(w.total) + " bytes, enf_flow_negll_grad_workspace)").c_str());
  return ENF_OK;
}
}  // namespace

enf_status negll_grad(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                      int32_t nlayers, void* out, void* workspace, size_t workspace_bytes, hipStream_t st) {
  if (fits_one_launch(f64, D, N, layers, nlayers))
    return negll_grad_single(f64, D, N, X, ldx, layers, nlayers, out, workspace, workspace_bytes, st);
  std::vector<GradChunk> ch;
  ChunkWs w;
  enf_status s = chunked_setup(f64, D, N, layers, nlayers, workspace, workspace_bytes, ch, w, "enf_flow_negll_grad");
  if (s != ENF_OK) return s;
  return negll_grad_chunked(f64, D, N, X, ldx, ch, out, (char*)workspace, w, st);
}

enf_status flow_vjp(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const void* dY, int64_t lddy,
                    const void* dladj, const enf_layer* layers, int32_t nlayers, void* dX, int64_t lddx, void* dparams,
                    void* workspace, size_t workspace_bytes, hipStream_t st) {
  if (fits_one_launch(f64, D, N, layers, nlayers))
    return flow_vjp_single(f64, D, N, X, ldx, dY, lddy, dladj, layers, nlayers, dX, lddx, dparams, workspace,
                           workspace_bytes, st);
  std::vector<GradChunk> ch;
  ChunkWs w;
  enf_status s = chunked_setup(f64, D, N, layers, nlayers, workspace, workspace_bytes, ch, w, "enf_flow_vjp");
  if (s != ENF_OK) return s;
  char* ws = (char*)workspace;
  s = chunk_forward(f64, D, N, X, ldx, ch, ws, w, false, st);
  if (s != ENF_OK) return s;
  return chunk_backward(f64, D, N, X, ldx, dY, lddy, dladj, ch, dX, lddx, (char*)dparams, ws, w, st);
}

enf_status whitening_step(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                          int32_t nlayers, void* theta, void* acc, const int64_t* runs, int32_t nruns,
                          const int64_t* hb, int32_t nhb, double eta, double epsilon, double* loss_out,
                          void* workspace, size_t workspace_bytes, hipStream_t st) {
  return whitening_step_dp(f64, D, N, X, ldx, layers, nlayers, theta, acc, runs, nruns, hb, nhb, eta, epsilon, N,
                           loss_out, nullptr, nullptr, workspace, workspace_bytes, st, 1);
}

enf_status whitening_step_dp(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                             int32_t nlayers, void* theta, void* acc, const int64_t* runs, int32_t nruns,
                             const int64_t* hb, int32_t nhb, double eta, double epsilon, int64_t B, double* loss_out,
                             AllreduceFn ar, void* ar_ctx, void* workspace, size_t workspace_bytes, hipStream_t st,
                             int nranks) {
  if (fits_one_launch(f64, D, N, layers, nlayers))
    return whitening_step_single(f64, D, N, X, ldx, layers, nlayers, theta, acc, runs, nruns, hb, nhb, eta, epsilon,
                                 loss_out, workspace, workspace_bytes, st, B, ar, ar_ctx, nranks);
  std::vector<GradChunk> ch;
  ChunkWs w;
  enf_status s = chunked_setup(f64, D, N, layers, nlayers, workspace, workspace_bytes, ch, w, "enf_whitening_step");
  if (s != ENF_OK) return s;
  // the gradient sums into g (zeroed), then the update half of the step (enf_whitening_apply's kernel, B = N)
  char* ws = (char*)workspace;
  const int64_t np = total_params(D, layers, nlayers);
  if (hipMemsetAsync(ws + w.g, 0, (size_t)(1 + np) * (f64 ? 8 : 4), st) != hipSuccess)
    return set_error(ENF_ERR_HIP, "hipMemsetAsync");
  if (N > 0) {
    s = negll_grad_chunked(f64, D, N, X, ldx, ch, ws + w.g, ws, w, st);
    if (s != ENF_OK) return s;
  }
  if (ar) {
    s = ar(ar_ctx, ws + w.g, 1 + np, f64, st);
    if (s != ENF_OK) return s;
  }
  return whitening_apply(f64, D, np, ws + w.g, B, theta, acc, runs, nruns, hb, nhb, eta, epsilon, loss_out, st);
}

// The single-rank steps of one epoch (enf_whitening_epoch): the minibatches [b0, b0 + bs) of the N columns in order,
// step j's loss to loss_out[j]. While the batches fit the one-launch step (whitening_step_single's small-batch
// path), all of them run in ONE launch of whitening_epoch_small_kernel -- the same arithmetic step by step, so the
// result is enf_whitening_step's, bit for bit; a last, shorter batch with another layout and every other flow take
// enf_whitening_step's path, one call per batch.
enf_status whitening_epoch(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, int64_t bs,
                           const enf_layer* layers, int32_t nlayers, void* theta, void* acc, const int64_t* runs,
                           int32_t nruns, const int64_t* hb, int32_t nhb, double eta, double epsilon, double* loss_out,
                           void* workspace, size_t workspace_bytes, hipStream_t st) {
  if (N < 1 || bs < 1) return set_error(ENF_ERR_INVALID, "enf_whitening_epoch: N and batchsize must be >= 1");
  if (bs > N) bs = N;
  const size_t esz = f64 ? 8 : 4;
  const int64_t nb = (N + bs - 1) / bs;
  int64_t done = 0;  // batches run by the epoch kernel
  static const int epoch_ok = ENF_KNOB("ENF_EPOCH_KERNEL", 1);
  if (epoch_ok && fits_one_launch(f64, D, bs, layers, nlayers) && (f64 || !hj_grad_eligible(D, ldx, X, layers, nlayers))) {
    Plan P;
    enf_status s = make_plan(f64, D, bs, layers, nlayers, P);
    if (s != ENF_OK) return s;
    if (P.blocks == 1 && P.small_lds <= kGradLdsMax) {
      int64_t ncols = (N / bs) * bs;
      if (N > ncols) {  // the last batch in the same launch when its own plan has the same layout
        Plan Q;
        s = make_plan(f64, D, N - ncols, layers, nlayers, Q);
        if (s != ENF_OK) return s;
        if (Q.blocks == 1 && Q.vl == P.vl && Q.nw == P.nw) ncols = N;
      }
      StepArgs a;
      s = step_args(D, theta, acc, runs, nruns, hb, nhb, eta, epsilon, loss_out, bs, P.ga.nparams, a);
      if (s != ENF_OK) return s;
      P.ga.X = X;
      P.ga.ldx = ldx;
      P.ga.partial = nullptr;
      if (ncols > 0) {
        hipError_t e = f64 ? launch_epoch_small<double>(P, a, ncols, bs, st) : launch_epoch_small<float>(P, a, ncols, bs, st);
        if (e != hipSuccess) return set_error(ENF_ERR_HIP, hipGetErrorString(e));
      }
      done = (ncols + bs - 1) / bs;
    }
  }
  for (int64_t j = done; j < nb; ++j) {
    const int64_t b0 = j * bs, B = N - b0 < bs ? N - b0 : bs;
    enf_status s = whitening_step_dp(f64, D, B, (const char*)X + (size_t)b0 * (size_t)ldx * esz, ldx, layers, nlayers,
                                     theta, acc, runs, nruns, hb, nhb, eta, epsilon, B, loss_out + j, nullptr, nullptr,
                                     workspace, workspace_bytes, st, 1);
    if (s != ENF_OK) return s;
  }
  return ENF_OK;
}

}  // namespace enf
