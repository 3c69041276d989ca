// enf_flow_hj64.hip -- compiled fp64 program for the (J o H)^n flows of configs 3-5 in Float64, the
// reference's default parameter type (src/johnson_trafo.jl:61-66): J_n o H_n o ... o J_1 o H_1, each H one
// Householder reflection (src/householder_trafo.jl:8-11), each J a JohnsonTrafo (src/johnson_trafo.jl:
// 29-32, ladj :39-42 / :76-80), D in {32, 64}, fused in one launch (X read once, Y and ladj written once).
//
// Per pair, in the fp64 interpreter's operations (enf_steps.h step_householder / step_johnson fp64):
//   dot = vh'y (vh = v sqrt(2/v'v)),  x = fma(-dot, vh, y),  z = fma(x, 1/lambda, -xi/lambda) (as the fp32
//   program; round 4, one instruction fewer than (x - xi) * (1/lambda)),
//   y   = fma(delta, asinh64_tab(z), gamma),       ladj += log|delta/lambda| - log(q_1 ... q_R)/2
// with q = fma(z, z, 1) and one table logarithm per column and lane of the product of the lane's R = 8 q of
// every pair (round 4; before, one per pair), carried as a mantissa and an exponent sum so that it never
// overflows. A tile in which some |z| of the wave reaches 2^26, Inf or NaN is redone from X on the whole-range
// path (asinh64_tab over the whole double range, logprod64_tab per pair: Inf / NaN propagate as the
// reference's log(1/sqrt(Inf)) / NaN do).
//
// Why: the interpreter's fp64 fragment is 2 rows (16 bytes), so at D = 32 a column spans 16 lanes: every
// reflection dot needs 4 DPP stages of two 32-bit halves per 2 rows and the ladj one table log per 2
// rows. Here a lane owns R = 8 rows of one column (4 fragments): 2 DPP stages per dot for 8 rows and one
// table log per 8 rows, the step table is compiled away, and the records are read per pair.
//
// Layout: a lane owns rows h*(D/4) + 2g + e (fragment h = 0..3, e = 0..1, g = lane % G the lane's row
// group, G = D/8 lanes per column, adjacent); a slab is one load instruction per fragment and covers
// CPS = 64/G columns (16 B per lane, 2 rows of each of CPS columns per 64 lanes... 1 KiB per
// wave-instruction); a wave tile is U slabs. Records (LDS, double): per pair and group
// [param q][8 values, value 2h+e = row h*(D/4)+2g+e], q = {vh, -xi/lambda, 1/lambda, delta, gamma}.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "enf_frag.h"
#include "enf_internal.h"
#include "enf_logtab.h"
#include "enf_math64.h"

namespace enf {

constexpr int kHj64MaxPairs = 8;
constexpr int kHj64W = 5;  // record parameters per row
enum : int { H64_VH = 0, H64_XI = 1, H64_IL = 2, H64_DL = 3, H64_GM = 4 };
// the inverse program's records (round 4): {1/delta, -gamma/delta, lambda, xi, vh}
enum : int { HI64_ID = 0, HI64_NG = 1, HI64_LM = 2, HI64_XI = 3, HI64_VH = 4 };

struct HJ64Args {
  const double* X;
  double* Y;
  double* ladj;
  int64_t N;
  int32_t n;  // pairs
  int32_t dreal;  // rows of the batch: D, or fewer on the padded layout (PAD: rows past dreal are inert)
  const double* v[kHj64MaxPairs];
  const double* g[kHj64MaxPairs];
  const double* d[kHj64MaxPairs];
  const double* xi[kHj64MaxPairs];
  const double* lam[kHj64MaxPairs];
};

// LDS: [scratch: per pair {hs, cl} + ctot][log table][ladj staging: 4 waves x kStagePerWave][records]
constexpr size_t kHj64Scratch = ((2 * kHj64MaxPairs + 2) * sizeof(double) + 15) / 16 * 16;
constexpr size_t kHj64Tab = ((3 * kLogTabN) * sizeof(double) + 15) / 16 * 16;
constexpr size_t kHj64Header = kHj64Scratch + kHj64Tab + 4 * kStagePerWave * sizeof(double);
static size_t hj64_lds_bytes(int D, int n) { return kHj64Header + (size_t)n * kHj64W * D * sizeof(double); }

template <int D, int U>
struct H64Lay {
  static constexpr int R = 8, NF = 4;
  static constexpr int G = D / R;
  static constexpr int CPS = 64 / G;
  static constexpr int TC = CPS * U;  // columns per wave tile
  static constexpr int NLS = (TC + 63) / 64;
  static_assert(D % R == 0 && G >= 2 && G <= 64, "layout");
  static_assert(TC <= kStagePerWave, "ladj staging");
  __device__ static __forceinline__ int64_t col(int64_t col0, int u, int lane) {
    return col0 + (int64_t)u * CPS + lane / G;
  }
  __device__ static __forceinline__ int row(int h, int lane) { return h * (D / NF) + 2 * (lane % G); }
  __device__ static __forceinline__ int64_t ladj_col(int64_t col0, int k, int lane) {
    return col0 + (int64_t)k * 64 + (TC >= 64 ? lane : lane % TC);
  }
};

// PAD (padded layout, round 3): D is the power-of-two layout, columns are a.dreal rows apart; a fragment
// (2 rows) at or past a.dreal holds zeros and is neither loaded nor stored (a.dreal is even).
template <int D, int U, bool TAIL, bool PAD = false>
__device__ __forceinline__ void h64_load(const HJ64Args& a, int64_t col0, double (&x)[U][8]) {
  using L = H64Lay<D, U>;
  const int lane = threadIdx.x & 63;
  const int64_t ld = PAD ? (int64_t)a.dreal : (int64_t)D;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t c = L::col(col0, u, lane);
#pragma unroll
    for (int h = 0; h < L::NF; ++h) {
      const int64_t off = c * ld + L::row(h, lane);
      if (PAD && L::row(h, lane) >= a.dreal) {
        x[u][2 * h] = 0.0;
        x[u][2 * h + 1] = 0.0;
      } else if (!TAIL) {
        if (ENF_INB(c < a.N, "hj64 load X", c, a.N)) {
          const u32x4 v4 = *reinterpret_cast<const u32x4*>(a.X + off);
          __builtin_memcpy(&x[u][2 * h], &v4, 16);
        }
      } else {
        x[u][2 * h] = c < a.N ? a.X[off] : 0.0;
        x[u][2 * h + 1] = c < a.N ? a.X[off + 1] : 0.0;
      }
    }
  }
}

template <int D, int U, int LM>
__device__ __forceinline__ void h64_load_old(const HJ64Args& a, int64_t col0, double (&old)[H64Lay<D, U>::NLS],
                                             bool tail) {
  using L = H64Lay<D, U>;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < L::NLS; ++k) {
    const int64_t c = L::ladj_col(col0, k, lane);
    old[k] = (LM == 2 && (!tail || c < a.N)) ? a.ladj[c] : 0.0;
  }
}

template <int D, int U, int LM, bool TAIL, bool PAD = false>
__device__ __forceinline__ void h64_store(const HJ64Args& a, double ctot, int64_t col0, const double (&x)[U][8],
                                          const double (&acc)[U], const double (&old)[H64Lay<D, U>::NLS],
                                          double* __restrict__ stage) {
  using L = H64Lay<D, U>;
  const int lane = threadIdx.x & 63;
  const int64_t ld = PAD ? (int64_t)a.dreal : (int64_t)D;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t c = L::col(col0, u, lane);
#pragma unroll
    for (int h = 0; h < L::NF; ++h) {
      const int64_t off = c * ld + L::row(h, lane);
      if (PAD && L::row(h, lane) >= a.dreal) {
        continue;
      } else if (!TAIL) {
        u32x4 v4;
        __builtin_memcpy(&v4, &x[u][2 * h], 16);
        if (!ENF_INB(c < a.N, "hj64 store Y", c, a.N)) continue;
        __builtin_nontemporal_store(v4, reinterpret_cast<u32x4*>(a.Y + off));
      } else if (c < a.N) {
        a.Y[off] = x[u][2 * h];
        a.Y[off + 1] = x[u][2 * h + 1];
      }
    }
  }
  if constexpr (LM > 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double tot = group_sum<L::G>(acc[u]);
      if ((lane % L::G) == 0) stage[u * L::CPS + lane / L::G] = tot;
    }
#pragma unroll
    for (int k = 0; k < L::NLS; ++k) {
      const int c = k * 64 + (L::TC >= 64 ? lane : lane % L::TC);
      const double v = (ctot + stage[c]) + old[k];
      const int64_t col = col0 + c;
      if ((!TAIL && ENF_INB(col < a.N, "hj64 ladj", col, a.N)) || (TAIL && col < a.N)) a.ladj[col] = v;
    }
  }
}

// Block prologue: the log table, then per pair (one wave each) v'v and sum_d log|delta/lambda| in double,
// then the records. ctot = the sum of the per-pair constants (INV: their negation, -johnsontrafo_ladj).
template <int D, bool INV>
__device__ void build_hj64_program(const HJ64Args& a, double* __restrict__ rec, double* __restrict__ scr,
                                   double* __restrict__ tab, double* ctot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int n = a.n;
  for (int i = threadIdx.x; i < 3 * kLogTabN; i += blockDim.x) tab[i] = kLogTab[i];
  for (int p = wave; p < n; p += nw) {
    double vv = 0.0, cl = 0.0;
    for (int d = lane; d < a.dreal; d += 64) {  // the batch's rows (padded rows: neutral records below)
      const double vd = a.v[p][d];
      vv += vd * vd;
      cl += log(fabs(a.d[p][d])) - log(fabs(a.lam[p][d]));  // johnson_trafo.jl:41
    }
    for (int m = 32; m >= 1; m >>= 1) {
      vv += __shfl_xor(vv, m);
      cl += __shfl_xor(cl, m);
    }
    if (lane == 0) {
      scr[2 * p] = sqrt(2.0 / vv);  // householder_trafo.jl:9-10: 2 v (v'x) / (v'v)
      scr[2 * p + 1] = cl;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n * D; i += blockDim.x) {
    const int p = i / D, d = i % D;
    const int h = d / (D / 4), w = d % (D / 4), g = w / 2, e = w % 2;
    double* r = rec + (size_t)p * kHj64W * D + g * kHj64W * 8 + 2 * h + e;
    // a padded row (d >= dreal): vh = 0, xi = 0, 1/lambda = 1, gamma = 0 (inverse: 1/delta = 1, lambda = 1,
    // the rest 0) -- its zeros stay zero with q = 1
    const bool real = d < a.dreal;
    if constexpr (!INV) {
      r[H64_VH * 8] = real ? a.v[p][d] * scr[2 * p] : 0.0;
      r[H64_XI * 8] = real ? -(a.xi[p][d] / a.lam[p][d]) : 0.0;
      r[H64_IL * 8] = real ? 1.0 / a.lam[p][d] : 1.0;  // one multiply per element instead of a division
      r[H64_DL * 8] = real ? a.d[p][d] : 1.0;
      r[H64_GM * 8] = real ? a.g[p][d] : 0.0;
    } else {
      r[HI64_ID * 8] = real ? 1.0 / a.d[p][d] : 1.0;
      r[HI64_NG * 8] = real ? -(a.g[p][d] / a.d[p][d]) : 0.0;
      r[HI64_LM * 8] = real ? a.lam[p][d] : 1.0;
      r[HI64_XI * 8] = real ? a.xi[p][d] : 0.0;
      r[HI64_VH * 8] = real ? a.v[p][d] * scr[2 * p] : 0.0;
    }
  }
  if (threadIdx.x == 0) {
    double c = 0.0;
    for (int p = 0; p < n; ++p) c += scr[2 * p + 1];
    *ctot = INV ? -c : c;
  }
  __syncthreads();
}

// 8 doubles of one parameter of the lane's rows: four 16-byte LDS reads
__device__ __forceinline__ void h64_param(const double* __restrict__ r, double (&p)[8]) {
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const u32x4 w = *reinterpret_cast<const u32x4*>(r + 2 * h);
    __builtin_memcpy(&p[2 * h], &w, 16);
  }
}

// fma(a, b, c) as the three-address v_fma_f64: the compiler's two-address v_fmac_f64 for y = fma(delta, asinh,
// gamma) needed a v_mov_b64 of gamma into the loop-carried register per element (round 4)
__device__ __forceinline__ double fma3_f64(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// v = 2^k m for v >= 1 finite: returns m in [1, 2) and adds k to ke (the running q product of h64_pair)
__device__ __forceinline__ double h64_mant(double v, int& ke) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t hi = (uint32_t)(b >> 32);
  ke += (int)(hi >> 20) - 1023;
  return __builtin_bit_cast(double, ((uint64_t)((hi & 0xFFFFFu) | 0x3FF00000u) << 32) | (uint32_t)b);
}

// One pair. FULL = false (the tile's first pass): the range-free asinh64_tab_fin, and the ladj's q products
// carried across the pairs as a mantissa pm in [1, 2) and an exponent sum pk (one table log per tile and lane
// instead of one per pair; round 4), with far set when some |z| of this lane reaches 2^26, Inf or NaN -- no
// branch, so the pair loop has no per-pair vote and no register copies at a join. FULL = true: asinh64_tab over the
// whole double range and logprod64_tab per pair into acc (the tile's redo when some lane of the wave was far).
template <int D, int U, bool LADJ, bool FULL>
__device__ __forceinline__ void h64_pair(double (&x)[U][8], double (&acc)[U], double (&pm)[U], int (&pk)[U],
                                         bool& far, const double* __restrict__ r, const double* __restrict__ tab) {
  constexpr int G = H64Lay<D, U>::G;
  double vh[8];
  h64_param(r + H64_VH * 8, vh);
  // Householder: dot over the lane's 8 rows (two chains), then the G lanes of the column
  double dot[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    double d0 = vh[0] * x[u][0], d1 = vh[1] * x[u][1];
#pragma unroll
    for (int e = 2; e < 8; e += 2) {
      d0 = fma(vh[e], x[u][e], d0);
      d1 = fma(vh[e + 1], x[u][e + 1], d1);
    }
    dot[u] = group_sum<G>(d0 + d1);
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) x[u][e] = fma(-dot[u], vh[e], x[u][e]);
  // Johnson: z = (x - xi) / lambda as fma(x, 1/lambda, -xi/lambda), y = gamma + delta asinh(z),
  // ladj -= log(prod q)/2
  double pxi[8], pil[8];
  h64_param(r + H64_XI * 8, pxi);
  h64_param(r + H64_IL * 8, pil);
  double q[U][8];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const double z = fma(x[u][e], pil[e], pxi[e]);
      x[u][e] = z;
      q[u][e] = fma(z, z, 1.0);
    }
  double pd[8], pg[8];
  h64_param(r + H64_DL * 8, pd);
  h64_param(r + H64_GM * 8, pg);
  if constexpr (!FULL) {
    // Range check: every q of the lane below 2^52 (|z| < 2^26, where asinh64_tab_fin equals asinh64_tab; past
    // ~2^40 its 1/u = (s1 - a) + corr loses to rounding, tools/asinh64_tab_check.hip), as the largest high
    // word of the 8 q (q >= 1, so the unsigned order of the high words is the order of the values; +Inf and
    // NaN of either sign compare above): three v_max3_u32 and one compare per 8 elements instead of a compare per
    // element.
    // The product of the 8 q (< 2^416) times the tile's running mantissa is renormalised.
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t mx = 0;
      double p = q[u][0];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        mx = max(mx, (uint32_t)(__builtin_bit_cast(uint64_t, q[u][e]) >> 32));
        if (e) p *= q[u][e];
      }
      far = far || !(mx < 0x43300000u);  // 2^52
      if (LADJ) pm[u] = h64_mant(pm[u] * p, pk[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) x[u][e] = fma3_f64(pd[e], asinh64_tab_fin(x[u][e], tab), pg[e]);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) x[u][e] = fma(pd[e], asinh64_tab(x[u][e], tab), pg[e]);
    if (LADJ)
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] -= 0.5 * logprod64_tab<8>(q[u], tab);
  }
}

// One pair of the inverse program (round 4): J^-1 then the reflection (inverse(J o H) = H o J^-1,
// johnson_trafo.jl:82, householder_trafo.jl:153-154):
//   w = (y - gamma)/delta as fma(y, 1/delta, -gamma/delta),  sh = sinh(w),  x = fma(lambda, sh, xi)
//   ladj += -log|delta/lambda| + log(1 + sh^2)/2 (the reference's -johnsontrafo_ladj of the output,
//   johnson_trafo.jl:103-104, whose (x - xi)/lambda is sh up to the rounding of x; the constant in ctot)
//   dot = vh'x,  x = fma(-dot, vh, x)
// FULL = false: sinh64_in and the q = 1 + sh^2 products carried as in h64_pair (the product below 2^1000 is the
// range check: |sh| < 2^500, so |w| < ~347 where sinh64_in holds); FULL = true: the interpreter's step
// (sinh64 over the whole range, log1p64_tab of sh^2 per element: +Inf where the reference's 1 + z^2 overflows).
template <int D, int U, bool LADJ, bool FULL>
__device__ __forceinline__ void h64i_pair(double (&x)[U][8], double (&acc)[U], double (&pm)[U], int (&pk)[U],
                                          bool& far, const double* __restrict__ r, const double* __restrict__ tab) {
  constexpr int G = H64Lay<D, U>::G;
  double pid[8], png[8], pl[8], px[8];
  h64_param(r + HI64_ID * 8, pid);
  h64_param(r + HI64_NG * 8, png);
  h64_param(r + HI64_LM * 8, pl);
  h64_param(r + HI64_XI * 8, px);
  double q[U][8];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const double w = fma(x[u][e], pid[e], png[e]);
      const double sh = FULL ? sinh64(w) : sinh64_in(w);
      x[u][e] = fma3_f64(pl[e], sh, px[e]);
      q[u][e] = FULL ? sh * sh : fma(sh, sh, 1.0);
    }
  if constexpr (!FULL) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      double p = q[u][0];
#pragma unroll
      for (int e = 1; e < 8; ++e) p *= q[u][e];
      far = far || !(p < 0x1p1000);
      if (LADJ) pm[u] = h64_mant(pm[u] * p, pk[u]);
    }
  } else if (LADJ) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[u] += 0.5 * log1p64_tab(q[u][e], tab);
  }
  double vh[8];
  h64_param(r + HI64_VH * 8, vh);
  double dot[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    double d0 = vh[0] * x[u][0], d1 = vh[1] * x[u][1];
#pragma unroll
    for (int e = 2; e < 8; e += 2) {
      d0 = fma(vh[e], x[u][e], d0);
      d1 = fma(vh[e + 1], x[u][e + 1], d1);
    }
    dot[u] = group_sum<G>(d0 + d1);
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) x[u][e] = fma(-dot[u], vh[e], x[u][e]);
}

// A tile: every pair on the in-range path; if any lane of the wave left it (a wave-uniform
// vote after the last pair), the wave reloads the tile's X (not yet overwritten: Y is stored after this) and
// redoes every pair on the whole-range path.
template <int D, int U, int LM, bool TAIL, bool PAD, bool INV>
__device__ __forceinline__ void h64_tile(const HJ64Args& a, const double* __restrict__ rec, const double* tab,
                                         double ctot, double* stage, int64_t col0, double (&x)[U][8],
                                         const double (&old)[H64Lay<D, U>::NLS]) {
  double acc[U], pm[U];
  int pk[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    acc[u] = 0.0;
    pm[u] = 1.0;
    pk[u] = 0;
  }
  bool far = false;
  for (int p = 0; p < a.n; ++p) {
    if constexpr (INV) h64i_pair<D, U, (LM > 0), false>(x, acc, pm, pk, far, rec + (size_t)p * kHj64W * D, tab);
    else h64_pair<D, U, (LM > 0), false>(x, acc, pm, pk, far, rec + (size_t)p * kHj64W * D, tab);
  }
  if (__builtin_expect(__any(far), 0)) {
    h64_load<D, U, TAIL, PAD>(a, col0, x);
    for (int p = 0; p < a.n; ++p) {
      if constexpr (INV) h64i_pair<D, U, (LM > 0), true>(x, acc, pm, pk, far, rec + (size_t)p * kHj64W * D, tab);
      else h64_pair<D, U, (LM > 0), true>(x, acc, pm, pk, far, rec + (size_t)p * kHj64W * D, tab);
    }
  } else if constexpr (LM > 0) {
    // -+log(prod q)/2 over the pairs: log(pm 2^pk), pm in [1, 2)
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] += (INV ? 0.5 : -0.5) * log64_tab(pm[u], pk[u], tab);
  }
  h64_store<D, U, LM, TAIL, PAD>(a, ctot, col0, x, acc, old, stage);
}

// OCC: minimum waves per SIMD the register allocation must allow (1: no constraint; the D = 32 / 64 program
// takes 164 VGPRs, 3 waves per SIMD; OCC = 4 caps it at 128). INV: the inverse program (J^-1, H)^n (round 4).
template <int D, int U, int LM, bool PAD = false, int OCC = 1, bool INV = false>
__global__ __launch_bounds__(256, OCC) void flow_hj64_kernel(HJ64Args a) {
  using L = H64Lay<D, U>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* scr = reinterpret_cast<double*>(smem);
  double* ctotp = scr + 2 * kHj64MaxPairs;
  double* tab = reinterpret_cast<double*>(smem + kHj64Scratch);
  double* stage = reinterpret_cast<double*>(smem + kHj64Scratch + kHj64Tab) + (threadIdx.x >> 6) * kStagePerWave;
  double* rec = reinterpret_cast<double*>(smem + kHj64Header);
  build_hj64_program<D, INV>(a, rec, scr, tab, ctotp);
  const double ctot = *ctotp;
  const double* myrec = rec + ((threadIdx.x & 63) % L::G) * kHj64W * 8;
  constexpr int64_t CT = L::TC;
  const int64_t ntiles_full = a.N / CT;
  const int64_t wave_id = (int64_t)blockIdx.x * (blockDim.x >> 6) +
                          __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  double xa[U][8], xb[U][8], old[L::NLS];
  int64_t t = wave_id;
  if (t < ntiles_full) {
    h64_load<D, U, false, PAD>(a, t * CT, xa);
    h64_load_old<D, U, LM>(a, t * CT, old, false);
    for (;;) {
      const int64_t t1 = t + nwaves;
      const bool more = t1 < ntiles_full;
      h64_load<D, U, false, PAD>(a, (more ? t1 : t) * CT, xb);  // prefetch (the current tile again at the end)
      h64_tile<D, U, LM, false, PAD, INV>(a, myrec, tab, ctot, stage, t * CT, xa, old);
      if (!more) break;
      h64_load_old<D, U, LM>(a, t1 * CT, old, false);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) xa[u][e] = xb[u][e];
      t = t1;
    }
  }
  if (ntiles_full * CT < a.N && wave_id == ntiles_full % nwaves) {
    const int64_t c0 = ntiles_full * CT;
    h64_load<D, U, true, PAD>(a, c0, xa);
    h64_load_old<D, U, LM>(a, c0, old, true);
    h64_tile<D, U, LM, true, PAD, INV>(a, myrec, tab, ctot, stage, c0, xa, old);
  }
}

template <int D, int U, int LM, bool PAD = false, int OCC = 1, bool INV = false>
static hipError_t launch_hj64(const HJ64Args& h, hipStream_t st, const DeviceInfo& dev) {
  const size_t lds = hj64_lds_bytes(D, h.n);
  const void* k = reinterpret_cast<const void*>(&flow_hj64_kernel<D, U, LM, PAD, OCC, INV>);
  int64_t blocks = 0;
  hipError_t e = frag_grid(k, h.N, (int64_t)H64Lay<D, U>::TC * 4, lds, dev, &blocks);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((flow_hj64_kernel<D, U, LM, PAD, OCC, INV>), dim3((unsigned)blocks), dim3(256), lds, st, h);
  return hipGetLastError();
}

template <int D, bool PAD, bool INV>
static hipError_t launch_hj64_lm(const HJ64Args& h, int lm, hipStream_t st, const DeviceInfo& dev) {
#if ENF_DIAG
  // ENF_HJ64_OCC (diagnostics build): 4 = the register allocation capped for 4 waves per SIMD (A/B)
  static const int occ = ENF_KNOB("ENF_HJ64_OCC", 1);
  if (occ == 4 && lm == 1 && !PAD && D <= 64) return launch_hj64<D, 1, 1, false, 4, INV>(h, st, dev);
#endif
  if (lm == 0) return launch_hj64<D, 1, 0, PAD, 1, INV>(h, st, dev);
  if (lm == 1) return launch_hj64<D, 1, 1, PAD, 1, INV>(h, st, dev);
  return launch_hj64<D, 1, 2, PAD, 1, INV>(h, st, dev);
}

template <bool INV>
static hipError_t launch_hj64_layout(const HJ64Args& h, int dl, int lm, hipStream_t st, const DeviceInfo& dev) {
  const bool pad = dl != h.dreal;
  if (dl == 32) return pad ? launch_hj64_lm<32, true, INV>(h, lm, st, dev) : launch_hj64_lm<32, false, INV>(h, lm, st, dev);
  if (dl == 64) return pad ? launch_hj64_lm<64, true, INV>(h, lm, st, dev) : launch_hj64_lm<64, false, INV>(h, lm, st, dev);
  if (dl == 128) return pad ? launch_hj64_lm<128, true, INV>(h, lm, st, dev) : launch_hj64_lm<128, false, INV>(h, lm, st, dev);
  return hipErrorNotSupported;
}

// the compiled fp64 inverse program (round 4): (J^-1, H)^n flows, i.e. inverse(J_n o H_n o ... o J_1 o H_1)
// (hji_program_pairs: steps J^-1, H, J^-1, H, ... on layout 32 / 64 / 128, padded or not)
hipError_t launch_hji64_program(const FlowArgs& a, int lm, hipStream_t st, const DeviceInfo& dev) {
  const int n = hji_program_pairs(a);
  if (n < 1 || n > kHj64MaxPairs) return hipErrorNotSupported;
  HJ64Args h;
  memset(&h, 0, sizeof h);
  h.X = (const double*)a.X;
  h.Y = (double*)a.Y;
  h.ladj = (double*)a.ladj;
  h.N = a.N;
  h.n = n;
  h.dreal = a.D;
  for (int p = 0; p < n; ++p) {
    const LayerDesc& J = a.layers[a.steps[2 * p].layer];
    const Step& sh = a.steps[2 * p + 1];
    h.v[p] = (const double*)a.layers[sh.layer].p[0] + (int64_t)sh.col * a.D;
    h.g[p] = (const double*)J.p[0];
    h.d[p] = (const double*)J.p[1];
    h.xi[p] = (const double*)J.p[2];
    h.lam[p] = (const double*)J.p[3];
  }
  return launch_hj64_layout<true>(h, a.dk ? a.dk : a.D, lm, st, dev);
}

hipError_t launch_hj64_program(const FlowArgs& a, int lm, hipStream_t st, const DeviceInfo& dev) {
  const int n = hj_program_pairs(a);  // layout 32 / 64 / 128, padded or not
  if (n < 1 || n > kHj64MaxPairs) return hipErrorNotSupported;
  const int dl = a.dk ? a.dk : a.D;
  HJ64Args h;
  memset(&h, 0, sizeof h);
  h.X = (const double*)a.X;
  h.Y = (double*)a.Y;
  h.ladj = (double*)a.ladj;
  h.N = a.N;
  h.n = n;
  h.dreal = a.D;
  for (int p = 0; p < n; ++p) {
    const Step& sh = a.steps[2 * p];
    const LayerDesc& J = a.layers[a.steps[2 * p + 1].layer];
    h.v[p] = (const double*)a.layers[sh.layer].p[0] + (int64_t)sh.col * a.D;
    h.g[p] = (const double*)J.p[0];
    h.d[p] = (const double*)J.p[1];
    h.xi[p] = (const double*)J.p[2];
    h.lam[p] = (const double*)J.p[3];
  }
  return launch_hj64_layout<false>(h, dl, lm, st, dev);
}

}  // namespace enf
