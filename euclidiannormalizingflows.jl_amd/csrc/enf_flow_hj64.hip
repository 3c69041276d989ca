// enf_flow_hj64.hip -- compiled fp64 program for the (J o H)^n flows of configs 3-5 in Float64, the
// reference's default parameter type (src/johnson_trafo.jl:61-66): J_n o H_n o ... o J_1 o H_1, each H one
// Householder reflection (src/householder_trafo.jl:8-11), each J a JohnsonTrafo (src/johnson_trafo.jl:
// 29-32, ladj :39-42 / :76-80), D in {32, 64}, fused in one launch (X read once, Y and ladj written once).
//
// Per pair, in the fp64 interpreter's operations (enf_steps.h step_householder / step_johnson fp64):
//   dot = vh'y (vh = v sqrt(2/v'v)),  x = fma(-dot, vh, y),  z = (x - xi) * (1/lambda),
//   y   = fma(delta, asinh64_tab(z), gamma),       ladj += log|delta/lambda| - log(q_1 ... q_R)/2
// with q = fma(z, z, 1) and one table logarithm of the product of a lane's R = 8 q per column and pair
// (logprod64_tab: exponents summed as integers, so the product never overflows; Inf / NaN propagate as
// the reference's log(1/sqrt(Inf)) / NaN do). asinh64_tab covers the whole double range itself
// (|z| >= 2^26, Inf, NaN), so there is no exact-range redo as in the fp32 program.
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
// [param q][8 values, value 2h+e = row h*(D/4)+2g+e], q = {vh, xi, 1/lambda, delta, gamma}.
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
// then the records. ctot = the sum of the per-pair constants.
template <int D>
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
    // a padded row (d >= dreal): vh = 0, xi = 0, 1/lambda = 1, gamma = 0 -- its zeros stay zero with q = 1
    const bool real = d < a.dreal;
    r[H64_VH * 8] = real ? a.v[p][d] * scr[2 * p] : 0.0;
    r[H64_XI * 8] = real ? a.xi[p][d] : 0.0;
    r[H64_IL * 8] = real ? 1.0 / a.lam[p][d] : 1.0;  // one multiply per element instead of a division
    r[H64_DL * 8] = real ? a.d[p][d] : 1.0;
    r[H64_GM * 8] = real ? a.g[p][d] : 0.0;
  }
  if (threadIdx.x == 0) {
    double c = 0.0;
    for (int p = 0; p < n; ++p) c += scr[2 * p + 1];
    *ctot = c;
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

template <int D, int U, bool LADJ>
__device__ __forceinline__ void h64_pair(double (&x)[U][8], double (&acc)[U], const double* __restrict__ r,
                                         const double* __restrict__ tab) {
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
  // Johnson: z = (x - xi) / lambda, y = gamma + delta asinh(z), ladj -= log(prod q)/2
  double pxi[8], pil[8];
  h64_param(r + H64_XI * 8, pxi);
  h64_param(r + H64_IL * 8, pil);
  double q[U][8];
  bool far = false;  // some |z| >= 2^26, Inf or NaN in this lane
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const double z = (x[u][e] - pxi[e]) * pil[e];
      x[u][e] = z;
      q[u][e] = fma(z, z, 1.0);
      far = far || !asinh64_fin_ok(z);
    }
  double pd[8], pg[8];
  h64_param(r + H64_DL * 8, pd);
  h64_param(r + H64_GM * 8, pg);
  if (!__any(far)) {
    // the whole wave in |z| < 2^26: the range-free asinh and the plain table log of the q product (the same
    // values as asinh64_tab / logprod64_tab there: the product of 8 q < 2^53 stays below 2^424)
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) x[u][e] = fma(pd[e], asinh64_tab_fin(x[u][e], tab), pg[e]);
    if (LADJ)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        double p = q[u][0];
#pragma unroll
        for (int e = 1; e < 8; ++e) p *= q[u][e];
        acc[u] -= 0.5 * log64_tab(p, 0, tab);
      }
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

template <int D, int U, int LM, bool TAIL, bool PAD>
__device__ __forceinline__ void h64_tile(const HJ64Args& a, const double* __restrict__ rec, const double* tab,
                                         double ctot, double* stage, int64_t col0, double (&x)[U][8],
                                         const double (&old)[H64Lay<D, U>::NLS]) {
  double acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = 0.0;
  for (int p = 0; p < a.n; ++p) h64_pair<D, U, (LM > 0)>(x, acc, rec + (size_t)p * kHj64W * D, tab);
  h64_store<D, U, LM, TAIL, PAD>(a, ctot, col0, x, acc, old, stage);
}

// OCC: minimum waves per SIMD the register allocation must allow (1: no constraint; the D = 32 / 64 program
// takes 140 VGPRs, 3 waves per SIMD; OCC = 4 caps it at 128)
template <int D, int U, int LM, bool PAD = false, int OCC = 1>
__global__ __launch_bounds__(256, OCC) void flow_hj64_kernel(HJ64Args a) {
  using L = H64Lay<D, U>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* scr = reinterpret_cast<double*>(smem);
  double* ctotp = scr + 2 * kHj64MaxPairs;
  double* tab = reinterpret_cast<double*>(smem + kHj64Scratch);
  double* stage = reinterpret_cast<double*>(smem + kHj64Scratch + kHj64Tab) + (threadIdx.x >> 6) * kStagePerWave;
  double* rec = reinterpret_cast<double*>(smem + kHj64Header);
  build_hj64_program<D>(a, rec, scr, tab, ctotp);
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
      h64_tile<D, U, LM, false, PAD>(a, myrec, tab, ctot, stage, t * CT, xa, old);
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
    h64_tile<D, U, LM, true, PAD>(a, myrec, tab, ctot, stage, c0, xa, old);
  }
}

template <int D, int U, int LM, bool PAD = false, int OCC = 1>
static hipError_t launch_hj64(const HJ64Args& h, hipStream_t st, const DeviceInfo& dev) {
  const size_t lds = hj64_lds_bytes(D, h.n);
  const void* k = reinterpret_cast<const void*>(&flow_hj64_kernel<D, U, LM, PAD, OCC>);
  int64_t blocks = 0;
  hipError_t e = frag_grid(k, h.N, (int64_t)H64Lay<D, U>::TC * 4, lds, dev, &blocks);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((flow_hj64_kernel<D, U, LM, PAD, OCC>), dim3((unsigned)blocks), dim3(256), lds, st, h);
  return hipGetLastError();
}

template <int D, bool PAD>
static hipError_t launch_hj64_lm(const HJ64Args& h, int lm, hipStream_t st, const DeviceInfo& dev) {
#if ENF_DIAG
  // ENF_HJ64_OCC (diagnostics build): 4 = the register allocation capped for 4 waves per SIMD (A/B)
  static const int occ = ENF_KNOB("ENF_HJ64_OCC", 1);
  if (occ == 4 && lm == 1 && !PAD && D <= 64) return launch_hj64<D, 1, 1, false, 4>(h, st, dev);
#endif
  if (lm == 0) return launch_hj64<D, 1, 0, PAD>(h, st, dev);
  if (lm == 1) return launch_hj64<D, 1, 1, PAD>(h, st, dev);
  return launch_hj64<D, 1, 2, PAD>(h, st, dev);
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
  const bool pad = dl != a.D;
  if (dl == 32) return pad ? launch_hj64_lm<32, true>(h, lm, st, dev) : launch_hj64_lm<32, false>(h, lm, st, dev);
  if (dl == 64) return pad ? launch_hj64_lm<64, true>(h, lm, st, dev) : launch_hj64_lm<64, false>(h, lm, st, dev);
  if (dl == 128) return pad ? launch_hj64_lm<128, true>(h, lm, st, dev) : launch_hj64_lm<128, false>(h, lm, st, dev);
  return hipErrorNotSupported;
}

}  // namespace enf
