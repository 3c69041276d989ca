// enf_steps.h -- per-layer parameter records and the per-fragment step bodies shared by the
// fused flow kernels (enf_flow.hip: fragment-layout interpreter; enf_flow_wy.hip: dense-Householder
// MFMA kernel). See enf_flow.hip's header for the layout and arithmetic notes.
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <type_traits>

#include "enf_frag.h"
#include "enf_math64.h"
#include "enf_internal.h"
#include "enf_logtab.h"

namespace enf {

// The fp64 log reduction table (enf_math64.h log64_tab) in LDS: copied from constant memory by
// build_program in every fp64 kernel that runs the fragment steps (3 KB).
static __shared__ double g_logtab[3 * kLogTabN];

// ------------------------------------------------------------------------------------------
// parameter records in LDS
// ------------------------------------------------------------------------------------------
// A step's record holds W(op) parameter values per row (enf_internal.h record_width):
//  fp32                                              fp64
//  HOUSEHOLDER  W=1 {v_d * sqrt(2/v'v)}              same
//  SCALESHIFT   W=2 {a, b}                           same
//  JOHNSON      W=4 {gamma, delta*ln2, xi, 1/lambda} {gamma, delta, xi, 1/lambda}
//  JOHNSON_INV  W=4 {gamma, 1/delta, xi, lambda}     {gamma, 1/delta, xi, lambda}
//  CENTER_*     W=8 {b*log2e, c, ln2/b, exp(b*a),    {a, b, c, exp(b*a), exp(2*b*a), exp(-b*a), 1/b, 0}
//                    exp(2*b*a), b*a*log2e, a, b}
// Layout: [group g][param q][element e] with RV elements per group; element (g, e) is row
// g*RV + e (D >= RV) or e % D (D < RV). The fragment kernel uses RV = V = 16/sizeof(T), so a
// lane reads each parameter of its V rows with ONE 16-byte LDS read; the generic kernel uses
// RV = 1 (row-major records). Size: W * max(D, RV) values (enf_internal.h record_elems).
template <typename T>
__device__ __forceinline__ void param_values(int op, const LayerDesc& L, int col, int D, int row, double hscale,
                                             T (&out)[8]) {
  if (op == OP_HOUSEHOLDER) {
    out[0] = (T)((double)((const T*)L.p[0])[(int64_t)col * D + row] * hscale);
  } else if (op == OP_SCALESHIFT) {
    out[0] = ((const T*)L.p[0])[row];
    out[1] = ((const T*)L.p[1])[row];
  } else if (op == OP_JOHNSON || op == OP_JOHNSON_INV) {
    const T g = ((const T*)L.p[0])[row], de = ((const T*)L.p[1])[row];
    const T xi = ((const T*)L.p[2])[row], la = ((const T*)L.p[3])[row];
    out[0] = g;
    out[2] = xi;
    if constexpr (std::is_same_v<T, float>) {
      if (op == OP_JOHNSON) {
        out[1] = (float)((double)de * kLn2);
        out[3] = (float)(1.0 / (double)la);
      } else {
        out[1] = (float)(1.0 / (double)de);
        out[3] = la;
      }
    } else {  // reciprocals in the prologue: one multiply per element instead of a division
      out[1] = op == OP_JOHNSON ? de : 1.0 / de;
      out[3] = op == OP_JOHNSON ? 1.0 / la : la;
    }
  } else {  // CENTER_STRETCH / CENTER_CONTRACT
    const T av = ((const T*)L.p[0])[row], bv = ((const T*)L.p[1])[row], cv = ((const T*)L.p[2])[row];
    if constexpr (std::is_same_v<T, float>) {
      const double b = bv, aa = av;
      out[0] = (float)(b * kLog2e);
      out[1] = cv;
      out[2] = (float)(kLn2 / b);
      out[3] = expf(bv * av);         // exp(b*a) in T, as the reference (center_stretch.jl:7)
      out[4] = expf(2.0f * bv * av);  // exp(2*b*a)
      out[5] = (float)(b * aa * kLog2e);
      out[6] = av;  // raw a, b for the generic kernel
      out[7] = bv;
    } else {
      out[0] = av;
      out[1] = bv;
      out[2] = cv;
      // the row constants of center_stretch.jl:7, once per row instead of per element (round 4): the same
      // double operations as the per-element expressions they replace, so the same values
      out[3] = exp(bv * av);
      out[4] = exp(2.0 * bv * av);
      out[5] = exp(-bv * av);  // CenterContract: exp(-b(xu + a)) = exp(-b a) / exp(b xu) (round 4)
      out[6] = 1.0 / bv;       // the in-range paths multiply by it instead of dividing (round 4, last session)
      out[7] = 0.0;
    }
  }
}

// Block prologue: one wave per step. Pass 1 reduces over the D distinct rows (v'v for a
// reflection; the constant ladj part sum log|delta/lambda|, sum log|a| in double); pass 2 writes
// the records in the layout above. Returns ctot = sum of the per-step constants (natural log) to
// every thread. One barrier, LDS only (lds_barrier): the caller may have global loads in flight
// (the frag kernels issue their first tile before the prologue) and they are not waited for here.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Padded fragment path (a.dk != 0): D (= DC) is the power-of-two layout and Dr = a.D the real rows;
// the parameters are read and the constants summed over the Dr real rows, and the rows past Dr get
// neutral records that map the zeros those lanes hold to 0 with ladj 0: reflection v = 0, ScaleShift
// (1, 0), Johnson / JohnsonInv gamma = xi = 0, delta = lambda = 1, CenterStretch / CenterContract
// a = c = 0, b = 1 (center_stretch(0) = sign(0)... + c = 0 and center_contract(0) = 0; both ladjs are
// log|1/2 + 1/2| = 0, center_stretch.jl:4-22; exactly so in the fp32 steps: exp2(0) = 1, sqrt(4) = 2,
// log2(1) = 0, rcp(2) = 1/2).
template <typename T>
__device__ __forceinline__ void neutral_values(int op, T (&out)[8]) {
  for (int q = 0; q < 8; ++q) out[q] = (T)0;
  if (op == OP_SCALESHIFT) out[0] = (T)1;
  if (op == OP_JOHNSON || op == OP_JOHNSON_INV) {
    out[1] = (std::is_same_v<T, float> && op == OP_JOHNSON) ? (T)kLn2 : (T)1;  // delta (ln2 delta), 1/delta
    out[3] = (T)1;                                                               // 1/lambda, lambda
  }
  if (op == OP_CENTER_STRETCH || op == OP_CENTER_CONTRACT) {
    if constexpr (std::is_same_v<T, float>) {  // {b log2e, c, ln2/b, exp(ba), exp(2ba), ba log2e, a, b}
      out[0] = (float)kLog2e;
      out[2] = (float)kLn2;
      out[3] = 1.0f;
      out[4] = 1.0f;
      out[7] = 1.0f;
    } else {  // {a, b, c, exp(ba), exp(2ba), exp(-ba), 1/b}
      out[1] = 1.0;
      out[3] = 1.0;
      out[4] = 1.0;
      out[5] = 1.0;
      out[6] = 1.0;
    }
  }
}

template <typename T, int DC, int RV>
__device__ double build_program(const FlowArgs& a, T* __restrict__ rec, double* __restrict__ stepc) {
  const int D = DC > 0 ? DC : a.D;
  const int Dr = a.dk ? a.D : D;  // real rows
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int nent = D > RV ? D : RV;  // record entries per parameter
  if constexpr (std::is_same_v<T, double>)
    for (int i = threadIdx.x; i < 3 * kLogTabN; i += blockDim.x) g_logtab[i] = kLogTab[i];
  for (int s = wave; s < a.nsteps; s += nw) {
    const Step st = a.steps[s];
    if (st.op == OP_DENSE) {  // built by the dense kernel's own prologue; no ladj constant
      if (lane == 0) stepc[s] = 0.0;
      continue;
    }
    const LayerDesc& L = a.layers[st.layer];
    const int W = record_width(st.op);
    T* r = rec + st.off;
    double part = 0.0;
    for (int d = lane; d < Dr; d += 64) {
      if (st.op == OP_HOUSEHOLDER) {
        const double v = (double)((const T*)L.p[0])[(int64_t)st.col * Dr + d];
        part += v * v;
      } else if (st.op == OP_SCALESHIFT) {
        // scale_shift_trafo.jl:22, summed over a's own length (k = 1: a length-1 a broadcast to the rows)
        if (L.k != 1 || d == 0) part += log(fabs((double)((const T*)L.p[0])[d]));
      } else if (st.op == OP_JOHNSON || st.op == OP_JOHNSON_INV) {
        // log|delta/lambda| (johnson_trafo.jl:41,51); the inverse negates (johnson_trafo.jl:104)
        const double c = log(fabs((double)((const T*)L.p[1])[d])) - log(fabs((double)((const T*)L.p[3])[d]));
        part += st.op == OP_JOHNSON ? c : -c;
      }
    }
    // lanes >= D hold 0: log2(D) butterfly stages put the total in lane 0 (D = 2: one stage), then
    // lane 0's value is made wave-uniform
    for (int m = 1; m < D && m < 64; m <<= 1) part += __shfl_xor(part, m);
    {
      const uint64_t pb = __builtin_bit_cast(uint64_t, part);
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)pb), hi = __builtin_amdgcn_readfirstlane((uint32_t)(pb >> 32));
      part = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
    }
    // normalised reflection: H x = x - vh (vh'x), vh = v*sqrt(2/v'v) (householder_trafo.jl:9-10)
    const double hscale = st.op == OP_HOUSEHOLDER ? sqrt(2.0 / part) : 0.0;
    for (int i = lane; i < nent; i += 64) {
      const int g = D >= RV ? i / RV : 0, e = i % RV;
      const int row = D >= RV ? i : e % D;
      T vals[8];
      if (row < Dr) param_values<T>(st.op, L, st.col, Dr, row, hscale, vals);
      else neutral_values<T>(st.op, vals);
      for (int q = 0; q < W; ++q) r[(g * W + q) * RV + e] = vals[q];
    }
    if (lane == 0)
      stepc[s] = (st.op == OP_HOUSEHOLDER || st.op == OP_CENTER_STRETCH || st.op == OP_CENTER_CONTRACT) ? 0.0 : part;
  }
  lds_barrier();
  double c = 0.0;  // every thread sums the (broadcast) LDS values: no second barrier
  for (int s = 0; s < a.nsteps; ++s) c += stepc[s];
  return c;
}

// Per-wave prologue of the small-D fragment kernels (round 5; D <= 2 and nsteps * D <= 64): the same records and
// the same constant as build_program, built by ONE wave into its own LDS slice with no block barrier -- lane
// s * D + d handles row d of step s (its parameter loads, the double logs, the reflection's v'v over the D
// adjacent lanes) -- so no wave waits for the others, and the steps' global round trips overlap instead of
// running one step per wave. The fp64 log table is written by every wave (the same values to the same
// addresses: no barrier needed either).
template <typename T, int RV>
__device__ double build_program_wave(const FlowArgs& a, T* __restrict__ rec) {
  const int lane = threadIdx.x & 63;
  const int D = a.D;  // 1 or 2 (no padded layout here)
  if constexpr (std::is_same_v<T, double>)
    for (int i = lane; i < 3 * kLogTabN; i += 64) g_logtab[i] = kLogTab[i];
  const int s = lane / D, d = lane % D;
  const bool live = s < a.nsteps;
  const Step st = a.steps[live ? s : 0];
  const LayerDesc& L = a.layers[st.layer];
  double part = 0.0;
  if (live) {
    if (st.op == OP_HOUSEHOLDER) {
      const double v = (double)((const T*)L.p[0])[(int64_t)st.col * D + d];
      part = v * v;
    } else if (st.op == OP_SCALESHIFT) {
      if (L.k != 1 || d == 0) part = log(fabs((double)((const T*)L.p[0])[d]));
    } else if (st.op == OP_JOHNSON || st.op == OP_JOHNSON_INV) {
      const double c = log(fabs((double)((const T*)L.p[1])[d])) - log(fabs((double)((const T*)L.p[3])[d]));
      part = st.op == OP_JOHNSON ? c : -c;
    }
  }
  if (D == 2) part += __shfl_xor(part, 1);  // the step's two rows, as build_program's one butterfly stage
  const double hscale = (live && st.op == OP_HOUSEHOLDER) ? sqrt(2.0 / part) : 0.0;
  if (live && st.op != OP_DENSE) {
    const int W = record_width(st.op);
    T* r = rec + st.off;
    T vals[8];
    param_values<T>(st.op, L, st.col, D, d, hscale, vals);
    for (int e = d; e < RV; e += D)  // D < RV: the row's value fills every element e with e % D == d
      for (int q = 0; q < W; ++q) r[q * RV + e] = vals[q];
  }
  const double cs = (live && (st.op == OP_SCALESHIFT || st.op == OP_JOHNSON || st.op == OP_JOHNSON_INV)) ? part : 0.0;
  // the constants summed in step order (lane s * D holds step s's): uniform loop of readlanes
  double c = 0.0;
  for (int k = 0; k < a.nsteps; ++k) {
    const uint64_t b = __builtin_bit_cast(uint64_t, cs);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, k * D), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), k * D);
    c += __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's LDS writes land before its reads
  __builtin_amdgcn_wave_barrier();
  return c;
}

// y = x - vh (vh'x), vh = v*sqrt(2/v'v): householder_trafo!(y, v, x) (householder_trafo.jl:8-11)
template <typename T, int D, int U>
__device__ __forceinline__ void step_householder(Tile<T, D, U>& x, const T* __restrict__ r) {
  ENF_FRAG_CONSTS
  T vh[V];
  lds_vec<T, V>(r, vh);
  T dot[U][CPF];
  tile_dots<T, D, U>(x, vh, dot);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < V; ++e) x[u][e] = fma(-dot[u][e / SEG], vh[e], x[u][e]);
}

// fp32 Johnson layer from z (in x): y = gamma + delta*asinh(z), ladj += log|delta/lambda| -
// log(1+z^2)/2 (the constant part is in ctot). zmax = max |z| over the tile.
template <int D, int U, bool LADJ>
__device__ __forceinline__ void johnson_from_z(Tile<float, D, U>& x, Acc<float, D, U>& acc,
                                               const float (&pg)[4], const float (&pd)[4], float zmax) {
  using T = float;
  ENF_FRAG_CONSTS
        if (__builtin_expect(!(zmax <= 32768.f), 0)) {
#pragma unroll
          for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < V; ++e) {
              const YL r2 = johnson_fwd_f32_slow(x[u][e], pg[e], pd[e]);
              x[u][e] = r2.y;
              if (LADJ) acc[u][e / SEG] += r2.l;
            }
        } else {
          const uint32_t csign = sign_mask_vgpr();
#pragma unroll
          for (int u = 0; u < U; ++u) {
            float prod[CPF];
#pragma unroll
            for (int c = 0; c < CPF; ++c) prod[c] = 1.0f;
#pragma unroll
            for (int e = 0; e < V; ++e) {
              const float z = x[u][e];
              const float q = fmaf(z, z, 1.0f);
              x[u][e] = fmaf(pd[e], asinh2_f32(z, q, hw_sqrt(q), csign), pg[e]);
              prod[e / SEG] *= q;
            }
            if (LADJ)
#pragma unroll
              for (int c = 0; c < CPF; ++c) acc[u][c] = fmaf(-0.5f, hw_log2(prod[c]), acc[u][c]);
          }
        }
}

template <typename T, int D, int U, bool LADJ>
__device__ __forceinline__ void step_johnson(Tile<T, D, U>& x, Acc<T, D, U>& acc,
                                             const T* __restrict__ r) {
  ENF_FRAG_CONSTS
  T pg[V], pd[V], px[V], pl[V];
  lds_vec<T, V>(r, pg);
  lds_vec<T, V>(r + V, pd);
  lds_vec<T, V>(r + 2 * V, px);
  lds_vec<T, V>(r + 3 * V, pl);
      if constexpr (std::is_same_v<T, float>) {
        // y = gamma + delta*asinh(z), asinh|z| = ln2*log2(|z| + sqrt(1+z^2))  (johnson_trafo.jl:31)
        // ladj: log|delta/lambda| - log(1+z^2)/2, one log2 of the product of the q = 1+z^2 of a
        // fragment's rows                                                    (johnson_trafo.jl:41,51)
        // Pass 1: z for the whole tile (in place) and its largest |z|; the product of <= 4 q stays
        // finite for |z| <= 2^15, larger or infinite |z| take the exact elementwise path (one
        // uniform branch per tile, so the fast path interleaves all U*V elements). NaN needs no
        // special path: it propagates through the fast formulas as through the reference's.
        float zmax = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int e = 0; e < V; ++e) {
            x[u][e] = (x[u][e] - px[e]) * pl[e];
            zmax = fmaxf(zmax, fabsf(x[u][e]));
          }
        johnson_from_z<D, U, LADJ>(x, acc, pg, pd, zmax);
      } else {
        // y = gamma + delta*asinh(z) (asinh64_tab: enf_math64.h, the table log, no reciprocal);
        // ladj: -log(prod of the fragment column segment's q = 1 + z^2)/2, one table log per segment
        // (exponents summed as integers, so no product overflows; q = +Inf gives -Inf as the
        // reference's log(1/sqrt(Inf)) does). Round 4, last session: a wave whose |z| are all below 2^26
        // takes the range-free asinh64_tab_fin (the same values there) and the plain table log of the
        // segment's q product (< 2^104), as the compiled fp64 programs do.
        bool far = false;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int e = 0; e < V; ++e) far = far || !asinh64_fin_ok((x[u][e] - px[e]) * pl[e]);
        if (!__any(far)) {
#pragma unroll
          for (int u = 0; u < U; ++u) {
            double q[V];
#pragma unroll
            for (int e = 0; e < V; ++e) {
              const double z = (x[u][e] - px[e]) * pl[e];
              x[u][e] = fma(pd[e], asinh64_tab_fin(z, g_logtab), pg[e]);
              q[e] = fma(z, z, 1.0);
            }
            if (LADJ)
#pragma unroll
              for (int c = 0; c < CPF; ++c) {
                double qp = q[c * SEG];
#pragma unroll
                for (int e = 1; e < SEG; ++e) qp *= q[c * SEG + e];
                acc[u][c] -= 0.5 * log64_tab(qp, 0, g_logtab);
              }
          }
          return;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          double q[V];
#pragma unroll
          for (int e = 0; e < V; ++e) {
            const double z = (x[u][e] - px[e]) * pl[e];
            x[u][e] = fma(pd[e], asinh64_tab(z, g_logtab), pg[e]);
            q[e] = fma(z, z, 1.0);
          }
          if (LADJ)
#pragma unroll
            for (int c = 0; c < CPF; ++c) {
              double qs[SEG];
#pragma unroll
              for (int e = 0; e < SEG; ++e) qs[e] = q[c * SEG + e];
              acc[u][c] -= 0.5 * logprod64_tab<SEG>(qs, g_logtab);
            }
        }
      }
}

template <typename T, int D, int U, bool LADJ>
__device__ __forceinline__ void step_johnson_inv(Tile<T, D, U>& x, Acc<T, D, U>& acc,
                                                 const T* __restrict__ r) {
  ENF_FRAG_CONSTS
  T pg[V], pd[V], px[V], pl[V];
  lds_vec<T, V>(r, pg);
  lds_vec<T, V>(r + V, pd);
  lds_vec<T, V>(r + 2 * V, px);
  lds_vec<T, V>(r + 3 * V, pl);
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int e = 0; e < V; ++e) {
          if constexpr (std::is_same_v<T, float>) {
            // x = lambda*sinh((y-gamma)/delta) + xi (johnson_trafo.jl:36); ladj = -ladj_fwd(x_out)
            // (johnson_trafo.jl:103-104) = -log|delta/lambda| + log(1 + sinh(w)^2)/2
            const float w = (x[u][e] - pg[e]) * pd[e];
            const float aw = fabsf(w);
            // sinh: Taylor to w^7 below |w| = 0.5 (truncation < 1e-8 relative), else (E - 1/E)/2
            const float E = hw_exp2(aw * (float)kLog2e);
            const float big = 0.5f * (E - hw_rcp(E));
            const float w2 = w * w;
            const float sm = aw * fmaf(w2, fmaf(w2, fmaf(w2, 1.0f / 5040.0f, 1.0f / 120.0f), 1.0f / 6.0f), 1.0f);
            const float sh = copysignf(aw < 0.5f ? sm : big, w);
            x[u][e] = fmaf(pl[e], sh, px[e]);
            if (LADJ) acc[u][e / SEG] = fmaf(0.5f, hw_log2(fmaf(sh, sh, 1.0f)), acc[u][e / SEG]);
          } else {
            // the reference's ladj is from the output, log(1 + ((x_out - xi)/lambda)^2)/2, and
            // (x_out - xi)/lambda = sinh(w) up to the rounding of x_out
            const double w = (x[u][e] - pg[e]) * pd[e];
            const double sh = sinh64(w);
            x[u][e] = fma(pl[e], sh, px[e]);
            if (LADJ) acc[u][e / SEG] += 0.5 * log1p64_tab(sh * sh, g_logtab);
          }
        }
      }
}

template <typename T, int D, int U>
__device__ __forceinline__ void step_scaleshift(Tile<T, D, U>& x, const T* __restrict__ r) {
  ENF_FRAG_CONSTS
      // y = muladd(x, a, b) (scale_shift_trafo.jl:16); ladj = sum log|a| (constant, in ctot)
      T pa[V], pb[V];
      lds_vec<T, V>(r, pa);
      lds_vec<T, V>(r + V, pb);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < V; ++e) x[u][e] = fma(x[u][e], pa[e], pb[e]);
}

// fp64 Center steps (round 4): the wave votes on its tile. When every |b x| (stretch) / |b (x - c)|
// (contract) is <= 200 and every row's b and exp(b a) are moderate (|b| in [1e-100, 1e100], exp(b a) in
// [1e-50, 1e50]), no exp, sqrt, reciprocal or log below can overflow, underflow or meet Inf, and the wave
// takes the in-range path: exp64_in / sqrt64_ge1 / div64 / the table log (enf_math64.h), no range selects,
// and the stretch's ladj without its two exps (b (y - c) = sign(x) log(inner), so exp(-b (yu - a)) and
// exp(b (yu + a)) are E1 / inner and E1 inner, the two swapping with the sign of x), the contract's four
// exps from one, P = exp(b xu): P / E1, Ei / P, E1 / P, P E1 (E1 = exp(b a), Ei = exp(-b a), row records).
// Any other wave runs the reference's formulas literally (ocml), the pre-round-4 code. Instruction counts
// per element (gfx950 ISA): stretch ~395 -> ~110, contract ~510 -> ~120.
template <int V>
__device__ __forceinline__ bool center_rows_moderate(const double (&bv)[V], const double (&E1)[V]) {
  bool ok = true;
#pragma unroll
  for (int e = 0; e < V; ++e)
    ok = ok && fabs(bv[e]) >= 1e-100 && fabs(bv[e]) <= 1e100 && E1[e] >= 1e-50 && E1[e] <= 1e50;
  return ok;
}

template <typename T, int D, int U, bool LADJ>
__device__ __forceinline__ void step_center_stretch(Tile<T, D, U>& x, Acc<T, D, U>& acc,
                                                    const T* __restrict__ r) {
  ENF_FRAG_CONSTS
      T rr[8][V];
#pragma unroll
      for (int q = 0; q < 8; ++q) lds_vec<T, V>(r + q * V, rr[q]);
  if constexpr (!std::is_same_v<T, float>) {
    bool in = center_rows_moderate<V>(rr[1], rr[3]);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < V; ++e) in = in && fabs(rr[1][e] * x[u][e]) <= 200.0;
    if (__all(in)) {
#pragma unroll
      for (int e = 0; e < V; ++e)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          // center_stretch.jl:4-8; ladj -contract_ladj(y) (:17-22, :41-42) as dy = 1/(1 + E1/inner) + 1/(1 + E1 inner)
          // = (inner (1 + E1 inner) + inner + E1) / ((inner + E1)(1 + E1 inner)): one division instead of three
          // (every term positive: inner >= 1, E1 > 0), and log(inner) / b as a product with the record's 1/b
          // (round 4, last session)
          const double bv = rr[1][e], c = rr[2][e], E1 = rr[3][e], E2 = rr[4][e], ib = rr[6][e];
          const double xv = x[u][e];
          const double ex = exp64_in(fabs(bv * xv));
          const double ome = 1.0 - ex;
          const double inner = (sqrt64_ge1(ome * ome * E2 + 4.0 * ex) - ome * E1) / 2.0;
          // sign(x) log(inner): inner = 1 exactly at x = +-0 (log 0, so the sign of zero only reaches -0 + c)
          x[u][e] = fma(__builtin_copysign(log64_tab(inner, 0, g_logtab), xv), ib, c);
          if (LADJ) {
            const double pe = fma(E1, inner, 1.0), ie = inner + E1;
            const double dy = div64(fma(inner, pe, ie), ie * pe);
            acc[u][e / SEG] -= log64_tab(dy, 0, g_logtab);
          }
        }
      return;
    }
  }
#pragma unroll
      for (int e = 0; e < V; ++e) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if constexpr (std::is_same_v<T, float>) {
            // center_stretch.jl:4-8 with e = exp(|b x|); ladj = -contract_ladj(y) (:41-42)
            const float bl = rr[0][e], c = rr[1][e], lnb = rr[2][e], E1 = rr[3][e], E2 = rr[4][e];
            const float xv = x[u][e];
            const float ex = hw_exp2(fabsf(xv * bl));
            const float ome = 1.0f - ex;
            const float A = fmaf(ome * ome, E2, 4.0f * ex);
            const float inner = (hw_sqrt(A) - ome * E1) * 0.5f;
            const float L = hw_log2(inner);
            const float sg = xv > 0.f ? 1.f : (xv < 0.f ? -1.f : xv);  // Julia sign()
            const float y = sg * L * lnb + c;
            x[u][e] = y;
            if (LADJ) {
              // -contract_ladj(y): exp(-b(yu - a)) and exp(b(yu + a)) are E1/inner and E1 inner (b yu = sign(x)
              // log(inner); the two swap with the sign of x), so dy = inner/(inner + E1) + 1/(1 + E1 inner) --
              // two rcp instead of two exp2 and two rcp (round 4, last session, as the fp64 in-range path). inner =
              // +Inf: Inf * rcp(Inf) is NaN and fminf takes the 1 (the reference's 1/(1 + 0)).
              const float dy = fminf(inner * hw_rcp(inner + E1), 1.0f) + hw_rcp(fmaf(E1, inner, 1.0f));
              acc[u][e / SEG] -= hw_log2(dy);
            }
          } else {
            // out of range somewhere in the wave: center_stretch.jl:4-8, :17-22 literally (ocml)
            const double av = rr[0][e], bv = rr[1][e], c = rr[2][e], E1 = rr[3][e], E2 = rr[4][e];
            const double xv = x[u][e];
            const double ex = exp(fabs(bv * xv));
            const double ome = 1.0 - ex;
            const double inner = (sqrt(ome * ome * E2 + 4.0 * ex) - ome * E1) / 2.0;
            const double sg = xv > 0. ? 1. : (xv < 0. ? -1. : xv);
            const double y = sg * log(inner) / bv + c;
            x[u][e] = y;
            if (LADJ) {
              const double yu = y - c;
              const double dy = 1.0 / (1.0 + exp(-bv * (yu - av))) + 1.0 / (1.0 + exp(bv * (yu + av)));
              acc[u][e / SEG] -= log(fabs(dy));
            }
          }
        }
      }
}

template <typename T, int D, int U, bool LADJ>
__device__ __forceinline__ void step_center_contract(Tile<T, D, U>& x, Acc<T, D, U>& acc,
                                                     const T* __restrict__ r) {
  ENF_FRAG_CONSTS
      T rr[8][V];
#pragma unroll
      for (int q = 0; q < 8; ++q) lds_vec<T, V>(r + q * V, rr[q]);
  if constexpr (!std::is_same_v<T, float>) {
    bool in = center_rows_moderate<V>(rr[1], rr[3]);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < V; ++e) in = in && fabs(rr[1][e] * (x[u][e] - rr[2][e])) <= 200.0;
    if (__all(in)) {
#pragma unroll
      for (int e = 0; e < V; ++e)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          // center_stretch.jl:11-15 / :17-22 in t = b xu (round 4, last session): with P = e^|t| and A = b a,
          // b y = log(1 + e^(t-A)) - log(1 + e^(-t-A)) is odd in t, and for t >= 0 it is
          // log1p(e^-A (P^2 - 1) / (P + e^-A)), P^2 - 1 = em (2 + em), em = expm1(|t|): one log1p of a
          // positive argument instead of a difference of two logs (which cancels near t = 0 -- this form does
          // not); dy = 1/(1 + e^(-(t-A))) + 1/(1 + e^(t+A)) is even in t, = P/(P + E1) + 1/(1 + P E1)
          // = (P (1 + P E1) + P + E1) / ((P + E1)(1 + P E1)), one division. (E1 = e^A, Ei = e^-A, ib = 1/b.)
          const double bv = rr[1][e], c = rr[2][e], E1 = rr[3][e], Ei = rr[5][e], ib = rr[6][e];
          const double t = bv * (x[u][e] - c);
          const double em = expm1_64_in(fabs(t));
          const double P = 1.0 + em;
          const double arg = div64(Ei * (em * (2.0 + em)), P + Ei);
          // (+ 0.0: the reference's difference is +0 at t = +-0, so its y is +0 / b; the product keeps that sign)
          x[u][e] = (__builtin_copysign(log1p64_tab(arg, g_logtab), t) + 0.0) * ib;
          if (LADJ) {
            const double pe = fma(P, E1, 1.0), pi = P + E1;
            const double dy = div64(fma(P, pe, pi), pi * pe);
            acc[u][e / SEG] += log64_tab(dy, 0, g_logtab);
          }
        }
      return;
    }
  }
#pragma unroll
      for (int e = 0; e < V; ++e) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if constexpr (std::is_same_v<T, float>) {
            // center_stretch.jl:11-15; ladj = contract_ladj(x) (:17-22, :65)
            const float bl = rr[0][e], c = rr[1][e], lnb = rr[2][e], bal = rr[5][e];
            const float xu = x[u][e] - c;
            const float e1 = hw_exp2(fmaf(bl, xu, -bal));   // exp(b(xu - a))
            const float e2 = hw_exp2(fmaf(-bl, xu, -bal));  // exp(-b(xu + a))
            // exp(-b(xu - a)) = 1/e1 and exp(b(xu + a)) = 1/e2, so dy = e1/(1 + e1) + e2/(1 + e2), and
            // log(1 + e1) - log(1 + e2) = log((1 + e1)/(1 + e2)): two exp2, two rcp and two log2 instead of four
            // exp2, two rcp and three log2 (round 4, last session; the output the same with or without the ladj).
            // An overflowing e (Inf * rcp(Inf) = NaN) gives its term 1 by a select on e == +Inf, as the
            // reference's 1/(1 + 0); a NaN input keeps its NaN (round 5: a min(., 1) clamp turned it into 1);
            // (1 + e1) r2 is Inf / 0 exactly where the reference's difference of logs is +-Inf.
            const float r2 = hw_rcp(1.0f + e2);
            x[u][e] = hw_log2((1.0f + e1) * r2) * lnb;
            if (LADJ) {
              const float t1 = e1 == __builtin_inff() ? 1.0f : e1 * hw_rcp(1.0f + e1);
              const float t2 = e2 == __builtin_inff() ? 1.0f : e2 * r2;
              acc[u][e / SEG] += hw_log2(t1 + t2);
            }
          } else {
            // out of range somewhere in the wave: the literal formulas (ocml)
            const double av = rr[0][e], bv = rr[1][e], c = rr[2][e];
            const double xu = x[u][e] - c;
            x[u][e] = (log(1.0 + exp(bv * (xu - av))) - log(1.0 + exp(-bv * (xu + av)))) / bv;
            if (LADJ) {
              const double dy = 1.0 / (1.0 + exp(-bv * (xu - av))) + 1.0 / (1.0 + exp(bv * (xu + av)));
              acc[u][e / SEG] += log(fabs(dy));
            }
          }
        }
      }
}

}  // namespace enf
