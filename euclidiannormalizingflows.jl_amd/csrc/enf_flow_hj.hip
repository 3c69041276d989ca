// enf_flow_hj.hip -- the compiled (J o H)^n program (enf_hj.h: layouts, records, pair loop, the streaming
// kernel flow_hj_kernel) launched for configs 3-5, and the compiled inverse program (J^-1, H)^n below.
// (The variants measured and rejected in rounds 1-5 -- the wave-specialised and mailbox kernels, the other
// asinh forms -- are described in docs/HISTORY.md; round 6 removed their sources.)
#include "enf_hj.h"

namespace enf {

// ---------------------------------------------------------------------------------------------------
// The inverse program (round 4): inverse(J_n o H_n o ... o J_1 o H_1) = H_1 o J_1^-1 o ... o H_n o J_n^-1
// (src/johnson_trafo.jl:82 inverse(JohnsonTrafo) = JohnsonTrafoInv, src/householder_trafo.jl:153-154 a single
// reflection is its own inverse), i.e. the layers J^-1, H, J^-1, H, ... applied in this order, fp32, the
// layouts of the forward program (D = 32 / 64 / 128, padded or not), fused in one launch. Per pair p:
//   w   = (y - gamma)/delta                                                            (johnson_trafo.jl:36)
//   sh  = sinh(w): |w| < 1/2: w (1 + w^2/6 + w^4/120 + w^6/5040) (truncation < 1e-8 relative),
//         else H - 1/(4H), H = E/2 = exp2(w log2 e - 1) -- both odd in w, merged branch-free by a mask from w^2
//   x   = lambda sh + xi                      the JohnsonTrafoInv output              (johnson_trafo.jl:36)
//   ladj += -log|delta/lambda| + log(1 + sh^2)/2: the reference's -johnsontrafo_ladj of the output
//         (johnson_trafo.jl:103-104), whose (x - xi)/lambda is sh up to the rounding of x; the constant part
//         once per column (ctot), +1/2 log2 of the product of the q = 1 + sh^2 of a lane's 8 rows over all
//         pairs (one log2 per lane and column per tile, round 6)
//   dot = vh'x, x -= dot vh                   householder_trafo! (householder_trafo.jl:8-11)
// Round 6: the hop x -> H -> the next pair's w is folded into per-row constants as in the forward program
// (enf_hj.h): the tile carries sh between pairs, and every hop is dot = W'sh, v = fma(-dot, C, fma(sh, B, A)),
// the same three operations as the forward's front (hj_front), with (entry records E_p, p = 1 .. n)
//   p < n: W = vh_{p-1} lambda_{p-1}, B = lambda_{p-1}/delta_p, A = ((H_{p-1} xi_{p-1}) - gamma_p)/delta_p,
//          C = vh_{p-1}/delta_p                                    (v = w_p, the next pair's argument)
//   p = n: W = vh_{n-1} lambda_{n-1}, B = lambda_{n-1}, A = H_{n-1} xi_{n-1}, C = vh_{n-1}   (v = the output)
// and E_0 = {0, 1/delta_0, -gamma_0/delta_0, 0} applied to the input without a dot: 3 instead of 4 dependent
// operations per element and hop. Records built in double; the multipliers of tile registers one slot rotated
// (hj_rot). A tile whose q product overflows (|sh| ~ 2^16 on every row, Inf, NaN) is redone from X elementwise
// (exact-range sinh, log2 per element: ladj +Inf where the reference's fp32 1 + z^2 overflows).

template <int D, int R>
__device__ void build_hji_program(const HJArgs& a, int n, float* __restrict__ rec, double* __restrict__ scr,
                                  float* ctot) {
  constexpr int NF = R / 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // v'v, sum_d log|delta/lambda| (johnson_trafo.jl:41) and v'xi (the reflection of the shift xi, folded into A)
  for (int p = wave; p < n; p += nw) {
    const float* v = a.v[p];
    double vv = 0.0, cl = 0.0, vx = 0.0;
    for (int d = lane; d < a.dreal; d += 64) {
      const double vd = v[d];
      vv += vd * vd;
      cl += log(fabs((double)a.d[p][d])) - log(fabs((double)a.lam[p][d]));
      vx += vd * (double)a.xi[p][d];
    }
    for (int m = 32; m >= 1; m >>= 1) {
      vv += __shfl_xor(vv, m);
      cl += __shfl_xor(cl, m);
      vx += __shfl_xor(vx, m);
    }
    if (lane == 0) {
      const double hs = sqrt(2.0 / vv);
      scr[3 * p] = hs;
      scr[3 * p + 1] = cl;
      scr[3 * p + 2] = hs * vx;  // vh'xi
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < (n + 1) * D; i += blockDim.x) {
    const int p = i / D, d = i % D;
    const int h = d / (D / NF), w = d % (D / NF), g = w / 4, e = w % 4;
    float* r = rec + (size_t)p * kHjW * D + g * kHjW * R + 4 * h;
    // a padded row (d >= dreal): W = C = 0, B = 1, A = 0 -- its zeros stay zero with q = 1 (ladj 0)
    double q[kHjW] = {0.0, 1.0, 0.0, 0.0};
    if (d < a.dreal) {
      if (p == 0) {
        const double id = 1.0 / (double)a.d[0][d];
        q[HJ_B] = id;
        q[HJ_A] = -(double)a.g[0][d] * id;
      } else {
        const double vh = (double)a.v[p - 1][d] * scr[3 * (p - 1)];
        const double lm = (double)a.lam[p - 1][d];
        const double hx = (double)a.xi[p - 1][d] - vh * scr[3 * (p - 1) + 2];  // (H_{p-1} xi_{p-1})_d
        const double id = p < n ? 1.0 / (double)a.d[p][d] : 1.0;
        const double gm = p < n ? (double)a.g[p][d] : 0.0;
        q[HJ_W] = vh * lm;
        q[HJ_B] = lm * id;
        q[HJ_A] = (hx - gm) * id;
        q[HJ_C] = vh * id;
      }
    }
#pragma unroll
    for (int k = 0; k < kHjW; ++k) r[k * R + (hj_rotated(k) ? hj_rot(e) : e)] = (float)q[k];
  }
  if (threadIdx.x == 0) {
    double c = 0.0;
    for (int p = 0; p < n; ++p) c -= scr[3 * p + 1];  // -johnsontrafo_ladj: -log|delta/lambda|
    *ctot = (float)c;
  }
  __syncthreads();
}

// sinh(w) for |w| < 1/2 (the Taylor form) and w^2 < 1/4 as an all-ones mask (the integer difference of the
// bit patterns of w^2 and 1/4 is negative exactly when w^2 < 1/4)
__device__ __forceinline__ float sinh_small(float w, float w2) {
  return w * fmaf(w2, fmaf(w2, fmaf(w2, 1.0f / 5040.0f, 1.0f / 120.0f), 1.0f / 6.0f), 1.0f);
}
__device__ __forceinline__ uint32_t sinh_small_mask(float w2) {
  return (uint32_t)((int32_t)(__builtin_bit_cast(uint32_t, w2) - 0x3E800000u) >> 31);
}

// The input's entry E_0: w_0 = fma(y, 1/delta_0, -gamma_0/delta_0) (no reflection before the first J^-1)
template <int R, int U>
__device__ __forceinline__ void hji_entry0(float (&x)[U][R], const HJParams<R>& prm) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) x[u][e] = fmaf(x[u][e], prm.m(HJ_B, e), prm.m(HJ_A, e));
}

// One pair (J^-1, then the folded hop H -> next) on the register tile, fast form: x holds w_p on entry and w_{p+1}
// (after the last pair: the output) on exit; prm holds entry record E_p's successor on exit (r advanced). prod[u]
// accumulates the product of the q of the lane's rows of column u.
template <int D, int R, int U>
__device__ __forceinline__ void hji_pair_fast(float (&x)[U][R], float (&prod)[U], const float*& r, HJParams<R>& prm) {
  r += kHjW * D;
  float w[U][R], E[U][R], rE[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) {
      w[u][e] = x[u][e];
      E[u][e] = fmaf(w[u][e], (float)kLog2e, -1.0f);  // exp2 of this is E/2
    }
  // wave priority 3 around the transcendental groups, as in hj_pair_fast
  __builtin_amdgcn_s_setprio(3);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if constexpr (R == 8) {
      float t[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) t[e] = E[u][e];
      exp2_8(E[u], t);
    } else {
#pragma unroll
      for (int e = 0; e < R; ++e) E[u][e] = hw_exp2(E[u][e]);
    }
  }
  __builtin_amdgcn_s_setprio(0);
  uint32_t msk[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) {
      const float w2 = w[u][e] * w[u][e];
      msk[u][e] = sinh_small_mask(w2);
      w[u][e] = sinh_small(w[u][e], w2);
    }
  __builtin_amdgcn_s_setprio(3);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if constexpr (R == 8) {
      rcp8(rE[u], E[u]);
    } else {
#pragma unroll
      for (int e = 0; e < R; ++e) rE[u][e] = hw_rcp(E[u][e]);
    }
  }
  __builtin_amdgcn_s_setprio(0);
  float q[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u) {
#pragma unroll
    for (int e = 0; e < R; ++e) {
      // (E - 1/E)/2 = E/2 - 1/(4 E/2): one fma on the halved exponential and its reciprocal
      x[u][e] = asinh2_pick(w[u][e], fmaf(-0.25f, rE[u][e], E[u][e]), msk[u][e]);
      q[u][e] = fmaf(x[u][e], x[u][e], 1.0f);
    }
    prod[u] *= prod_tree<R>(q[u]);
  }
  prm.load(r);  // E_{p+1} (read once the sinh's temporaries are dead: 10 VGPRs spilled when read before it)
  hj_front<D, R, U>(x, prm);
}

// The same pair elementwise over the whole fp32 range: sinh finite up to |w| ~ 89.4 (E/2 formed as
// exp2(|w| log2 e - 1)), the ladj's log2 per element (+Inf where 1 + sh^2 overflows, as the reference's).
template <int D, int R, int U>
__device__ __forceinline__ void hji_pair_exact(float (&x)[U][R], float (&acc)[U], const float*& r, HJParams<R>& prm) {
  r += kHjW * D;
  prm.load(r);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) {
      const float w = x[u][e];
      const float aw = fabsf(w);
      const float h = hw_exp2(fmaf(aw, (float)kLog2e, -1.0f));
      const float big = copysignf(fmaf(-0.25f, hw_rcp(h), h), w);
      const float sh = aw < 0.5f ? sinh_small(w, w * w) : big;
      x[u][e] = sh;
      acc[u] = fmaf(0.5f, hw_log2(fmaf(sh, sh, 1.0f)), acc[u]);
    }
  hj_front<D, R, U>(x, prm);
}

template <int D, int R, int U, int LM, bool PAD>
struct HJIBody {
  const HJArgs& a;
  const float* rec;
  float ctot;
  float* stage;
  int n;

  template <bool TAIL, int DBG>
  __device__ __forceinline__ void tile(int64_t col0, float (&x)[U][R], const float (&old)[HJLay<D, R, U>::NLS]) {
    float acc[U], prod[U];
#pragma unroll
    for (int u = 0; u < U; ++u) prod[u] = 1.f;
    const float* r = rec;
    HJParams<R> prm;
    prm.load(r);
    hji_entry0<R, U>(x, prm);
    for (int p = 0; p < n; ++p) hji_pair_fast<D, R, U>(x, prod, r, prm);
    if (__builtin_expect(hj_redo<HJLay<D, R, U>::G>(prod), 0)) {
      hj_load<D, R, U, TAIL, DBG, PAD>(a, col0, x);
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = 0.f;
      r = rec;
      prm.load(r);
      hji_entry0<R, U>(x, prm);
      for (int p = 0; p < n; ++p) hji_pair_exact<D, R, U>(x, acc, r, prm);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = 0.5f * hw_log2(prod[u]);
    }
    hj_store<D, R, U, LM, TAIL, DBG, PAD>(a, ctot, col0, x, acc, old, stage);
  }
};

template <int D, int R, int U, int LM, bool PAD>
__global__ __launch_bounds__(256, 4) void flow_hji_kernel(HJArgs a) {
  const int n = a.n;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* scr = reinterpret_cast<double*>(smem);
  float* ctotp = reinterpret_cast<float*>(scr + 3 * kHjMaxPairs);
  float* stage = reinterpret_cast<float*>(smem + kHjScratch) + (threadIdx.x >> 6) * kStagePerWave;
  float* rec = reinterpret_cast<float*>(smem + kHjHeader);
  build_hji_program<D, R>(a, n, rec, scr, ctotp);
  constexpr int G = HJLay<D, R, U>::G;
  HJIBody<D, R, U, LM, PAD> body{a, rec + ((threadIdx.x & 63) % G) * kHjW * R, *ctotp, stage, n};
  hj_stream<D, R, U, LM, 0, PAD>(a, body);
}

// (J o H)^n flows for the compiled programs (fp32 enf_flow_hj.hip, fp64 enf_flow_hj64.hip): the layout D
// (a.dk on the padded fragment path, else a.D) 32, 64 or 128
int hj_program_pairs(const FlowArgs& a) {
  const int dl = a.dk ? a.dk : a.D;
  if (!a.frag || (dl != 32 && dl != 64 && dl != 128) || a.nsteps < 2 || (a.nsteps & 1)) return 0;
  for (int s = 0; s < a.nsteps; ++s) {
    const int want = (s & 1) ? OP_JOHNSON : OP_HOUSEHOLDER;
    if (a.steps[s].op != want) return 0;
  }
  return a.nsteps / 2;
}




template <int LM>
static hipError_t dispatch_hj(const HJArgs& a, int D, int dbg, hipStream_t st, const DeviceInfo& dev) {
#if ENF_DIAG
  // diagnostics build only: ENF_DEBUG_MODE 1 = synthesized tile, 2 = no stores either (compute-only timing);
  // ENF_HJ_R16 = 16 rows per lane, one column per lane tile (two lanes per column at D = 32; spills at this record
  // count)
  if (a.dreal == D && LM == 1) {
    static const int r16 = ENF_KNOB("ENF_HJ_R16", 0);
    if (dbg == 1) return launch_hj<32, 8, 2, 1, 4, 1>(a, st, dev);
    if (dbg == 2) return launch_hj<32, 8, 2, 1, 4, 2>(a, st, dev);
    if (r16 && D == 32) return launch_hj<32, 16, 1, 1, 4>(a, st, dev);
    if (r16 && D == 64) return launch_hj<64, 16, 1, 1, 4>(a, st, dev);
  }
#else
  (void)dbg;
#endif
  // padded layout (round 3): D = 24 / 100 / 36 ... on the next power of two, rows past a.dreal inert
  if (a.dreal != D) {
    if (D == 32) return launch_hj<32, 8, 2, LM, 4, 0, true>(a, st, dev);
    if (D == 64) return launch_hj<64, 8, 2, LM, 4, 0, true>(a, st, dev);
    return launch_hj<128, 8, 2, LM, 4, 0, true>(a, st, dev);
  }
  if (D == 128) return launch_hj<128, 8, 2, LM, 4>(a, st, dev);
  if (D == 32) return launch_hj<32, 8, 2, LM, 4>(a, st, dev);
  return launch_hj<64, 8, 2, LM, 4>(a, st, dev);
}

// (J^-1, H)^n flows -- inverse((J o H)^n) -- for the compiled inverse program (fp32)
int hji_program_pairs(const FlowArgs& a) {
  const int dl = a.dk ? a.dk : a.D;
  if (!a.frag || (dl != 32 && dl != 64 && dl != 128) || a.nsteps < 2 || (a.nsteps & 1)) return 0;
  for (int s = 0; s < a.nsteps; ++s) {
    const int want = (s & 1) ? OP_HOUSEHOLDER : OP_JOHNSON_INV;
    if (a.steps[s].op != want) return 0;
  }
  return a.nsteps / 2;
}

template <int D, int LM, bool PAD>
static hipError_t launch_hji(const HJArgs& h, hipStream_t st, const DeviceInfo& dev) {
  constexpr int R = 8, U = 2;
  const size_t lds = hj_lds_bytes(D, h.n);
  const void* k = reinterpret_cast<const void*>(&flow_hji_kernel<D, R, U, LM, PAD>);
  int64_t blocks = 0;
  hipError_t e = frag_grid(k, h.N, (int64_t)HJLay<D, R, U>::TC * 4, lds, dev, &blocks);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((flow_hji_kernel<D, R, U, LM, PAD>), dim3((unsigned)blocks), dim3(256), lds, st, h);
  return hipGetLastError();
}

template <int LM>
static hipError_t dispatch_hji(const HJArgs& h, int D, hipStream_t st, const DeviceInfo& dev) {
  if (h.dreal != D) {
    if (D == 32) return launch_hji<32, LM, true>(h, st, dev);
    if (D == 64) return launch_hji<64, LM, true>(h, st, dev);
    return launch_hji<128, LM, true>(h, st, dev);
  }
  if (D == 32) return launch_hji<32, LM, false>(h, st, dev);
  if (D == 64) return launch_hji<64, LM, false>(h, st, dev);
  return launch_hji<128, LM, false>(h, st, dev);
}

hipError_t launch_hji_program(const FlowArgs& a, int lm, hipStream_t st, const DeviceInfo& dev) {
  const int n = hji_program_pairs(a);
  if (n < 1 || n > kHjMaxPairs) return hipErrorNotSupported;
  HJArgs h;
  memset(&h, 0, sizeof h);
  h.X = a.X;
  h.Y = a.Y;
  h.ladj = a.ladj;
  h.N = a.N;
  h.n = n;
  h.dreal = a.D;
  for (int p = 0; p < n; ++p) {
    const LayerDesc& J = a.layers[a.steps[2 * p].layer];
    const Step& sh = a.steps[2 * p + 1];
    h.v[p] = (const float*)a.layers[sh.layer].p[0] + (int64_t)sh.col * a.D;
    h.g[p] = (const float*)J.p[0];
    h.d[p] = (const float*)J.p[1];
    h.xi[p] = (const float*)J.p[2];
    h.lam[p] = (const float*)J.p[3];
  }
  const int dl = a.dk ? a.dk : a.D;
  if (lm == 0) return dispatch_hji<0>(h, dl, st, dev);
  if (lm == 1) return dispatch_hji<1>(h, dl, st, dev);
  return dispatch_hji<2>(h, dl, st, dev);
}

hipError_t launch_hj_program(const FlowArgs& a, int lm, int dbg, hipStream_t st, const DeviceInfo& dev) {
  const int n = hj_program_pairs(a);
  if (n < 1 || n > kHjMaxPairs) return hipErrorNotSupported;
  const int dl = a.dk ? a.dk : a.D;
  if (dl != a.D && dbg != 0) return hipErrorNotSupported;  // (diagnostics variants: unpadded only)
  HJArgs h;
  memset(&h, 0, sizeof h);
  h.X = a.X;
  h.Y = a.Y;
  h.ladj = a.ladj;
  h.N = a.N;
  h.n = n;
  h.dreal = a.D;
  for (int p = 0; p < n; ++p) {
    const Step& sh = a.steps[2 * p];
    const LayerDesc& J = a.layers[a.steps[2 * p + 1].layer];
    h.v[p] = (const float*)a.layers[sh.layer].p[0] + (int64_t)sh.col * a.D;
    h.g[p] = (const float*)J.p[0];
    h.d[p] = (const float*)J.p[1];
    h.xi[p] = (const float*)J.p[2];
    h.lam[p] = (const float*)J.p[3];
  }
  if (lm == 0) return dispatch_hj<0>(h, dl, dbg, st, dev);
  if (lm == 1) return dispatch_hj<1>(h, dl, dbg, st, dev);
  return dispatch_hj<2>(h, dl, dbg, st, dev);
}

}  // namespace enf
