// enf_flow_hj.hip -- compiled program for the flows of configs 3-5:
//   J_n o H_n o ... o J_1 o H_1   (layers H_1, J_1, H_2, J_2, ... applied in this order),
// each H one Householder reflection (src/householder_trafo.jl:8-11), each J a JohnsonTrafo
// (src/johnson_trafo.jl:29-32, ladj :39-42 / :76-80), fp32, D in {32, 64}, fused in one launch:
// X is read once, Y and the per-sample ladj are written once.
//
// Folded layer constants. Inside the flow a Johnson output y = gamma + delta*asinh(z) is only ever
// consumed by the next reflection and the next Johnson layer, both affine in y. With
// L = sign(z) log2(|z| + sqrt(1 + z^2)) (= asinh(z)/ln2) and delta' = delta*ln2, y = gamma + delta' L,
// so for pair p >= 1 (vh = v*sqrt(2/v'v), the reflection x - vh (vh'x) of householder_trafo!):
//   dot = vh'y            = sum_d a_d L_d + c_p,              a_d = vh_d delta'_{p-1,d},
//                                                            c_p = sum_d vh_d gamma_{p-1,d}
//   z   = (y - dot vh - xi)/lambda
//       = L P + Q - dotL R,   P = delta'_{p-1}/lambda, Q = (gamma_{p-1} - xi - c_p vh)/lambda,
//                             R = vh/lambda                      (pair 0: a = vh, P = 1/lambda,
//                                                                 Q = -xi/lambda, L := x)
// and only the last pair forms y = gamma_n + delta'_n L. Per element and pair that is one FMA for
// the dot product, two for z, then q = 1 + z^2, sqrt, |z| + s, log2, the sign (v_bfi), and for the
// ladj -1/2 log2 of the product of a fragment's four q (one log per 4 elements). The records are
// derived in double in each block's prologue from the raw device parameter vectors.
//
// Fast-path guard: the product of a fragment's q stays finite for |z| < 2^16; a larger (or infinite)
// |z| makes it +Inf, and then the wave redoes the layer with the elementwise exact-range form
// (johnson_fwd_f32_slow in enf_frag.h: asinh finite up to FLT_MAX, ladj -Inf where the reference's
// fp32 1 + z^2 overflows). NaN propagates through the fast formulas as through the reference's.
//
// Loop structure: the pair loop is a runtime loop over one compact body (small code: the I-cache
// holds it), with the next pair's four parameter vectors read from LDS while the current one runs.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>

#include "enf_frag.h"
#include "enf_internal.h"

namespace enf {

constexpr int kHjMaxPairs = kMaxSteps / 2;
// LDS: [per pair {hs, c, cl} + ctot: doubles][ladj staging: 4 waves x kStagePerWave floats][records]
constexpr size_t kHjScratch = ((3 * kHjMaxPairs + 1) * sizeof(double) + 15) / 16 * 16;
constexpr size_t kHjHeader = kHjScratch + 4 * kStagePerWave * sizeof(float);

static size_t hj_lds_bytes(int D, int n) { return kHjHeader + (size_t)(n + 1) * 4 * D * sizeof(float); }

// Records, pair p < n: [group g = d / 4][param q in (a, P, Q, R)][e = d % 4]; record n (final):
// same layout with (gamma_{n-1}, delta'_{n-1}, 0, 0). A lane of group g reads each parameter of its
// four rows with one 16-byte LDS read.
template <int D>
__device__ void build_hj_program(const FlowArgs& a, int n, float* __restrict__ rec, double* __restrict__ scr,
                                 float* ctot) {
  constexpr int V = 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // pass 1 (one wave per pair): v'v, sum_d v_d gamma_{p-1,d}, and the constant ladj part
  // sum_d log|delta/lambda| (johnson_trafo.jl:41) in double
  for (int p = wave; p < n; p += nw) {
    const Step& sh = a.steps[2 * p];
    const LayerDesc& H = a.layers[sh.layer];
    const LayerDesc& J = a.layers[a.steps[2 * p + 1].layer];
    const float* v = (const float*)H.p[0] + (int64_t)sh.col * D;
    const float* gprev = p > 0 ? (const float*)a.layers[a.steps[2 * p - 1].layer].p[0] : nullptr;
    double vv = 0.0, cg = 0.0, cl = 0.0;
    for (int d = lane; d < D; d += 64) {
      const double vd = v[d];
      vv += vd * vd;
      if (gprev) cg += vd * (double)gprev[d];
      cl += log(fabs((double)((const float*)J.p[1])[d])) - log(fabs((double)((const float*)J.p[3])[d]));
    }
    for (int m = 32; m >= 1; m >>= 1) {
      vv += __shfl_xor(vv, m);
      cg += __shfl_xor(cg, m);
      cl += __shfl_xor(cl, m);
    }
    if (lane == 0) {
      const double hs = sqrt(2.0 / vv);  // householder_trafo.jl:9-10: 2 v (v'x) / (v'v)
      scr[3 * p] = hs;
      scr[3 * p + 1] = hs * cg;
      scr[3 * p + 2] = cl;
    }
  }
  __syncthreads();
  // pass 2: folded records
  for (int i = threadIdx.x; i < (n + 1) * D; i += blockDim.x) {
    const int p = i / D, d = i % D;
    float* r = rec + (size_t)p * 4 * D + (d / V) * 4 * V + (d % V);
    double q0, q1, q2, q3;
    if (p < n) {
      const Step& sh = a.steps[2 * p];
      const LayerDesc& J = a.layers[a.steps[2 * p + 1].layer];
      const double vh = (double)((const float*)a.layers[sh.layer].p[0])[(int64_t)sh.col * D + d] * scr[3 * p];
      const double xi = ((const float*)J.p[2])[d];
      const double il = 1.0 / (double)((const float*)J.p[3])[d];
      if (p == 0) {
        q0 = vh;
        q1 = il;
        q2 = -xi * il;
      } else {
        const LayerDesc& Jp = a.layers[a.steps[2 * p - 1].layer];
        const double gp = ((const float*)Jp.p[0])[d];
        const double dp = (double)((const float*)Jp.p[1])[d] * kLn2;
        q0 = vh * dp;
        q1 = dp * il;
        q2 = (gp - xi - scr[3 * p + 1] * vh) * il;
      }
      q3 = vh * il;
    } else {
      const LayerDesc& Jl = a.layers[a.steps[2 * n - 1].layer];
      q0 = ((const float*)Jl.p[0])[d];
      q1 = (double)((const float*)Jl.p[1])[d] * kLn2;
      q2 = q3 = 0.0;
    }
    r[0] = (float)q0;
    r[V] = (float)q1;
    r[2 * V] = (float)q2;
    r[3 * V] = (float)q3;
  }
  if (threadIdx.x == 0) {
    double c = 0.0;
    for (int p = 0; p < n; ++p) c += scr[3 * p + 2];
    *ctot = (float)c;
  }
  __syncthreads();
}

// One pair (reflection + Johnson) on the register tile, fast form. x holds L (pair 0: the input x)
// on entry and the new L on exit; r points at the lane's record group of this pair and is advanced
// to the next record (the parameter registers are reloaded for it). Returns the largest product of
// a fragment's four q = 1 + z^2 of this lane (+Inf / NaN: the fast form is not valid for the tile).
template <int D, int U, bool LADJ>
__device__ __forceinline__ float hj_pair_fast(Tile<float, D, U>& x, float (&acc)[U][1], const float*& r,
                                              float (&pa)[4], float (&pP)[4], float (&pQ)[4], float (&pR)[4]) {
  using T = float;
  constexpr int V = 4;
  T dot[U][1];
  tile_dots<T, D, U>(x, pa, dot);
  // z = L P + Q - dotL R (in place; the first FMA does not wait for the dot reduction)
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < V; ++e) x[u][e] = fmaf(x[u][e], pP[e], pQ[e]);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < V; ++e) x[u][e] = fmaf(-dot[u][0], pR[e], x[u][e]);
  // next pair's records (record n holds gamma_n, delta'_n for the output)
  r += 4 * D;
  lds_vec<T, V>(r, pa);
  lds_vec<T, V>(r + V, pP);
  lds_vec<T, V>(r + 2 * V, pQ);
  lds_vec<T, V>(r + 3 * V, pR);
  // stage by stage over the whole tile (U*V independent chains per stage)
  T q[U][V], t[U][V], pr[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < V; ++e) q[u][e] = fmaf(x[u][e], x[u][e], 1.0f);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < V; ++e) t[u][e] = hw_sqrt(q[u][e]);
#pragma unroll
  for (int u = 0; u < U; ++u) pr[u] = (q[u][0] * q[u][1]) * (q[u][2] * q[u][3]);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < V; ++e) t[u][e] = fabsf(x[u][e]) + t[u][e];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < V; ++e) t[u][e] = hw_log2(t[u][e]);
  if (LADJ)
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u][0] = fmaf(-0.5f, hw_log2(pr[u]), acc[u][0]);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < V; ++e) x[u][e] = copysignf(t[u][e], x[u][e]);
  T m = pr[0];
#pragma unroll
  for (int u = 1; u < U; ++u) m = fmaxf(m, pr[u]);
  return m;
}

// The same pair in the exact-range elementwise form (johnson_fwd_f32_slow): asinh finite up to
// FLT_MAX, ladj -Inf where the reference's fp32 1 + z^2 overflows.
template <int D, int U, bool LADJ>
__device__ __forceinline__ void hj_pair_exact(Tile<float, D, U>& x, float (&acc)[U][1], const float*& r,
                                              float (&pa)[4], float (&pP)[4], float (&pQ)[4], float (&pR)[4]) {
  using T = float;
  constexpr int V = 4;
  T dot[U][1];
  tile_dots<T, D, U>(x, pa, dot);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const YL yl = johnson_fwd_f32_slow(fmaf(-dot[u][0], pR[e], fmaf(x[u][e], pP[e], pQ[e])), 0.f, 1.f);
      x[u][e] = yl.y;
      if (LADJ) acc[u][0] += yl.l;
    }
  r += 4 * D;
  lds_vec<T, V>(r, pa);
  lds_vec<T, V>(r + V, pP);
  lds_vec<T, V>(r + 2 * V, pQ);
  lds_vec<T, V>(r + 3 * V, pR);
}

template <int D, int U, int LM>
struct HJBody {
  using T = float;
  const FlowArgs& a;
  const float* rec;  // this lane's record group
  float ctot;
  float* stage;
  int n;

  template <bool TAIL, int DBG>
  __device__ __forceinline__ void tile(int64_t col0, Tile<T, D, U>& x,
                                       const T (&old)[LadjOut<T, D, U>::NLS][LadjOut<T, D, U>::W]) {
    ENF_FRAG_CONSTS
    static_assert(CPF == 1 && SEG == V, "D >= 4 layout");
    constexpr bool LADJ = LM > 0;
    T acc[U][1];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u][0] = 0.f;
    // No "+v" asm fence on x here (the interpreter uses one to pin the vmcnt wait): with the
    // runtime pair loop below it made the register allocator reuse live tile registers (hipcc 7.2,
    // wrong results). The compiler's own counted waits keep the next tile's loads in flight.
    const float* r = rec;
    T pa[V], pP[V], pQ[V], pR[V];
    lds_vec<T, V>(r, pa);
    lds_vec<T, V>(r + V, pP);
    lds_vec<T, V>(r + 2 * V, pQ);
    lds_vec<T, V>(r + 3 * V, pR);
    // branch-free pair loop; the rare tile with |z| >= 2^16 (or Inf / NaN) is redone below
    T m = 0.f;
    for (int p = 0; p < n; ++p) m = fmaxf(m, hj_pair_fast<D, U, LADJ>(x, acc, r, pa, pP, pQ, pR));
    if (__builtin_expect(!(m <= FLT_MAX), 0)) {
      load_tile<T, D, U, TAIL, DBG>(a, col0, x);
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u][0] = 0.f;
      r = rec;
      lds_vec<T, V>(r, pa);
      lds_vec<T, V>(r + V, pP);
      lds_vec<T, V>(r + 2 * V, pQ);
      lds_vec<T, V>(r + 3 * V, pR);
      for (int p = 0; p < n; ++p) hj_pair_exact<D, U, LADJ>(x, acc, r, pa, pP, pQ, pR);
    }
    // y = gamma_n + delta'_n L
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < V; ++e) x[u][e] = fmaf(x[u][e], pP[e], pa[e]);
    store_tile<T, D, U, LM, TAIL, DBG>(a, ctot, col0, x, acc, old, stage);
  }
};

template <int D, int U, int LM, int OCC, int DBG>
__global__ __launch_bounds__(256, OCC) void flow_hj_kernel(FlowArgs a, int n) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* scr = reinterpret_cast<double*>(smem);
  float* ctotp = reinterpret_cast<float*>(scr + 3 * kHjMaxPairs);
  float* stage = reinterpret_cast<float*>(smem + kHjScratch) + (threadIdx.x >> 6) * kStagePerWave;
  float* rec = reinterpret_cast<float*>(smem + kHjHeader);
  build_hj_program<D>(a, n, rec, scr, ctotp);
  constexpr int G = Frag<float, D>::G;
  HJBody<D, U, LM> body{a, rec + ((threadIdx.x & 63) % G) * 16, *ctotp, stage, n};
  frag_stream<float, D, U, LM, DBG>(a, body);
}

int hj_program_pairs(const FlowArgs& a) {
  if (!a.frag || (a.D != 32 && a.D != 64) || a.nsteps < 2 || (a.nsteps & 1)) return 0;
  for (int s = 0; s < a.nsteps; ++s) {
    const int want = (s & 1) ? OP_JOHNSON : OP_HOUSEHOLDER;
    if (a.steps[s].op != want) return 0;
  }
  return a.nsteps / 2;
}

template <int D, int U, int LM, int OCC = 1, int DBG = 0>
static hipError_t launch_hj(const FlowArgs& a, int n, hipStream_t st, const DeviceInfo& dev) {
  const size_t lds = hj_lds_bytes(D, n);
  const void* k = reinterpret_cast<const void*>(&flow_hj_kernel<D, U, LM, OCC, DBG>);
  int64_t blocks = 0;
  hipError_t e = frag_grid(k, a.N, (int64_t)Frag<float, D>::COLS_PER_INSTR * U * 4, lds, dev, &blocks);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((flow_hj_kernel<D, U, LM, OCC, DBG>), dim3((unsigned)blocks), dim3(256), lds, st, a, n);
  return hipGetLastError();
}

// Tuning variants (development only, fp32 D = 32 with ladj): ENF_HJ_U in {2, 4, 8}, ENF_HJ_OCC in {1, 5, 6}.
template <int LM>
static hipError_t dispatch_hj(const FlowArgs& a, int n, int dbg, hipStream_t st, const DeviceInfo& dev) {
  if (a.D == 32) {
    if constexpr (LM == 1) {
      static const int u = env_int("ENF_HJ_U", 4);
      static const int occ = env_int("ENF_HJ_OCC", 1);
      if (dbg == 1) return launch_hj<32, 4, 1, 1, 1>(a, n, st, dev);
      if (dbg == 2) return launch_hj<32, 4, 1, 1, 2>(a, n, st, dev);
      if (u == 2) return launch_hj<32, 2, 1>(a, n, st, dev);
      if (u == 8) return launch_hj<32, 8, 1>(a, n, st, dev);
      if (occ == 5) return launch_hj<32, 4, 1, 5>(a, n, st, dev);
      if (occ == 6) return launch_hj<32, 4, 1, 6>(a, n, st, dev);
    }
    return launch_hj<32, 4, LM>(a, n, st, dev);
  }
  return launch_hj<64, 4, LM>(a, n, st, dev);
}

hipError_t launch_hj_program(const FlowArgs& a, int lm, int dbg, hipStream_t st, const DeviceInfo& dev) {
  const int n = hj_program_pairs(a);
  if (n < 1 || n > kHjMaxPairs) return hipErrorNotSupported;
  if (lm == 0) return dispatch_hj<0>(a, n, dbg, st, dev);
  if (lm == 1) return dispatch_hj<1>(a, n, dbg, st, dev);
  return dispatch_hj<2>(a, n, dbg, st, dev);
}

}  // namespace enf
