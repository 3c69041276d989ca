// enf_grad_hj.hip -- fused forward + backward of the whitening loss for the config-5 flows
// J_n o H_n o ... o J_1 o H_1 (fp32, D in {32, 64}, n <= 8, one reflection per H, contiguous
// 16-byte aligned columns): mvnormal_negll_trafo / mvnormal_negll_trafograd
// (src/optimize_whitening.jl:7-22) for the N local samples, as per-block partial sums in the
// layout of enf_grad.hip (reduced and Householder-projected by enf_grad_tail.h's reduction).
//
// Forward (per pair, per element; hardware transcendentals as the forward kernel):
//   dot = vh'u, h = u - dot vh, z = (h - xi)/lambda, y = gamma + delta asinh z,
//   ladj += log|delta/lambda| - log(1 + z^2)/2    (householder_trafo.jl:8-11, johnson_trafo.jl:29-52)
// Backward with g = dS/dy (g = y at the output), s = sqrt(1 + z^2):
//   dS/dgamma += g, dS/ddelta += g asinh z - 1/delta, dz = g delta/s + z/s^2,
//   dS/dxi -= dz/lambda, dS/dlambda += -dz z/lambda + 1/lambda, g_h = dz/lambda,
//   Householder: dS/dvh-direction += g_h (vh'u) + u (vh'g_h) (projected in the reduction),
//   g_u = g_h - vh (vh'g_h).
// The layer inputs are recovered as h = lambda z + xi, u = h + dot vh, as the reference's pullback
// recomputes them by re-reflection (householder_trafo.jl:91-101).
//
// Round 5 (the per-step fixed cost at small minibatch shares):
// * the register kernel takes V rows per lane (V = 4: one 16-byte fragment, as before; V = 2 / 1: a column
//   over 16 / 32 lanes): at a share of 12 500 columns a wave had about one 8-column tile and ran it alone on
//   its SIMD at a quarter of the issue rate; with V = 2 the same columns make twice the waves at half the
//   registers (more waves per SIMD) and the cross-lane sums of a D = 32 column stay within DPP rows;
// * a block holds W waves (the records and the partial row are per block);
// * the per-block prologue no longer evaluates the double log|delta| - log|lambda| of every row: the flow's
//   constant ladj does not depend on the samples and enters the loss only (its gradients are the -1/delta,
//   +1/lambda terms, added from the block's column count), so block 0 of the grid computes it once and the
//   reduction subtracts N times it from the loss.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "enf_frag.h"
#include "enf_grad_hj.h"
#include "enf_train.h"

namespace enf {

namespace {

constexpr int kNP = 8;  // records per pair: vh, gamma, delta*ln2, 1/lambda, -xi/lambda, lambda, xi, delta
constexpr int kScrBytes = 512;  // block scratch: [0, 8) per-pair scale, [16, 16 + 2W) per-wave loss / count

typedef unsigned int u32x2h __attribute__((ext_vector_type(2)));

// V rows per lane: G = D / V lanes per column, S = 64 / G columns per wave instruction, TC per tile
template <int D, int V, int KU>
struct GL {
  static constexpr int G = D / V;
  static constexpr int S = 64 / G;
  static constexpr int TC = S * KU;
  static_assert(D % V == 0 && G <= 64 && 64 % G == 0, "a column within one wave");
};

template <int V>
__device__ __forceinline__ void gload_rows(const float* __restrict__ src, float (&x)[V]) {
  if constexpr (V == 4) {
    const u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
    __builtin_memcpy(&x[0], &w, 16);
  } else if constexpr (V == 2) {
    const u32x2h w = __builtin_nontemporal_load(reinterpret_cast<const u32x2h*>(src));
    __builtin_memcpy(&x[0], &w, 8);
  } else {
    x[0] = __builtin_nontemporal_load(src);
  }
}

template <int V>
__device__ __forceinline__ void lds_rows(const float* __restrict__ p, float (&v)[V]) {
  if constexpr (V == 4) {
    lds_vec<float, 4>(p, v);
  } else if constexpr (V == 2) {
    const u32x2h w = *reinterpret_cast<const u32x2h*>(p);
    __builtin_memcpy(&v[0], &w, 8);
  } else {
    v[0] = *p;
  }
}

template <int V>
__device__ __forceinline__ float prod_rows(const float (&q)[V]) {
  if constexpr (V == 4) return (q[0] * q[1]) * (q[2] * q[3]);
  else if constexpr (V == 2) return q[0] * q[1];
  else return q[0];
}

// cross-slot sum: lanes with equal lane % G hold the same rows
template <int G>
__device__ __forceinline__ float slot_sum(float v) {
  // strides G, 2G, ... < 64 in that order, as `v += __shfl_xor(v, m)`, without LDS round trips (enf_train.h)
  static_assert(G >= 8, "D >= 32, at most 4 rows per lane");
  if constexpr (G == 8) v += dpp_mov<0x128>(v);  // row_ror:8 = lane ^ 8
  if constexpr (G <= 16) v = add_xor_swap<16>(v);
  if constexpr (G <= 32) v = add_xor_swap<32>(v);
  return v;
}

// the records of the lane's rows r0 = V grp .. r0 + V - 1 (layout [pair][4-row group][param][4]); parameter q at +4q
template <int D, int V>
__device__ __forceinline__ const float* rec_lane(const float* __restrict__ rec, int p, int grp) {
  const int r0 = V * grp;
  return rec + (size_t)p * kNP * D + (r0 / 4) * kNP * 4 + (r0 % 4);
}

// LDS variant (n > 4 pairs): z and the reflection dot of every pair stored in LDS between the passes
template <int D, int KU, bool TAIL>
__device__ __forceinline__ void grad_tile(const HJGradArgs& a, int64_t col0, int lane, const float* __restrict__ rec,
                                          float* __restrict__ zst, float* __restrict__ dst, float* __restrict__ acc,
                                          double& lossp, int& nvalid) {
  const uint32_t csign = sign_mask_vgpr();  // asinh2_f32: the accurate fp32 asinh (enf_frag.h)
  using L = GL<D, 4, KU>;
  constexpr int V = 4, G = L::G, S = L::S;
  const int grp = lane % G;
  const int n = a.n;
  float x[KU][V];
  float vm[KU];  // 1 for a valid column, 0 past N
#pragma unroll
  for (int u = 0; u < KU; ++u) {
    const int64_t c = col0 + (int64_t)u * S + lane / G;
    const float* src = a.X + c * D + V * grp;
    vm[u] = (!TAIL || c < a.N) ? 1.f : 0.f;
    if (!TAIL) {
      gload_rows<V>(src, x[u]);
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) x[u][e] = c < a.N ? src[e] : 0.f;
    }
  }
  // ---- forward
  float lad[KU] = {};
  for (int p = 0; p < n; ++p) {
    const float* r = rec_lane<D, V>(rec, p, grp);
    float vh[V], gam[V], dl2[V], il[V], nxil[V];
    lds_rows<V>(r, vh);
    lds_rows<V>(r + 4, gam);
    lds_rows<V>(r + 8, dl2);
    lds_rows<V>(r + 12, il);
    lds_rows<V>(r + 16, nxil);
    float dot[KU];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      float t = vh[0] * x[u][0];
#pragma unroll
      for (int e = 1; e < V; ++e) t = fmaf(vh[e], x[u][e], t);
      dot[u] = group_sum<G>(t);
    }
    float z[KU][V], q[KU][V];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        z[u][e] = fmaf(fmaf(-dot[u], vh[e], x[u][e]), il[e], nxil[e]);
        q[u][e] = fmaf(z[u][e], z[u][e], 1.f);
      }
      dst[(p * KU + u) * 64 + lane] = dot[u];
      *reinterpret_cast<u32x4*>(zst + ((size_t)(p * KU + u) * 64 + lane) * V) = *reinterpret_cast<const u32x4*>(&z[u][0]);
    }
#pragma unroll
    for (int u = 0; u < KU; ++u) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float Lz = asinh2_f32(z[u][e], q[u][e], hw_sqrt(q[u][e]), csign);
        x[u][e] = fmaf(dl2[e], Lz, gam[e]);
      }
      lad[u] = fmaf(-0.5f, hw_log2(prod_rows<V>(q[u])), lad[u]);
    }
  }
  // ---- loss without the constant ladj: sum_d (y^2 + log 2 pi)/2 - ln2 * lad (valid columns)
#pragma unroll
  for (int u = 0; u < KU; ++u) {
    float t = 0.f;
#pragma unroll
    for (int e = 0; e < V; ++e) t = fmaf(x[u][e], x[u][e], t);
    const float ysq = group_sum<G>(t);
    const float ltot = group_sum<G>(lad[u]);
    if (grp == 0 && vm[u] != 0.f) {
      lossp += 0.5 * (double)ysq + 0.5 * D * 1.8378770664093454836 - kLn2 * (double)ltot;
      ++nvalid;
    }
  }
  // ---- backward, g = dS/dy = y
  float g[KU][V];
#pragma unroll
  for (int u = 0; u < KU; ++u)
#pragma unroll
    for (int e = 0; e < V; ++e) g[u][e] = x[u][e] * vm[u];
  for (int p = n - 1; p >= 0; --p) {
    const float* r = rec_lane<D, V>(rec, p, grp);
    float vh[V], il[V], lam[V], xi[V], del[V];
    lds_rows<V>(r, vh);
    lds_rows<V>(r + 12, il);
    lds_rows<V>(r + 20, lam);
    lds_rows<V>(r + 24, xi);
    lds_rows<V>(r + 28, del);
    float aG[V] = {}, aD[V] = {}, aX[V] = {}, aL[V] = {}, aV[V] = {};
    float gh[KU][V], u_[KU][V], dot1[KU];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      float z[V];
      *reinterpret_cast<u32x4*>(&z[0]) = *reinterpret_cast<const u32x4*>(zst + ((size_t)(p * KU + u) * 64 + lane) * V);
      dot1[u] = dst[(p * KU + u) * 64 + lane];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float q = fmaf(z[e], z[e], 1.f);
        const float s = hw_sqrt(q);
        const float rs = hw_rcp(s);
        const float Lz = asinh2_f32(z[e], q, s, csign);
        aG[e] += g[u][e];
        aD[e] = fmaf(g[u][e], Lz, aD[e]);
        const float dz = fmaf(g[u][e] * del[e], rs, z[e] * (rs * rs) * vm[u]);
        gh[u][e] = dz * il[e];
        aX[e] += gh[u][e];
        aL[e] = fmaf(gh[u][e], z[e], aL[e]);
        u_[u][e] = fmaf(dot1[u], vh[e], fmaf(lam[e], z[e], xi[e]));  // layer input u = h + dot vh
      }
    }
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      float t = vh[0] * gh[u][0];
#pragma unroll
      for (int e = 1; e < V; ++e) t = fmaf(vh[e], gh[u][e], t);
      const float vg = group_sum<G>(t);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        aV[e] = fmaf(gh[u][e], dot1[u], fmaf(u_[u][e], vg, aV[e]));
        g[u][e] = fmaf(-vg, vh[e], gh[u][e]);
      }
    }
    // flush: one lane per row adds the wave's sums (acc layout [pair][param 5][D])
    float* ap = acc + (size_t)p * 5 * D + V * grp;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const float sV = slot_sum<G>(aV[e]), sG = slot_sum<G>(aG[e]), sD = slot_sum<G>(aD[e]);
      const float sX = slot_sum<G>(aX[e]), sL = slot_sum<G>(aL[e]);
      if (lane < G) {
        ap[e] += sV;
        ap[D + e] += sG;
        ap[2 * D + e] += sD;
        ap[3 * D + e] += sX;
        ap[4 * D + e] += sL;
      }
    }
  }
}

// LDS-only block barrier: global loads issued before it (a wave's first tile) stay in flight
__device__ __forceinline__ void gh_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Block prologue: the per-row records of every pair in one round of global loads. Thread i of the first n*D
// handles row d = i % D of pair p = i / D; the pair's v'v is reduced over the D adjacent lanes that hold it
// (D <= 64: within one wave); after one LDS barrier each thread writes its row's records with the pair's
// reflection scale sqrt(2/v'v) (householder_trafo.jl:9-10). Double arithmetic for the derived values.
template <int D, int NT>
__device__ __forceinline__ void grad_prologue(const HJGradArgs& a, double* __restrict__ scr, float* __restrict__ rec) {
  static_assert(D <= 64 && 64 % D == 0, "a pair's rows within one wave");
  const int n = a.n;
  const int tid = threadIdx.x;
  constexpr int kIt = (kHJGradMaxPairs * D + NT - 1) / NT;
  float pv[kIt], pg[kIt], pd[kIt], px[kIt], pl[kIt];
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int i = tid + NT * it;
    const int p = i / D, d = i % D;
    double vv = 0.0;
    pv[it] = pg[it] = px[it] = 0.f;
    pd[it] = pl[it] = 1.f;
    if (p < n) {
      pv[it] = a.v[p][d];
      pg[it] = a.g[p][d];
      pd[it] = a.d[p][d];
      px[it] = a.xi[p][d];
      pl[it] = a.lam[p][d];
      vv = (double)pv[it] * (double)pv[it];
    }
#pragma unroll
    for (int m = D / 2; m >= 1; m >>= 1) vv += __shfl_xor(vv, m);  // the D lanes of pair p (whole wave active)
    if (p < n && d == 0) scr[p] = sqrt(2.0 / vv);
  }
  gh_lds_barrier();
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int i = tid + NT * it;
    const int p = i / D, d = i % D;
    if (p >= n) continue;
    float* r = rec + (size_t)p * kNP * D + (d / 4) * kNP * 4 + (d % 4);
    const double lam = pl[it], xi = px[it], del = pd[it];
    r[0] = (float)((double)pv[it] * scr[p]);
    r[4] = pg[it];
    r[8] = (float)(del * kLn2);
    r[12] = (float)(1.0 / lam);
    r[16] = (float)(-xi / lam);
    r[20] = pl[it];
    r[24] = px[it];
    r[28] = pd[it];
  }
  gh_lds_barrier();
}

// Block 0 of the grid: the flow's constant ladj sum_p sum_d (log|delta_d| - log|lambda_d|) (johnson_trafo.jl:41)
// in double -- per pair over its D lanes, then the pairs in order -- to *ctot_out.
template <int D, int NT>
__device__ __forceinline__ void ctot_block(const HJGradArgs& a, double* __restrict__ scr) {
  const int n = a.n;
  const int tid = threadIdx.x;
  constexpr int kIt = (kHJGradMaxPairs * D + NT - 1) / NT;
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int i = tid + NT * it;
    const int p = i / D, d = i % D;
    double cl = 0.0;
    if (p < n) cl = log(fabs((double)a.d[p][d])) - log(fabs((double)a.lam[p][d]));
#pragma unroll
    for (int m = D / 2; m >= 1; m >>= 1) cl += __shfl_xor(cl, m);
    if (p < n && d == 0) scr[p] = cl;
  }
  __syncthreads();
  if (tid == 0) {
    double c = 0.0;
    for (int p = 0; p < n; ++p) c += scr[p];
    *a.ctot_out = c;
    if (a.ctot_row) a.ctot_row[0] = -(double)a.N * c;
  }
  if (a.ctot_row)
    for (int i = 1 + tid; i <= a.nparams; i += NT) a.ctot_row[i] = 0.0;
}

// Block epilogue: loss (without the constant ladj) and the flow gradient (layer order, the enf_flow_param_count
// layout) of the block from its W waves' accumulators acc0 + w * wstride ([pair][param 5][D] floats each),
// summed in wave order (deterministic), to partial row blockIdx.x - 1.
template <int D, int W>
__device__ __forceinline__ void grad_epilogue(const HJGradArgs& a, double* __restrict__ scr, const float* __restrict__ rec,
                                              const float* __restrict__ acc0, size_t wstride, double lossp, int nvalid) {
  const int n = a.n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  lossp = xor_tree(lossp, 64);  // the 64-lane xor butterfly (enf_train.h)
  nvalid = xor_tree(nvalid, 64);
  double* wl = scr + 16;
  if (lane == 0) {
    wl[2 * wave] = lossp;
    wl[2 * wave + 1] = (double)nvalid;
  }
  __syncthreads();
  double* out = a.partial + (int64_t)(blockIdx.x - 1) * (1 + a.nparams);
  double nb = wl[1], lb = wl[0];
#pragma unroll
  for (int w = 1; w < W; ++w) {
    nb += wl[2 * w + 1];
    lb += wl[2 * w];
  }
  if (tid == 0) out[0] = lb;
  for (int i = tid; i < n * 5 * D; i += 64 * W) {
    const int p = i / (5 * D), k = (i / D) % 5, d = i % D;
    double s = (double)acc0[i];
#pragma unroll
    for (int w = 1; w < W; ++w) s += (double)acc0[w * wstride + i];
    // delta and lambda from the records (the fp32 parameters, exactly)
    const float* r = rec + (size_t)p * kNP * D + (d / 4) * kNP * 4 + (d % 4);
    const double del = r[28], lam = r[20];
    double gval;
    int64_t o;
    switch (k) {
      case 0: gval = s; o = a.goffH[p] + d; break;                             // raw Householder sum
      case 1: gval = s; o = a.goffJ[p] + d; break;                             // gamma
      case 2: gval = kLn2 * s - nb / del; o = a.goffJ[p] + D + d; break;       // delta
      case 3: gval = -s; o = a.goffJ[p] + 2 * D + d; break;                    // xi
      default: gval = -s + nb / lam; o = a.goffJ[p] + 3 * D + d; break;        // lambda
    }
    out[1 + o] = gval;
  }
}

// KU: fragments (columns) per lane per tile. 1 halves the LDS image of z per wave (more resident
// blocks per CU) but doubles the per-tile flush of the gradient partials; 2 measured faster.
template <int D, int KU>
__global__ __launch_bounds__(256) void hj_grad_kernel(HJGradArgs a) {
  using L = GL<D, 4, KU>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = a.n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // LDS: [scratch][records][per wave: acc, z, dot]
  double* scr = reinterpret_cast<double*>(smem);
  if (blockIdx.x == 0) {
    ctot_block<D, 256>(a, scr);
    return;
  }
  float* rec = reinterpret_cast<float*>(smem + kScrBytes);
  const size_t recb = (size_t)n * kNP * D * 4;
  const size_t accb = (size_t)n * 5 * D * 4;
  const size_t zb = (size_t)n * KU * 64 * 16;
  const size_t db = (size_t)n * KU * 64 * 4;
  unsigned char* wbase = smem + kScrBytes + recb + (size_t)wave * (accb + zb + db);
  float* acc = reinterpret_cast<float*>(wbase);
  float* zst = reinterpret_cast<float*>(wbase + accb);
  float* dst = reinterpret_cast<float*>(wbase + accb + zb);
  for (int i = lane; i < n * 5 * D; i += 64) acc[i] = 0.f;
  grad_prologue<D, 256>(a, scr, rec);
  double lossp = 0.0;
  int nvalid = 0;
  const int64_t ntiles = (a.N + L::TC - 1) / L::TC;
  const int64_t full = a.N / L::TC;
  const int64_t wave_id = (int64_t)(blockIdx.x - 1) * 4 + __builtin_amdgcn_readfirstlane(wave);
  for (int64_t t = wave_id; t < ntiles; t += (int64_t)(gridDim.x - 1) * 4) {
    if (t < full) grad_tile<D, KU, false>(a, t * L::TC, lane, rec, zst, dst, acc, lossp, nvalid);
    else grad_tile<D, KU, true>(a, t * L::TC, lane, rec, zst, dst, acc, lossp, nvalid);
  }
  grad_epilogue<D, 4>(a, scr, rec, reinterpret_cast<const float*>(smem + kScrBytes + recb), (accb + zb + db) / 4, lossp,
                      nvalid);
}

// ---- register variant (NP <= 4 pairs, compile time): z and the reflection dots of a tile stay in
// registers between its forward and backward, and the per-lane gradient partials accumulate in
// registers over all of the wave's tiles (acc[pair][param][row]); one cross-slot reduction per
// wave at the end instead of one per tile and pair. Same arithmetic per element as grad_tile.
// the lane's rows of a tile (zeros past N)
template <int D, int V, int KU>
__device__ __forceinline__ void grad_load_reg(const HJGradArgs& a, int64_t col0, int lane, float (&x)[KU][V]) {
  using L = GL<D, V, KU>;
  constexpr int G = L::G, S = L::S;
#pragma unroll
  for (int u = 0; u < KU; ++u) {
    const int64_t c = col0 + (int64_t)u * S + lane / G;
    if (c < a.N) {
      gload_rows<V>(a.X + c * D + V * (lane % G), x[u]);
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) x[u][e] = 0.f;
    }
  }
}

// RC (recompute): the backward re-derives sqrt(1 + z^2) and asinh(z) from z instead of keeping them from the
// forward (2 V KU NP fewer VGPRs, two transcendentals and the asinh merge more per element-pair)
template <int D, int V, int KU, int NP, bool TAIL, bool RC = false>
__device__ __forceinline__ void grad_tile_reg(const HJGradArgs& a, int64_t col0, int lane, const float* __restrict__ rec,
                                              const float (&xin)[KU][V], float (&acc)[NP][5][V], double& lossp,
                                              int& nvalid) {
  const uint32_t csign = sign_mask_vgpr();  // asinh2_f32: the accurate fp32 asinh (enf_frag.h)
  using L = GL<D, V, KU>;
  constexpr int G = L::G, S = L::S;
  const int grp = lane % G;
  float x[KU][V];
  float vm[KU];
#pragma unroll
  for (int u = 0; u < KU; ++u) {
    vm[u] = (!TAIL || col0 + (int64_t)u * S + lane / G < a.N) ? 1.f : 0.f;
#pragma unroll
    for (int e = 0; e < V; ++e) x[u][e] = xin[u][e];
  }
  float zs[NP][KU][V], ds[NP][KU];
  // sqrt(1 + z^2) and asinh(z)/ln2 of the forward, for the backward (RC: not kept)
  float ss[RC ? 1 : NP][KU][V], ls[RC ? 1 : NP][KU][V];
  float lad[KU] = {};
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const float* r = rec_lane<D, V>(rec, p, grp);
    float vh[V], gam[V], dl2[V], il[V], nxil[V];
    lds_rows<V>(r, vh);
    lds_rows<V>(r + 4, gam);
    lds_rows<V>(r + 8, dl2);
    lds_rows<V>(r + 12, il);
    lds_rows<V>(r + 16, nxil);
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      float t = vh[0] * x[u][0];
#pragma unroll
      for (int e = 1; e < V; ++e) t = fmaf(vh[e], x[u][e], t);
      ds[p][u] = group_sum<G>(t);
    }
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      float q[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        zs[p][u][e] = fmaf(fmaf(-ds[p][u], vh[e], x[u][e]), il[e], nxil[e]);
        q[e] = fmaf(zs[p][u][e], zs[p][u][e], 1.f);
        const float sq = hw_sqrt(q[e]);
        const float lz = asinh2_f32(zs[p][u][e], q[e], sq, csign);
        if constexpr (!RC) {
          ss[p][u][e] = sq;
          ls[p][u][e] = lz;
        }
        x[u][e] = fmaf(dl2[e], lz, gam[e]);
      }
      lad[u] = fmaf(-0.5f, hw_log2(prod_rows<V>(q)), lad[u]);
    }
  }
#pragma unroll
  for (int u = 0; u < KU; ++u) {
    float t = 0.f;
#pragma unroll
    for (int e = 0; e < V; ++e) t = fmaf(x[u][e], x[u][e], t);
    const float ysq = group_sum<G>(t);
    const float ltot = group_sum<G>(lad[u]);
    if (grp == 0 && vm[u] != 0.f) {
      lossp += 0.5 * (double)ysq + 0.5 * D * 1.8378770664093454836 - kLn2 * (double)ltot;
      ++nvalid;
    }
  }
  float g[KU][V];
#pragma unroll
  for (int u = 0; u < KU; ++u)
#pragma unroll
    for (int e = 0; e < V; ++e) g[u][e] = x[u][e] * vm[u];
#pragma unroll
  for (int p = NP - 1; p >= 0; --p) {
    const float* r = rec_lane<D, V>(rec, p, grp);
    float vh[V], il[V], lam[V], xi[V], del[V];
    lds_rows<V>(r, vh);
    lds_rows<V>(r + 12, il);
    lds_rows<V>(r + 20, lam);
    lds_rows<V>(r + 24, xi);
    lds_rows<V>(r + 28, del);
    float gh[KU][V], u_[KU][V];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        float z = zs[p][u][e];
        float sq, Lz;
        if constexpr (RC) {
          asm volatile("" : "+v"(z));  // an opaque copy: the compiler would otherwise reuse the forward's values
          const float q = fmaf(z, z, 1.f);
          sq = hw_sqrt(q);
          Lz = asinh2_f32(z, q, sq, csign);
        } else {
          sq = ss[p][u][e];
          Lz = ls[p][u][e];
        }
        const float rs = hw_rcp(sq);
        acc[p][1][e] += g[u][e];
        acc[p][2][e] = fmaf(g[u][e], Lz, acc[p][2][e]);
        const float dz = fmaf(g[u][e] * del[e], rs, z * (rs * rs) * vm[u]);
        gh[u][e] = dz * il[e];
        acc[p][3][e] += gh[u][e];
        acc[p][4][e] = fmaf(gh[u][e], z, acc[p][4][e]);
        u_[u][e] = fmaf(ds[p][u], vh[e], fmaf(lam[e], z, xi[e]));  // layer input u = h + dot vh
      }
    }
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      float t = vh[0] * gh[u][0];
#pragma unroll
      for (int e = 1; e < V; ++e) t = fmaf(vh[e], gh[u][e], t);
      const float vg = group_sum<G>(t);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        acc[p][0][e] = fmaf(gh[u][e], ds[p][u], fmaf(u_[u][e], vg, acc[p][0][e]));
        g[u][e] = fmaf(-vg, vh[e], gh[u][e]);
      }
    }
  }
}

template <int D, int V, int KU, int NP, int W, bool RC = false>
__global__ __launch_bounds__(64 * W) void hj_grad_reg_kernel(HJGradArgs a) {
  using L = GL<D, V, KU>;
  constexpr int G = L::G;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double* scr = reinterpret_cast<double*>(smem);
  if (blockIdx.x == 0) {
    ctot_block<D, 64 * W>(a, scr);
    return;
  }
  float* rec = reinterpret_cast<float*>(smem + kScrBytes);
  const size_t recb = (size_t)NP * kNP * D * 4;
  float* accs = reinterpret_cast<float*>(smem + kScrBytes + recb);  // per wave [pair][param 5][D]
  const int64_t ntiles = (a.N + L::TC - 1) / L::TC;
  const int64_t wave_id = (int64_t)(blockIdx.x - 1) * W + __builtin_amdgcn_readfirstlane(wave);
  // the wave's first tile is loaded before the prologue: its HBM latency overlaps the parameter round trip
  float xc[KU][V], xn[KU][V];
  if (wave_id < ntiles) grad_load_reg<D, V, KU>(a, wave_id * L::TC, lane, xc);
  grad_prologue<D, 64 * W>(a, scr, rec);
  float acc[NP][5][V];
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int e = 0; e < V; ++e) acc[p][k][e] = 0.f;
  double lossp = 0.0;
  int nvalid = 0;
  const int64_t full = a.N / L::TC;
  // the next tile's columns are loaded while the current one is processed
  const int64_t stride = (int64_t)(gridDim.x - 1) * W;
  for (int64_t t = wave_id; t < ntiles; t += stride) {
    if (t + stride < ntiles) grad_load_reg<D, V, KU>(a, (t + stride) * L::TC, lane, xn);
    if (t < full) grad_tile_reg<D, V, KU, NP, false, RC>(a, t * L::TC, lane, rec, xc, acc, lossp, nvalid);
    else grad_tile_reg<D, V, KU, NP, true, RC>(a, t * L::TC, lane, rec, xc, acc, lossp, nvalid);
#pragma unroll
    for (int u = 0; u < KU; ++u)
#pragma unroll
      for (int e = 0; e < V; ++e) xc[u][e] = xn[u][e];
  }
  // one cross-slot reduction per wave; lanes 0..G-1 then hold the row sums of their V rows
  float* wacc = accs + (size_t)wave * NP * 5 * D;
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float sv = slot_sum<G>(acc[p][k][e]);
        if (lane < G) wacc[(p * 5 + k) * D + V * lane + e] = sv;
      }
  __syncthreads();
  grad_epilogue<D, W>(a, scr, rec, accs, (size_t)NP * 5 * D, lossp, nvalid);
}

template <int D, int NP, int W>
constexpr size_t hj_grad_reg_lds() {
  return kScrBytes + (size_t)NP * kNP * D * 4 + (size_t)W * NP * 5 * D * 4;
}

template <int D, int KU>
size_t hj_grad_lds(int n) {
  return kScrBytes + (size_t)n * kNP * D * 4 + 4 * ((size_t)n * 5 * D * 4 + (size_t)n * KU * 64 * 16 + (size_t)n * KU * 64 * 4);
}

// ---- variant table: (V rows per lane, KU fragments per tile, W waves per block) of the register kernel.
// The product uses 0 or 1 by batch size (product_variant); the diagnostics build can force any (ENF_HJG_VARIANT).
struct RegVariant {
  int V, KU, W, RC;
};
constexpr RegVariant kRegVariants[] = {
    {2, 2, 8, 0},   // 0: the product (round 5) up to kLargeBatch columns
    {4, 1, 4, 0},   // 1: round 4's kernel shape (16-byte fragments, 4 waves per block): the product above it
    {4, 1, 8, 0},   // 2
    {2, 2, 4, 0},   // 3
    {1, 2, 8, 0},   // 4
    {1, 2, 16, 0},  // 5
    {2, 1, 8, 0},   // 6
    {2, 2, 4, 1},   // 7: recomputing sqrt / asinh in the backward (fewer registers, more waves)
    {2, 2, 8, 1},   // 8
    {4, 1, 4, 1},   // 9
};
constexpr int kNumRegVariants = ENF_DIAG ? (int)(sizeof(kRegVariants) / sizeof(kRegVariants[0])) : 1;
constexpr int kLargeVariant = 1;  // the product's shape for large batches (product_variant)

int reg_variant() {
  static const int v = ENF_KNOB("ENF_HJG_VARIANT", 0);
  return (v >= 0 && v < kNumRegVariants) ? v : 0;
}

template <int D, int V, int KU, int NP, int W, bool RC>
const void* reg_kernel_ptr() {
  return reinterpret_cast<const void*>(&hj_grad_reg_kernel<D, V, KU, NP, W, RC>);
}

// (kernel, LDS bytes, columns per wave tile, waves per block) of the register kernel for (D, n pairs, variant)
struct KSel {
  const void* k = nullptr;
  size_t lds = 0;
  int tc = 0, w = 0;
};

template <int D, int V, int KU, int W, bool RC = false>
KSel sel_np(int n) {
  KSel s;
  s.tc = GL<D, V, KU>::TC;
  s.w = W;
  switch (n) {
    case 1: s.k = reg_kernel_ptr<D, V, KU, 1, W, RC>(); s.lds = hj_grad_reg_lds<D, 1, W>(); break;
    case 2: s.k = reg_kernel_ptr<D, V, KU, 2, W, RC>(); s.lds = hj_grad_reg_lds<D, 2, W>(); break;
    case 3: s.k = reg_kernel_ptr<D, V, KU, 3, W, RC>(); s.lds = hj_grad_reg_lds<D, 3, W>(); break;
    default: s.k = reg_kernel_ptr<D, V, KU, 4, W, RC>(); s.lds = hj_grad_reg_lds<D, 4, W>(); break;
  }
  return s;
}

template <int D>
KSel select_reg(int n, int variant) {
  switch (variant) {
#if ENF_DIAG
    case 2: return sel_np<D, 4, 1, 8>(n);
    case 3: return sel_np<D, 2, 2, 4>(n);
    case 4: return sel_np<D, 1, 2, 8>(n);
    case 5: return sel_np<D, 1, 2, 16>(n);
    case 6: return sel_np<D, 2, 1, 8>(n);
    case 7: return sel_np<D, 2, 2, 4, true>(n);
    case 8: return sel_np<D, 2, 2, 8, true>(n);
    case 9: return sel_np<D, 4, 1, 4, true>(n);
#endif
    case kLargeVariant: return sel_np<D, 4, 1, 4>(n);
    default: return sel_np<D, 2, 2, 8>(n);
  }
}

// The product's register kernel by batch size: {2, 2, 8} up to kLargeBatch columns (the 8-rank share of config 5,
// 12 500 columns: 21.3 us per step against 26.6 for {4, 1, 4}), {4, 1, 4} above (B = 1e5: 39.4 against 41.2 us;
// profiles/r05/c5_variants_v3.jsonl). The crossover between the two measured sizes is not measured.
constexpr int64_t kLargeBatch = 50000;
int product_variant(int64_t N) {
  const int v = reg_variant();
  return v != 0 ? v : (N >= kLargeBatch ? kLargeVariant : 0);
}

KSel select_kernel(int64_t D, int n, int64_t N) {
  if (n <= 4) return D == 32 ? select_reg<32>(n, product_variant(N)) : select_reg<64>(n, product_variant(N));
  static const int ku = ENF_KNOB("ENF_GRAD_U", 2) == 1 ? 1 : 2;  // 2: measured 72 vs 93 us at config 5
  KSel s;
  s.w = 4;
  s.tc = (D == 32 ? GL<32, 4, 1>::S : GL<64, 4, 1>::S) * ku;
  s.lds = D == 32 ? (ku == 1 ? hj_grad_lds<32, 1>(n) : hj_grad_lds<32, 2>(n))
                  : (ku == 1 ? hj_grad_lds<64, 1>(n) : hj_grad_lds<64, 2>(n));
  s.k = D == 32 ? (ku == 1 ? (const void*)&hj_grad_kernel<32, 1> : (const void*)&hj_grad_kernel<32, 2>)
                : (ku == 1 ? (const void*)&hj_grad_kernel<64, 1> : (const void*)&hj_grad_kernel<64, 2>);
  return s;
}

// tile blocks for N columns: one tile per wave where the chip has room for them, otherwise the blocks that are
// resident at once (occupancy of the kernel at its LDS size), each wave striding over the tiles
int blocks_for(const KSel& s, int64_t N) {
  static int cached_cu = 0;
  if (!cached_cu) {
    DeviceInfo dev;
    cached_cu = current_device_info(&dev) == ENF_OK && dev.num_cu > 0 ? dev.num_cu : 256;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, s.k, 64 * s.w, s.lds) != hipSuccess || per_cu < 1) per_cu = 1;
  static const int cap_knob = ENF_KNOB("ENF_HJG_BPC", 0);  // diagnostics: blocks per CU cap (0: occupancy)
  if (cap_knob > 0 && per_cu > cap_knob) per_cu = cap_knob;
  const int64_t tiles = (N + s.tc - 1) / s.tc;
  int64_t blocks = (tiles + s.w - 1) / s.w;
  const int64_t cap = (int64_t)cached_cu * per_cu;
  if (blocks > cap) blocks = cap;
  static const int max_knob = ENF_KNOB("ENF_HJG_MAXBLOCKS", 0);  // diagnostics: a grid cap (0: none)
  if (max_knob > 0 && blocks > max_knob) blocks = max_knob;
  return (int)(blocks < 1 ? 1 : blocks);
}

}  // namespace

bool hj_grad_shape_ok(int64_t D, const enf_layer* layers, int32_t nlayers) {
  if (D != 32 && D != 64) return false;
  if (nlayers < 2 || (nlayers & 1) || nlayers / 2 > kHJGradMaxPairs) return false;
  for (int32_t l = 0; l < nlayers; ++l) {
    const int want = (l & 1) ? OP_JOHNSON : OP_HOUSEHOLDER;
    if (layers[l].op != want || (want == OP_HOUSEHOLDER && layers[l].k != 1)) return false;
  }
  return true;
}

bool hj_grad_eligible(int64_t D, int64_t ldx, const void* X, const enf_layer* layers, int32_t nlayers) {
  return ldx == D && (((uintptr_t)X) & 15) == 0 && hj_grad_shape_ok(D, layers, nlayers);
}

// Partial rows a launch for ANY batch of at most N columns may write (the workspace reservation, make_plan): the
// kernel's shape changes at kLargeBatch and the small-batch shape can have more blocks, so past it the reservation
// also covers the largest batch below it -- enf_flow_negll_grad_workspace(batchsize) then suffices for a ragged
// last minibatch.
int hj_grad_blocks(int64_t D, int64_t N, int32_t npairs) {
  int b = blocks_for(select_kernel(D, npairs, N), N);
  if (N >= kLargeBatch) b = std::max(b, blocks_for(select_kernel(D, npairs, kLargeBatch - 1), kLargeBatch - 1));
  return b;
}

int hj_grad_launch_rows(int64_t D, int64_t Nplan, int32_t npairs) {
  return blocks_for(select_kernel(D, npairs, Nplan), Nplan);
}

hipError_t launch_hj_grad(int64_t D, int64_t N, const void* X, const enf_layer* layers, int32_t nlayers,
                          int32_t nparams, double* partial, double* ctot_out, int* nblocks, hipStream_t st,
                          int64_t Nplan, bool ctot_row) {
  HJGradArgs a;
  std::memset(&a, 0, sizeof a);
  a.X = (const float*)X;
  a.N = N;
  a.n = nlayers / 2;
  a.D = (int32_t)D;
  a.partial = partial;
  a.ctot_out = ctot_out;
  a.nparams = nparams;
  int32_t off = 0;
  for (int p = 0; p < a.n; ++p) {
    const enf_layer& H = layers[2 * p];
    const enf_layer& J = layers[2 * p + 1];
    a.v[p] = (const float*)H.p[0];
    a.goffH[p] = off;
    off += (int32_t)D;
    a.g[p] = (const float*)J.p[0];
    a.d[p] = (const float*)J.p[1];
    a.xi[p] = (const float*)J.p[2];
    a.lam[p] = (const float*)J.p[3];
    a.goffJ[p] = off;
    off += 4 * (int32_t)D;
  }
  if (off != nparams) return hipErrorInvalidValue;
  const int64_t Np = Nplan > 0 ? Nplan : N;
  const KSel s = select_kernel(D, a.n, Np);
  const int blocks = blocks_for(s, Np);
  a.ctot_row = ctot_row ? partial + (int64_t)blocks * (1 + nparams) : nullptr;
  *nblocks = blocks + (ctot_row ? 1 : 0);
  if (s.lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(s.k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)s.lds);
    if (e != hipSuccess) return e;
  }
  void* args[] = {&a};
  return hipLaunchKernel(s.k, dim3(blocks + 1), dim3(64 * s.w), args, s.lds, st);
}

}  // namespace enf
