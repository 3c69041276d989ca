// enf_grad_hj.hip -- fused forward + backward of the whitening loss for the config-5 flows
// J_n o H_n o ... o J_1 o H_1 (fp32, D in {32, 64}, n <= 8, one reflection per H, contiguous
// 16-byte aligned columns): mvnormal_negll_trafo / mvnormal_negll_trafograd
// (src/optimize_whitening.jl:7-22) for the N local samples, as per-block partial sums in the
// layout of enf_grad.hip (reduced and Householder-projected there).
//
// Forward (per pair, per element; hardware transcendentals as the forward kernel):
//   dot = vh'u, h = u - dot vh, z = (h - xi)/lambda, y = gamma + delta asinh z,
//   ladj += log|delta/lambda| - log(1 + z^2)/2    (householder_trafo.jl:8-11, johnson_trafo.jl:29-52)
// storing z and dot per pair in LDS (the backward needs nothing else: h = lambda z + xi and
// u = h + dot vh recover the layer inputs exactly as in the reference's pullback, which recomputes
// them by re-reflection, householder_trafo.jl:91-101).
// Backward with g = dS/dy (g = y at the output), s = sqrt(1 + z^2):
//   dS/dgamma += g, dS/ddelta += g asinh z - 1/delta, dz = g delta/s + z/s^2,
//   dS/dxi -= dz/lambda, dS/dlambda += -dz z/lambda + 1/lambda, g_h = dz/lambda,
//   Householder: dS/dvh-direction += g_h (vh'u) + u (vh'g_h) (projected in grad_finalize_kernel),
//   g_u = g_h - vh (vh'g_h).
// Per-lane gradient partials of a tile are summed over the lanes holding the same rows (cross-
// lane shuffles) and added by one lane per row into the wave's LDS accumulators; the block sums
// its 4 waves in a fixed order (deterministic).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "enf_frag.h"
#include "enf_grad_hj.h"

namespace enf {

namespace {

constexpr int kNP = 8;  // records per pair: vh, gamma, delta*ln2, 1/lambda, -xi/lambda, lambda, xi, delta

template <int D, int KU>
struct GL {
  static constexpr int V = 4;
  static constexpr int G = D / V;            // lanes per column
  static constexpr int S = 64 / G;           // column slots per wave instruction
  static constexpr int TC = S * KU;          // columns per wave tile
};

// cross-slot sum: lanes with equal lane % G hold the same rows
template <int G>
__device__ __forceinline__ float slot_sum(float v) {
#pragma unroll
  for (int m = G; m < 64; m <<= 1) v += __shfl_xor(v, m);
  return v;
}

template <int D, int KU, bool TAIL>
__device__ __forceinline__ void grad_tile(const HJGradArgs& a, int64_t col0, int lane, const float* __restrict__ rec,
                                          float* __restrict__ zst, float* __restrict__ dst, float* __restrict__ acc,
                                          double& lossp, int& nvalid, float ctot) {
  const uint32_t csign = sign_mask_vgpr();  // asinh2_f32: the accurate fp32 asinh (enf_frag.h)
  using L = GL<D, KU>;
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
      const u32x4 v4 = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
      __builtin_memcpy(&x[u][0], &v4, 16);
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) x[u][e] = c < a.N ? src[e] : 0.f;
    }
  }
  // ---- forward
  float lad[KU] = {};
  for (int p = 0; p < n; ++p) {
    const float* r = rec + (size_t)p * kNP * D + grp * kNP * V;
    float vh[V], gam[V], dl2[V], il[V], nxil[V];
    lds_vec<float, V>(r, vh);
    lds_vec<float, V>(r + V, gam);
    lds_vec<float, V>(r + 2 * V, dl2);
    lds_vec<float, V>(r + 3 * V, il);
    lds_vec<float, V>(r + 4 * V, nxil);
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
      lad[u] = fmaf(-0.5f, hw_log2((q[u][0] * q[u][1]) * (q[u][2] * q[u][3])), lad[u]);
    }
  }
  // ---- loss: sum_d (y^2 + log 2 pi)/2 - ladj, ladj = ctot + ln2 * lad (valid columns)
#pragma unroll
  for (int u = 0; u < KU; ++u) {
    float t = 0.f;
#pragma unroll
    for (int e = 0; e < V; ++e) t = fmaf(x[u][e], x[u][e], t);
    const float ysq = group_sum<G>(t);
    const float ltot = group_sum<G>(lad[u]);
    if (grp == 0 && vm[u] != 0.f) {
      lossp += 0.5 * (double)ysq + 0.5 * D * 1.8378770664093454836 - ((double)ctot + kLn2 * (double)ltot);
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
    const float* r = rec + (size_t)p * kNP * D + grp * kNP * V;
    float vh[V], il[V], lam[V], xi[V], del[V];
    lds_vec<float, V>(r, vh);
    lds_vec<float, V>(r + 3 * V, il);
    lds_vec<float, V>(r + 5 * V, lam);
    lds_vec<float, V>(r + 6 * V, xi);
    lds_vec<float, V>(r + 7 * V, del);
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

// Block prologue shared by both kernels: per pair v'v and the constant ladj part sum log|delta/lambda|
// (double, scr), then the records [pair][group][param][4] in rec. Returns ctot = sum of the constants.
// LDS-only block barrier: global loads issued before it (a wave's first tile) stay in flight
__device__ __forceinline__ void gh_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Block prologue: the per-row records of every pair in ONE round of global loads (round 4; round 3 read the
// parameters twice, once per pass): thread i of the first n*D handles row d = i % D of pair p = i / D, loads its
// five parameters, and the per-pair sums v'v and sum_d log|delta/lambda| (johnson_trafo.jl:41) are reduced over
// the D adjacent lanes that hold pair p (D <= 64: within one wave); after one LDS barrier each thread writes its
// row's records with the pair's reflection scale sqrt(2/v'v) (householder_trafo.jl:9-10). Double arithmetic as
// before, so the same records and constant.
template <int D>
__device__ __forceinline__ float grad_prologue(const HJGradArgs& a, double* __restrict__ scr, float* __restrict__ rec) {
  static_assert(D <= 64 && 256 % D == 0, "a pair's rows within one wave");
  const int n = a.n;
  const int tid = threadIdx.x;
  constexpr int kIt = (kHJGradMaxPairs * D + 255) / 256;  // rows per thread (n * D <= 8 * 64)
  double pv[kIt], pg[kIt], pd[kIt], px[kIt], pl[kIt];
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int i = tid + 256 * it;
    const int p = i / D, d = i % D;
    double vv = 0.0, cl = 0.0;
    pv[it] = pg[it] = px[it] = 0.0;
    pd[it] = pl[it] = 1.0;
    if (p < n) {
      pv[it] = a.v[p][d];
      pg[it] = a.g[p][d];
      pd[it] = a.d[p][d];
      px[it] = a.xi[p][d];
      pl[it] = a.lam[p][d];
      vv = pv[it] * pv[it];
      cl = log(fabs(pd[it])) - log(fabs(pl[it]));
    }
#pragma unroll
    for (int m = D / 2; m >= 1; m >>= 1) {  // the D lanes of pair p (all lanes of the wave take part)
      vv += __shfl_xor(vv, m);
      cl += __shfl_xor(cl, m);
    }
    if (p < n && d == 0) {
      scr[2 * p] = sqrt(2.0 / vv);
      scr[2 * p + 1] = cl;
    }
  }
  gh_lds_barrier();
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int i = tid + 256 * it;
    const int p = i / D, d = i % D;
    if (p >= n) continue;
    float* r = rec + (size_t)p * kNP * D + (d / 4) * kNP * 4 + (d % 4);
    const double lam = pl[it], xi = px[it], del = pd[it];
    r[0] = (float)(pv[it] * scr[2 * p]);
    r[4] = (float)pg[it];
    r[8] = (float)(del * kLn2);
    r[12] = (float)(1.0 / lam);
    r[16] = (float)(-xi / lam);
    r[20] = (float)lam;
    r[24] = (float)xi;
    r[28] = (float)del;
  }
  gh_lds_barrier();
  double c = 0.0;
  for (int p = 0; p < n; ++p) c += scr[2 * p + 1];
  return (float)c;
}

// Block epilogue shared by both kernels: loss and the flow gradient (layer order, the
// enf_flow_param_count layout) of the block from the 4 waves' accumulators acc0 + w * wstride
// ([pair][param 5][D] floats each), summed in a fixed order (deterministic).
template <int D>
__device__ __forceinline__ void grad_epilogue(const HJGradArgs& a, double* __restrict__ scr, const float* __restrict__ rec,
                                              const float* __restrict__ acc0, size_t wstride, double lossp, int nvalid) {
  const int n = a.n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int m = 32; m >= 1; m >>= 1) {
    lossp += __shfl_xor(lossp, m);
    nvalid += __shfl_xor(nvalid, m);
  }
  double* wl = scr + 2 * kHJGradMaxPairs;
  if (lane == 0) {
    wl[2 * wave] = lossp;
    wl[2 * wave + 1] = (double)nvalid;
  }
  __syncthreads();
  double* out = a.partial + (int64_t)blockIdx.x * (1 + a.nparams);
  const double nb = wl[1] + wl[3] + wl[5] + wl[7];
  if (tid == 0) out[0] = ((wl[0] + wl[2]) + wl[4]) + wl[6];
  for (int i = tid; i < n * 5 * D; i += blockDim.x) {
    const int p = i / (5 * D), k = (i / D) % 5, d = i % D;
    const double s = (((double)acc0[i] + (double)acc0[wstride + i]) + (double)acc0[2 * wstride + i]) +
                     (double)acc0[3 * wstride + i];
    // delta and lambda from the records (the fp32 parameters, exactly), not a second round of global loads
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
  using L = GL<D, KU>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = a.n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // LDS: [scratch: per pair {hs, cl}, per wave {loss, nvalid}][records][per wave: acc, z, dot]
  double* scr = reinterpret_cast<double*>(smem);                       // 2*8 + 8 doubles
  float* rec = reinterpret_cast<float*>(smem + 256);                  // n * kNP * D floats
  const size_t recb = (size_t)n * kNP * D * 4;
  const size_t accb = (size_t)n * 5 * D * 4;
  const size_t zb = (size_t)n * KU * 64 * 16;
  const size_t db = (size_t)n * KU * 64 * 4;
  unsigned char* wbase = smem + 256 + recb + (size_t)wave * (accb + zb + db);
  float* acc = reinterpret_cast<float*>(wbase);
  float* zst = reinterpret_cast<float*>(wbase + accb);
  float* dst = reinterpret_cast<float*>(wbase + accb + zb);
  for (int i = lane; i < n * 5 * D; i += 64) acc[i] = 0.f;
  const float ctot = grad_prologue<D>(a, scr, rec);
  double lossp = 0.0;
  int nvalid = 0;
  const int64_t ntiles = (a.N + L::TC - 1) / L::TC;
  const int64_t full = a.N / L::TC;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(wave);
  for (int64_t t = wave_id; t < ntiles; t += (int64_t)gridDim.x * 4) {
    if (t < full) grad_tile<D, KU, false>(a, t * L::TC, lane, rec, zst, dst, acc, lossp, nvalid, ctot);
    else grad_tile<D, KU, true>(a, t * L::TC, lane, rec, zst, dst, acc, lossp, nvalid, ctot);
  }
  grad_epilogue<D>(a, scr, rec, reinterpret_cast<const float*>(smem + 256 + recb), (accb + zb + db) / 4, lossp, nvalid);
}

// ---- register variant (NP <= 4 pairs, compile time): z and the reflection dots of a tile stay in
// registers between its forward and backward, and the per-lane gradient partials accumulate in
// registers over all of the wave's tiles (acc[pair][param][row]); one cross-slot reduction per
// wave at the end instead of one per tile and pair. Same arithmetic per element as grad_tile.
// the lane's fragments of a tile (zeros past N)
template <int D, int KU>
__device__ __forceinline__ void grad_load_reg(const HJGradArgs& a, int64_t col0, int lane, float (&x)[KU][4]) {
  using L = GL<D, KU>;
  constexpr int G = L::G, S = L::S;
#pragma unroll
  for (int u = 0; u < KU; ++u) {
    const int64_t c = col0 + (int64_t)u * S + lane / G;
    if (c < a.N) {
      const u32x4 v4 = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.X + c * D + 4 * (lane % G)));
      __builtin_memcpy(&x[u][0], &v4, 16);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) x[u][e] = 0.f;
    }
  }
}

template <int D, int KU, int NP, bool TAIL>
__device__ __forceinline__ void grad_tile_reg(const HJGradArgs& a, int64_t col0, int lane, const float* __restrict__ rec,
                                              const float (&xin)[KU][4], float (&acc)[NP][5][4], double& lossp,
                                              int& nvalid, float ctot) {
  const uint32_t csign = sign_mask_vgpr();  // asinh2_f32: the accurate fp32 asinh (enf_frag.h)
  using L = GL<D, KU>;
  constexpr int V = 4, G = L::G, S = L::S;
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
  float ss[NP][KU][V], ls[NP][KU][V];  // sqrt(1 + z^2) and asinh(z)/ln2 of the forward, for the backward
  float lad[KU] = {};
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const float* r = rec + (size_t)p * kNP * D + grp * kNP * V;
    float vh[V], gam[V], dl2[V], il[V], nxil[V];
    lds_vec<float, V>(r, vh);
    lds_vec<float, V>(r + V, gam);
    lds_vec<float, V>(r + 2 * V, dl2);
    lds_vec<float, V>(r + 3 * V, il);
    lds_vec<float, V>(r + 4 * V, nxil);
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
        ss[p][u][e] = hw_sqrt(q[e]);
        ls[p][u][e] = asinh2_f32(zs[p][u][e], q[e], ss[p][u][e], csign);
        x[u][e] = fmaf(dl2[e], ls[p][u][e], gam[e]);
      }
      lad[u] = fmaf(-0.5f, hw_log2((q[0] * q[1]) * (q[2] * q[3])), lad[u]);
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
      lossp += 0.5 * (double)ysq + 0.5 * D * 1.8378770664093454836 - ((double)ctot + kLn2 * (double)ltot);
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
    const float* r = rec + (size_t)p * kNP * D + grp * kNP * V;
    float vh[V], il[V], lam[V], xi[V], del[V];
    lds_vec<float, V>(r, vh);
    lds_vec<float, V>(r + 3 * V, il);
    lds_vec<float, V>(r + 5 * V, lam);
    lds_vec<float, V>(r + 6 * V, xi);
    lds_vec<float, V>(r + 7 * V, del);
    float gh[KU][V], u_[KU][V];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float z = zs[p][u][e];
        const float rs = hw_rcp(ss[p][u][e]);
        const float Lz = ls[p][u][e];
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

template <int D, int KU, int NP>
__global__ __launch_bounds__(256) void hj_grad_reg_kernel(HJGradArgs a) {
  using L = GL<D, KU>;
  constexpr int G = L::G;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double* scr = reinterpret_cast<double*>(smem);
  float* rec = reinterpret_cast<float*>(smem + 256);
  const size_t recb = (size_t)NP * kNP * D * 4;
  float* accs = reinterpret_cast<float*>(smem + 256 + recb);  // per wave [pair][param 5][D]
  const int64_t ntiles = (a.N + L::TC - 1) / L::TC;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(wave);
  // the wave's first tile is loaded before the prologue: its HBM latency overlaps the parameter round trip
  // (round 4; at the 8-rank share of config 5 a wave has about one tile)
  float xc[KU][4], xn[KU][4];
  if (wave_id < ntiles) grad_load_reg<D, KU>(a, wave_id * L::TC, lane, xc);
  const float ctot = grad_prologue<D>(a, scr, rec);
  float acc[NP][5][4];
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[p][k][e] = 0.f;
  double lossp = 0.0;
  int nvalid = 0;
  const int64_t full = a.N / L::TC;
  // the next tile's columns are loaded while the current one is processed
  const int64_t stride = (int64_t)gridDim.x * 4;
  for (int64_t t = wave_id; t < ntiles; t += stride) {
    if (t + stride < ntiles) grad_load_reg<D, KU>(a, (t + stride) * L::TC, lane, xn);
    if (t < full) grad_tile_reg<D, KU, NP, false>(a, t * L::TC, lane, rec, xc, acc, lossp, nvalid, ctot);
    else grad_tile_reg<D, KU, NP, true>(a, t * L::TC, lane, rec, xc, acc, lossp, nvalid, ctot);
#pragma unroll
    for (int u = 0; u < KU; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) xc[u][e] = xn[u][e];
  }
  // one cross-slot reduction per wave; lanes 0..G-1 then hold the row sums of their 4 rows
  float* wacc = accs + (size_t)wave * NP * 5 * D;
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float sv = slot_sum<G>(acc[p][k][e]);
        if (lane < G) wacc[(p * 5 + k) * D + 4 * lane + e] = sv;
      }
  __syncthreads();
  grad_epilogue<D>(a, scr, rec, accs, (size_t)NP * 5 * D, lossp, nvalid);
}

template <int D, int KU, int NP>
size_t hj_grad_reg_lds() {
  return 256 + (size_t)NP * kNP * D * 4 + 4 * (size_t)NP * 5 * D * 4;
}

template <int D, int KU>
size_t hj_grad_lds(int n) {
  return 256 + (size_t)n * kNP * D * 4 + 4 * ((size_t)n * 5 * D * 4 + (size_t)n * KU * 64 * 16 + (size_t)n * KU * 64 * 4);
}

template <int D, int KU, int NP>
hipError_t launch_reg_np(const HJGradArgs& a, int blocks, hipStream_t st) {
  const size_t lds = hj_grad_reg_lds<D, KU, NP>();
  hipLaunchKernelGGL((hj_grad_reg_kernel<D, KU, NP>), dim3(blocks), dim3(256), lds, st, a);
  return hipGetLastError();
}

template <int D, int KU>
hipError_t launch_reg(const HJGradArgs& a, int blocks, hipStream_t st) {
  switch (a.n) {
    case 1: return launch_reg_np<D, KU, 1>(a, blocks, st);
    case 2: return launch_reg_np<D, KU, 2>(a, blocks, st);
    case 3: return launch_reg_np<D, KU, 3>(a, blocks, st);
    default: return launch_reg_np<D, KU, 4>(a, blocks, st);
  }
}

}  // namespace

bool hj_grad_eligible(int64_t D, int64_t ldx, const void* X, const enf_layer* layers, int32_t nlayers) {
  if ((D != 32 && D != 64) || ldx != D || (((uintptr_t)X) & 15) != 0) return false;
  if (nlayers < 2 || (nlayers & 1) || nlayers / 2 > kHJGradMaxPairs) return false;
  for (int32_t l = 0; l < nlayers; ++l) {
    const int want = (l & 1) ? OP_JOHNSON : OP_HOUSEHOLDER;
    if (layers[l].op != want || (want == OP_HOUSEHOLDER && layers[l].k != 1)) return false;
  }
  return true;
}

hipError_t launch_hj_grad(int64_t D, int64_t N, const void* X, const enf_layer* layers, int32_t nlayers,
                          int32_t nparams, double* partial, int blocks, hipStream_t st) {
  HJGradArgs a;
  std::memset(&a, 0, sizeof a);
  a.X = (const float*)X;
  a.N = N;
  a.n = nlayers / 2;
  a.D = (int32_t)D;
  a.partial = partial;
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
  // register variant for <= 4 pairs (ENF_GRAD_REG=0: the LDS variant; ENF_GRAD_RU: its KU)
  static const int reg = ENF_KNOB("ENF_GRAD_REG", 1);
  static const int ru = ENF_KNOB("ENF_GRAD_RU", 1) == 2 ? 2 : 1;  // 1: 215 VGPRs at 4 pairs (2 waves/SIMD)
  if (reg && a.n <= 4) {
    if (D == 32) return ru == 1 ? launch_reg<32, 1>(a, blocks, st) : launch_reg<32, 2>(a, blocks, st);
    return ru == 1 ? launch_reg<64, 1>(a, blocks, st) : launch_reg<64, 2>(a, blocks, st);
  }
  static const int ku = ENF_KNOB("ENF_GRAD_U", 2) == 1 ? 1 : 2;  // 2: measured 72 vs 93 us at config 5
  const size_t lds = D == 32 ? (ku == 1 ? hj_grad_lds<32, 1>(a.n) : hj_grad_lds<32, 2>(a.n))
                             : (ku == 1 ? hj_grad_lds<64, 1>(a.n) : hj_grad_lds<64, 2>(a.n));
  const void* k = D == 32 ? (ku == 1 ? (const void*)&hj_grad_kernel<32, 1> : (const void*)&hj_grad_kernel<32, 2>)
                          : (ku == 1 ? (const void*)&hj_grad_kernel<64, 1> : (const void*)&hj_grad_kernel<64, 2>);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (D == 32) {
    if (ku == 1) hipLaunchKernelGGL((hj_grad_kernel<32, 1>), dim3(blocks), dim3(256), lds, st, a);
    else hipLaunchKernelGGL((hj_grad_kernel<32, 2>), dim3(blocks), dim3(256), lds, st, a);
  } else {
    if (ku == 1) hipLaunchKernelGGL((hj_grad_kernel<64, 1>), dim3(blocks), dim3(256), lds, st, a);
    else hipLaunchKernelGGL((hj_grad_kernel<64, 2>), dim3(blocks), dim3(256), lds, st, a);
  }
  return hipGetLastError();
}

}  // namespace enf
