// enf_hj.h -- the compiled program for the flows of configs 3-5 (enf_flow_hj.hip):
//   J_n o H_n o ... o J_1 o H_1   (layers H_1, J_1, H_2, J_2, ... applied in this order),
// each H one Householder reflection (src/householder_trafo.jl:8-11), each J a JohnsonTrafo
// (src/johnson_trafo.jl:29-32, ladj :39-42 / :76-80), fp32, D in {32, 64, 128}, fused in one launch:
// X is read once, Y and the per-sample ladj are written once.
//
// The register tile carries L_p = asinh(z_p)/ln2 between pairs. Every pair p is the same three full-rate
// operations per element before its asinh (round 6: the interior hop J_{p-1} -> H_p -> J_p folded into
// per-row constants built in double in the block prologue):
//   dot = sum_d W_d L_d                              one FMA chain per column (W = vh_p delta'_{p-1})
//   z_p = fma(-dot, C, fma(L, B, A))                 two FMAs
// with vh = v sqrt(2/v'v), delta' = delta ln2 and, for p >= 1,
//   B = delta'_{p-1}/lambda_p,  A = ((H_p gamma_{p-1}) - xi_p)/lambda_p,  C = vh_p/lambda_p
// because z_p = (H_p(gamma_{p-1} + delta'_{p-1} L_{p-1}) - xi_p)/lambda_p and H_p y = y - vh (vh'y) is
// linear: the constant part H_p gamma_{p-1} goes into A, the L part into W and B. Pair 0 reads X itself:
// W = vh_0, B = 1/lambda_0, A = -xi_0/lambda_0, C = vh_0/lambda_0. The output is y_n = fma(L_n, delta'_n,
// gamma_n) from record n. Against round 5's explicit y = gamma + delta' L before each reflection this is
// one dependent FMA less per element and interior pair (4 -> 3). Round 1 tried a fold of gamma / delta'
// alone and lost accuracy where y cancels; this one keeps every term the reference has: its rounding
// errors are those of the reference's y (eps |delta' L|, which the reference incurs in delta*asinh) and of
// the constants (rounded once, from double). Priced on the CPU before it was built (tools/hj_fold_emul.py:
// the per-element criterion of tests/test_gpu_fp32_accuracy.py at D = 32 / 64, worst 0.59 / 0.52 of the
// bound against 0.75 / 0.46 for the round-5 form).
//   L_p = asinh(z_p)/ln2                             asinh2 (enf_frag.h): log2(|z| + sqrt(q)),
//                                                    q = 1 + z^2, or the Taylor form for |z| < 1/8
//   ladj = sum log|delta/lambda| - 1/2 sum log q     johnson_trafo.jl:41; the constant part once per
//                                                    column (ctot); the q of a lane's 8 rows of one column
//                                                    multiplied over ALL pairs (round 6: one log2 per lane
//                                                    and column per tile instead of one per pair)
//
// Parameter records (LDS, built in double in each block's prologue): per pair and row {W, B, A, C}; record
// n holds {0, delta'_n, gamma_n, 0} (the output: y = fma(L, B, A)).
//
// Fast-path guard: the running product of q stays finite unless the column's z are large (the sum of
// log2 q over a lane's 8 rows and n pairs above 128: about |z| > 4 on every one of them for n = 4; the
// survey's distributions reach 62, tools/hj_fold_emul.py), infinite or NaN; then the lanes of that
// column redo the whole program from X with the exact-range elementwise form (asinh finite up to FLT_MAX,
// ladj -Inf where the reference's fp32 1 + z^2 overflows).
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "enf_frag.h"
#include "enf_internal.h"

namespace enf {

constexpr int kHjMaxPairs = 8;
constexpr int kHjW = 4;  // record parameters per row: W, B, A, C

// Kernel arguments of the compiled program: the pair parameter vectors only (376 bytes; the
// generic FlowArgs table is ~2 KB, and kernel arguments that large are staged with an extra
// copy kernel per launch).
struct HJArgs {
  const void* X;
  void* Y;
  void* ladj;
  int64_t N;
  int32_t n;        // pairs
  int32_t dreal;    // rows of the batch: D, or fewer on the padded layout (PAD: rows past dreal are inert)
  const float* v[kHjMaxPairs];  // reflection vector (column of V) of pair p
  const float* g[kHjMaxPairs];  // Johnson gamma, delta, xi, lambda of pair p
  const float* d[kHjMaxPairs];
  const float* xi[kHjMaxPairs];
  const float* lam[kHjMaxPairs];
};
// LDS: [per pair {hs, cl, vh'gamma} + ctot: doubles][ladj staging: 4 waves x kStagePerWave floats][records]
constexpr size_t kHjScratch = ((3 * kHjMaxPairs + 1) * sizeof(double) + 15) / 16 * 16;
constexpr size_t kHjHeader = kHjScratch + 4 * kStagePerWave * sizeof(float);

static size_t hj_lds_bytes(int D, int n) { return kHjHeader + (size_t)(n + 1) * kHjW * D * sizeof(float); }

// Register layout of the compiled program: a lane owns R rows of ONE column as NF = R/4 16-byte
// fragments; fragment h holds rows h*(D/NF) + 4*g .. +3 with g = lane % G the lane's row group and
// G = D/R lanes per column (adjacent lanes). A slab is one load instruction per fragment and
// covers CPS = 64/G columns; a wave tile is U slabs. R = 8 halves the DPP reduction stages of the
// Householder dot and the ladj column sum against R = 4 and gives one ladj log2 per 8 rows; the
// price is that a D = 32 load instruction covers half of each 128-byte column line (16 lines, the
// other halves follow in the next instruction).
template <int D, int R, int U>
struct HJLay {
  static constexpr int NF = R / 4;
  static constexpr int G = D / R;
  static constexpr int CPS = 64 / G;
  static constexpr int TC = CPS * U;  // columns per wave tile
  static constexpr int NLS = (TC + 63) / 64;
  static_assert(R % 4 == 0 && D % R == 0 && G >= 2 && G <= 64, "layout");
  static_assert(TC <= kStagePerWave, "ladj staging");
  __device__ static __forceinline__ int64_t col(int64_t col0, int u, int lane) {
    return col0 + (int64_t)u * CPS + lane / G;
  }
  __device__ static __forceinline__ int row(int h, int lane) { return h * (D / NF) + 4 * (lane % G); }
  __device__ static __forceinline__ int64_t ladj_col(int64_t col0, int k, int lane) {
    return col0 + (int64_t)k * 64 + (TC >= 64 ? lane : lane % TC);
  }
};

// VGPR banks (register index mod 4): an FMA whose three source VGPRs sit in one bank issues at
// half rate on gfx950 (tools/microbench5: 1.8 vs 1.0-1.2 ns per wave-instruction). The tile and the
// records arrive by 16-byte loads into 4-register tuples whose bases the compiler aligns to even
// registers, so x[e] and the e-th value of every record vector would share a bank. The multiplier
// of each FMA (W with L in the dot, B with L, C with the previous result) is therefore stored one slot
// rotated within its 16-byte vector: row e uses slot hj_rot(e), an odd register distance from x[e]'s.
__host__ __device__ constexpr int hj_rot(int e) { return (e & ~3) | ((e + 1) & 3); }
enum : int { HJ_W = 0, HJ_B = 1, HJ_A = 2, HJ_C = 3 };
__host__ __device__ constexpr bool hj_rotated(int q) { return q != HJ_A; }

// DBG (diagnostic builds, ENF_DEBUG_MODE): 1 = synthesize the tile instead of loading it, 2 = also
// skip the stores (compute-only timing); cache policy A/B: 8 = nontemporal loads, 9 = plain stores.
// The product loads X with plain loads (0.800 / 0.798 vs 0.808 / 0.805 ms with nontemporal loads,
// profiles/r02_cache_policy_ab.jsonl) and writes Y with nontemporal stores (plain: 0.810 / 0.822).
// PAD (padded layout, round 3): D is the power-of-two layout, columns are a.dreal rows apart, and a
// fragment whose rows start at or past a.dreal holds zeros and is neither loaded nor stored (a.dreal is
// a multiple of 4, so a fragment is wholly inside or outside).
template <int D, int R, int U, bool TAIL, int DBG, bool PAD = false>
__device__ __forceinline__ void hj_load(const HJArgs& a, int64_t col0, float (&x)[U][R]) {
  using L = HJLay<D, R, U>;
  const int lane = threadIdx.x & 63;
  const float* __restrict__ X = (const float*)a.X;
  const int64_t ld = PAD ? (int64_t)a.dreal : (int64_t)D;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t c = L::col(col0, u, lane);
#pragma unroll
    for (int h = 0; h < L::NF; ++h) {
      const int64_t off = c * ld + L::row(h, lane);
      if (PAD && L::row(h, lane) >= a.dreal) {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[u][4 * h + e] = 0.f;
      } else if (DBG == 1 || DBG == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[u][4 * h + e] = (float)(lane + 3 * u + 5 * h + e) * 0.03125f - 1.f;
      } else if (!TAIL) {
        if (ENF_INB(c < a.N, "hj load X", c, a.N)) {
          const u32x4 v4 = DBG == 8 ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(X + off))
                                    : *reinterpret_cast<const u32x4*>(X + off);
          __builtin_memcpy(&x[u][4 * h], &v4, 16);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[u][4 * h + e] = c < a.N ? X[off + e] : 0.f;
      }
    }
  }
}

template <int D, int R, int U, int LM>
__device__ __forceinline__ void hj_load_old(const HJArgs& a, int64_t col0, float (&old)[HJLay<D, R, U>::NLS],
                                            bool tail) {
  using L = HJLay<D, R, U>;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < L::NLS; ++k) {
    const int64_t c = L::ladj_col(col0, k, lane);
    old[k] = (LM == 2 && (!tail || c < a.N)) ? ((const float*)a.ladj)[c] : 0.f;
  }
}

// Y fragments, then the ladj: column totals (group sums over the G lanes of a column) staged
// through the wave's LDS slots and written by NLS full-wave coalesced stores.
template <int D, int R, int U, int LM, bool TAIL, int DBG, bool PAD = false>
__device__ __forceinline__ void hj_store(const HJArgs& a, float ctot, int64_t col0, float (&x)[U][R],
                                         const float (&acc)[U], const float (&old)[HJLay<D, R, U>::NLS],
                                         float* __restrict__ stage) {
  using L = HJLay<D, R, U>;
  const int lane = threadIdx.x & 63;
  float* __restrict__ Y = (float*)a.Y;
  const int64_t ld = PAD ? (int64_t)a.dreal : (int64_t)D;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t c = L::col(col0, u, lane);
#pragma unroll
    for (int h = 0; h < L::NF; ++h) {
      const int64_t off = c * ld + L::row(h, lane);
      if (PAD && L::row(h, lane) >= a.dreal) {
        continue;
      } else if (DBG == 2) {
        if (x[u][4 * h] == 1234.5f) Y[off] = x[u][4 * h + 1];  // keeps the compute alive
      } else if (!TAIL) {
        u32x4 v4;
        __builtin_memcpy(&v4, &x[u][4 * h], 16);
        if (!ENF_INB(c < a.N, "hj store Y", c, a.N)) continue;
        if (DBG == 9) *reinterpret_cast<u32x4*>(Y + off) = v4;
        else __builtin_nontemporal_store(v4, reinterpret_cast<u32x4*>(Y + off));
      } else if (c < a.N) {
#pragma unroll
        for (int e = 0; e < 4; ++e) Y[off + e] = x[u][4 * h + e];
      }
    }
  }
  if constexpr (LM > 0) {
    float* __restrict__ ladj = (float*)a.ladj;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float tot = group_sum<L::G>(acc[u]);
      if ((lane % L::G) == 0) stage[u * L::CPS + lane / L::G] = tot;
    }
#pragma unroll
    for (int k = 0; k < L::NLS; ++k) {
      const int c = k * 64 + (L::TC >= 64 ? lane : lane % L::TC);
      const float w = fmaf((float)kLn2, stage[c], ctot);
      const float v = LM == 2 ? w + old[k] : w;  // (LM 1: no add of the zero `old`)
      const int64_t col = col0 + c;
      if ((!TAIL && ENF_INB(col < a.N, "hj ladj", col, a.N)) || (TAIL && col < a.N)) ladj[col] = v;
    }
  }
}

// Records, pair p <= n: [group g][param q][R values, value 4h+e = row h*D/NF+4g+e, rotated slot for
// the multipliers]. A lane reads each parameter of its rows with NF 16-byte LDS reads.
template <int D, int R>
__device__ void build_hj_program(const HJArgs& a, int n, float* __restrict__ rec, double* __restrict__ scr,
                                 float* ctot) {
  constexpr int NF = R / 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // pass 1 (one wave per pair): v'v, the constant ladj part sum_d log|delta/lambda| (johnson_trafo.jl:41)
  // and v'gamma_{p-1} (the reflection of the previous Johnson layer's shift, folded into A) in double
  for (int p = wave; p < n; p += nw) {
    const float* v = a.v[p];
    double vv = 0.0, cl = 0.0, vg = 0.0;
    for (int d = lane; d < a.dreal; d += 64) {  // the batch's rows (padded rows: neutral records below)
      const double vd = v[d];
      vv += vd * vd;
      cl += log(fabs((double)a.d[p][d])) - log(fabs((double)a.lam[p][d]));
      if (p > 0) vg += vd * (double)a.g[p - 1][d];
    }
    for (int m = 32; m >= 1; m >>= 1) {
      vv += __shfl_xor(vv, m);
      cl += __shfl_xor(cl, m);
      vg += __shfl_xor(vg, m);
    }
    if (lane == 0) {
      const double hs = sqrt(2.0 / vv);  // householder_trafo.jl:9-10: 2 v (v'x) / (v'v)
      scr[3 * p] = hs;
      scr[3 * p + 1] = cl;
      scr[3 * p + 2] = hs * vg;  // vh'gamma_{p-1}
    }
  }
  __syncthreads();
  // pass 2: records
  for (int i = threadIdx.x; i < (n + 1) * D; i += blockDim.x) {
    const int p = i / D, d = i % D;
    const int h = d / (D / NF), w = d % (D / NF), g = w / 4, e = w % 4;
    float* r = rec + (size_t)p * kHjW * D + g * kHjW * R + 4 * h;
    // a padded row (d >= dreal): W = C = 0, B = 1, A = 0 -- its zeros stay zero, with q = 1 (ladj 0);
    // its ladj constant is not in ctot (pass 1)
    const bool real = d < a.dreal;
    double q[kHjW] = {0.0, 1.0, 0.0, 0.0};
    if (p == n) {  // the output y_n = gamma_n + delta'_n L_n
      if (real) {
        q[HJ_B] = (double)a.d[p - 1][d] * kLn2;
        q[HJ_A] = (double)a.g[p - 1][d];
      }
    } else if (real) {
      const double vh = (double)a.v[p][d] * scr[3 * p];
      const double il = 1.0 / (double)a.lam[p][d];
      const double xi = (double)a.xi[p][d];
      if (p == 0) {
        q[HJ_W] = vh;
        q[HJ_B] = il;
        q[HJ_A] = -xi * il;
      } else {
        const double dp = (double)a.d[p - 1][d] * kLn2;
        const double hg = (double)a.g[p - 1][d] - vh * scr[3 * p + 2];  // (H_p gamma_{p-1})_d
        q[HJ_W] = vh * dp;
        q[HJ_B] = dp * il;
        q[HJ_A] = (hg - xi) * il;
      }
      q[HJ_C] = vh * il;
    }
#pragma unroll
    for (int k = 0; k < kHjW; ++k) r[k * R + (hj_rotated(k) ? hj_rot(e) : e)] = (float)q[k];
  }
  if (threadIdx.x == 0) {
    double c = 0.0;
    for (int p = 0; p < n; ++p) c += scr[3 * p + 1];
    *ctot = (float)c;
  }
  __syncthreads();
}

// One record's parameters of the lane's rows (kHjW x R values).
template <int R>
struct HJParams {
  float v[kHjW][R];
  __device__ __forceinline__ void load(const float* r) {
#pragma unroll
    for (int k = 0; k < kHjW; ++k)
#pragma unroll
      for (int h = 0; h < R / 4; ++h) lds_vec<float, 4>(r + k * R + 4 * h, *reinterpret_cast<float(*)[4]>(&v[k][4 * h]));
  }
  __device__ __forceinline__ float m(int k, int e) const { return v[k][hj_rotated(k) ? hj_rot(e) : e]; }
};

// Householder dot of every column of the tile: two independent partial chains per column (even
// and odd rows) over the lane's R rows, then log2(G) DPP stages across the G lanes of the column.
// (Q: the record slot of the row weights in the parameter set P)
// CH: partial chains per column -- 1 (product, round 6): one chain of R, no add; 2 (rounds 1-5): even / odd rows,
// one add to combine. One chain: 0.595 vs 0.603 ms on config 3 (9.08M vs 9.35M cycles, interleaved A/B,
// profiles/r06/ballot_ab_v1.jsonl): the dependent FMAs hide behind the other column and the other waves.
template <int D, int R, int U, int Q = HJ_W, typename P = HJParams<R>, int CH = 1>
__device__ __forceinline__ void hj_dots(const float (&y)[U][R], const P& prm, float (&dot)[U]) {
  constexpr int G = HJLay<D, R, U>::G;
  if constexpr (CH == 1) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u] = prm.m(Q, 0) * y[u][0];
#pragma unroll
    for (int e = 1; e < R; ++e)
#pragma unroll
      for (int u = 0; u < U; ++u) dot[u] = fmaf(prm.m(Q, e), y[u][e], dot[u]);
  } else {
    float d2[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < 2; ++c) d2[u][c] = prm.m(Q, c) * y[u][c];
#pragma unroll
    for (int e = 2; e < R; ++e)
#pragma unroll
      for (int u = 0; u < U; ++u) d2[u][e & 1] = fmaf(prm.m(Q, e), y[u][e], d2[u][e & 1]);
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u] = d2[u][0] + d2[u][1];
  }
  if constexpr (G >= 2) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u] += dpp<0xB1>(dot[u]);
  }
  if constexpr (G >= 4) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u] += dpp<0x4E>(dot[u]);
  }
  if constexpr (G >= 8) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u] += dpp<0x141>(dot[u]);
  }
  if constexpr (G >= 16) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u] += dpp<0x140>(dot[u]);
  }
  if constexpr (G >= 32) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u] += __shfl_xor(dot[u], 16);
  }
  if constexpr (G >= 64) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u] += __shfl_xor(dot[u], 32);
  }
}

// Product of the R values of a row of q, as a balanced tree.
template <int R>
__device__ __forceinline__ float prod_tree(const float (&q)[R]) {
  float t[R / 2];
#pragma unroll
  for (int i = 0; i < R / 2; ++i) t[i] = q[2 * i] * q[2 * i + 1];
  if constexpr (R == 4) {
    return t[0] * t[1];
  } else if constexpr (R == 8) {
    return (t[0] * t[1]) * (t[2] * t[3]);
  } else {
    float s = 1.f;
#pragma unroll
    for (int i = 0; i < R / 2; ++i) s *= t[i];
    return s;
  }
}

// The front of one pair, in place on the tile (x: L_{p-1}, or X for p = 0, on entry; z_p on exit):
// dot = W'x over the column, z = fma(-dot, C, fma(x, B, A)).
template <int D, int R, int U>
__device__ __forceinline__ void hj_front(float (&x)[U][R], const HJParams<R>& prm) {
  float dot[U];
  hj_dots<D, R, U>(x, prm, dot);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) x[u][e] = fmaf(x[u][e], prm.m(HJ_B, e), prm.m(HJ_A, e));
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) x[u][e] = fmaf(-dot[u], prm.m(HJ_C, e), x[u][e]);
}

// One pair (reflection + Johnson) on the register tile, fast form. x holds L_{p-1} (pair 0: the input x)
// on entry and L_p on exit; prm holds this pair's record on entry and the next one's on exit (r is
// advanced to it; read after the asinh's temporaries are dead: 128 VGPRs and 65 spilled when the reads were
// issued before the asinh, and reading W early and the rest late measured no better, profiles/r06/var_ab_v1.jsonl).
// prod[u] accumulates the product of the
// q = 1 + z^2 of the lane's R rows of column u (+Inf / NaN: the fast form is not valid for the tile).
// asinh: the mask-first merge asinh2_mask / asinh2_pick of the Taylor form and the log form (enf_frag.h).
template <int D, int R, int U>
__device__ __forceinline__ void hj_pair_fast(float (&x)[U][R], float (&prod)[U], const float*& r, HJParams<R>& prm,
                                             uint32_t csign) {
  hj_front<D, R, U>(x, prm);
  r += kHjW * D;
  // stage by stage over the whole tile (U*R independent chains per stage)
  float q[U][R], t[U][R];
  uint32_t msel[U][R];  // the select mask of asinh2_pick, from q (before the transcendentals)
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) q[u][e] = fmaf(x[u][e], x[u][e], 1.0f);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) msel[u][e] = asinh2_mask(q[u][e], csign);
  // Wave priority 3 while a wave issues its sqrt / log2 group, 0 otherwise (round 3): the SIMD's arbiter
  // then issues the transcendentals of the waves in that phase first and fills the transcendental pipe's
  // busy cycles with the other waves' FMAs, instead of picking by age. 0.682 / 0.683 / 0.686 vs
  // 0.725 / 0.721 / 0.723 ms streaming (profiles/r03_setprio_ab.jsonl; the other placements measured then
  // were slower or within noise: r03_setprio_placement_ab.jsonl, r03_setprio_placement2_ab.jsonl).
  __builtin_amdgcn_s_setprio(3);
  if constexpr (R == 8) {
#pragma unroll
    for (int u = 0; u < U; ++u) sqrt8(t[u], q[u]);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < R; ++e) t[u][e] = hw_sqrt(q[u][e]);
  }
  __builtin_amdgcn_s_setprio(0);
#pragma unroll
  for (int u = 0; u < U; ++u) prod[u] *= prod_tree<R>(q[u]);
  // small |z|: the Taylor form (enf_frag.h) in place of q
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) q[u][e] = asinh2_small(x[u][e], q[u][e]);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) t[u][e] = fabsf(x[u][e]) + t[u][e];
  __builtin_amdgcn_s_setprio(3);
  if constexpr (R == 8) {
#pragma unroll
    for (int u = 0; u < U; ++u) log2_8_inplace(t[u]);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < R; ++e) t[u][e] = hw_log2(t[u][e]);
  }
  __builtin_amdgcn_s_setprio(0);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) x[u][e] = asinh2_pick(q[u][e], t[u][e], msel[u][e]);
  prm.load(r);
}

// The same pair in the exact-range elementwise form: asinh finite up to FLT_MAX (log2(2|z|) above 1e18),
// ladj -Inf where the reference's fp32 1 + z^2 overflows (johnson_trafo.jl:41).
template <int D, int R, int U>
__device__ __forceinline__ void hj_pair_exact(float (&x)[U][R], float (&acc)[U], const float*& r, HJParams<R>& prm,
                                              uint32_t csign) {
  hj_front<D, R, U>(x, prm);
  r += kHjW * D;
  prm.load(r);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) {
      const float z = x[u][e];
      const float q = fmaf(z, z, 1.0f);
      x[u][e] = fabsf(z) > 1e18f ? copysignf(hw_log2(fabsf(z)) + 1.0f, z) : asinh2_f32(z, q, hw_sqrt(q), csign);
      acc[u] = fmaf(-0.5f, hw_log2(q), acc[u]);
    }
}

// Whether the fast form is invalid for a column of the lane's tile, the same on the G lanes of a column: a running
// q product that is not finite. (Tested per lane as a flag, not as a max of the products: an overflow in one pair
// is followed by Inf * 0 = NaN products in the next ones when the huge z turn into Inf - Inf in the next front,
// and fmaxf drops NaN operands. The flags of the wave by one ballot, then the lane's G-bit group of it: fewer
// VALU operations than a DPP max over the group. A wave-uniform test, redoing the whole wave tile, made the
// compiler spill 97 VGPRs.)
template <int G, int U>
__device__ __forceinline__ bool hj_redo(const float (&prod)[U]) {
  bool ok = true;
#pragma unroll
  for (int u = 0; u < U; ++u) ok = ok && prod[u] <= FLT_MAX;
  const uint64_t bad = __builtin_amdgcn_ballot_w64(!ok);
  if (bad == 0) return false;  // (uniform: the common case takes no per-lane work)
  const int lane = threadIdx.x & 63;
  return ((bad >> (lane & ~(G - 1))) & ((G >= 64 ? ~0ull : (1ull << G) - 1))) != 0;
}

template <int D, int R, int U, int LM, bool PAD = false>
struct HJBody {
  const HJArgs& a;
  const float* rec;  // this lane's record group
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
    const uint32_t csign = sign_mask_vgpr();
    // branch-free pair loop; a tile with a product overflow (|z| large, Inf, NaN) is redone below
    for (int p = 0; p < n; ++p) hj_pair_fast<D, R, U>(x, prod, r, prm, csign);
    // wave-uniform: the exact form's dot products read every lane of a column (DPP)
    if (__builtin_expect(hj_redo<HJLay<D, R, U>::G>(prod), 0)) {
      hj_load<D, R, U, TAIL, DBG, PAD>(a, col0, x);
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = 0.f;
      r = rec;
      prm.load(r);
      for (int p = 0; p < n; ++p) hj_pair_exact<D, R, U>(x, acc, r, prm, csign);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = -0.5f * hw_log2(prod[u]);
    }
    // the output y_n = gamma_n + delta'_n L_n (record n). (Writing this epilogue out in both branches, so that the
    // wait-count pass does not see the redo branch's reload of X outstanding at the join, measured the same:
    // 0.597 vs 0.594 ms, interleaved, profiles/r06/epi_ab_v1.jsonl.)
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < R; ++e) x[u][e] = fmaf(x[u][e], prm.m(HJ_B, e), prm.m(HJ_A, e));
    hj_store<D, R, U, LM, TAIL, DBG, PAD>(a, ctot, col0, x, acc, old, stage);
  }
};

// Persistent, software-pipelined tile loop (as frag_stream in enf_frag.h, for the HJLay layout):
// wave w processes tiles w, w + nwaves, ...; the next tile's loads are in flight while this tile
// computes; the ragged last tile (N not a multiple of the tile) is processed by one wave.
template <int D, int R, int U, int LM, int DBG, bool PAD, typename Body>
__device__ __forceinline__ void hj_stream(const HJArgs& a, Body& body) {
  using L = HJLay<D, R, U>;
  constexpr int64_t CT = L::TC;
  const int64_t ntiles_full = a.N / CT;
  const int64_t wave_id = (int64_t)blockIdx.x * (blockDim.x >> 6) +
                          __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  float xa[U][R], xb[U][R], old[L::NLS];
  const int64_t t = wave_id;
  if (t < ntiles_full) {
    hj_load<D, R, U, false, DBG, PAD>(a, t * CT, xa);
    int64_t t1 = t + nwaves;
    hj_load_old<D, R, U, LM>(a, t * CT, old, false);
    hj_load<D, R, U, false, DBG, PAD>(a, (t1 < ntiles_full ? t1 : t) * CT, xb);
    body.template tile<false, DBG>(t * CT, xa, old);
    while (t1 < ntiles_full) {
      const int64_t t2 = t1 + nwaves;
      hj_load_old<D, R, U, LM>(a, t1 * CT, old, false);
      hj_load<D, R, U, false, DBG, PAD>(a, (t2 < ntiles_full ? t2 : t1) * CT, xa);
      body.template tile<false, DBG>(t1 * CT, xb, old);
      if (t2 >= ntiles_full) break;
      const int64_t t3 = t2 + nwaves;
      hj_load_old<D, R, U, LM>(a, t2 * CT, old, false);
      hj_load<D, R, U, false, DBG, PAD>(a, (t3 < ntiles_full ? t3 : t2) * CT, xb);
      body.template tile<false, DBG>(t2 * CT, xa, old);
      t1 = t3;
    }
  }
  if (ntiles_full * CT < a.N && wave_id == ntiles_full % nwaves) {
    const int64_t c0 = ntiles_full * CT;
    hj_load<D, R, U, true, 0, PAD>(a, c0, xa);
    hj_load_old<D, R, U, LM>(a, c0, old, true);
    body.template tile<true, 0>(c0, xa, old);
  }
}

template <int D, int R, int U, int LM, int OCC, int DBG, bool PAD = false>
__global__ __launch_bounds__(256, OCC) void flow_hj_kernel(HJArgs a) {
  const int n = a.n;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* scr = reinterpret_cast<double*>(smem);
  float* ctotp = reinterpret_cast<float*>(scr + 3 * kHjMaxPairs);
  float* stage = reinterpret_cast<float*>(smem + kHjScratch) + (threadIdx.x >> 6) * kStagePerWave;
  float* rec = reinterpret_cast<float*>(smem + kHjHeader);
  build_hj_program<D, R>(a, n, rec, scr, ctotp);
  constexpr int G = HJLay<D, R, U>::G;
  HJBody<D, R, U, LM, PAD> body{a, rec + ((threadIdx.x & 63) % G) * kHjW * R, *ctotp, stage, n};
  hj_stream<D, R, U, LM, DBG, PAD>(a, body);
}

template <int D, int R, int U, int LM, int OCC = 1, int DBG = 0, bool PAD = false>
static hipError_t launch_hj(const HJArgs& h, hipStream_t st, const DeviceInfo& dev) {
  const size_t lds = hj_lds_bytes(D, h.n);
  const void* k = reinterpret_cast<const void*>(&flow_hj_kernel<D, R, U, LM, OCC, DBG, PAD>);
  int64_t blocks = 0;
  hipError_t e = frag_grid(k, h.N, (int64_t)HJLay<D, R, U>::TC * 4, lds, dev, &blocks);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((flow_hj_kernel<D, R, U, LM, OCC, DBG, PAD>), dim3((unsigned)blocks), dim3(256), lds, st, h);
  return hipGetLastError();
}

}  // namespace enf
