// enf_flow_hj.hip -- compiled program for the flows of configs 3-5:
//   J_n o H_n o ... o J_1 o H_1   (layers H_1, J_1, H_2, J_2, ... applied in this order),
// each H one Householder reflection (src/householder_trafo.jl:8-11), each J a JohnsonTrafo
// (src/johnson_trafo.jl:29-32, ladj :39-42 / :76-80), fp32, D in {32, 64}, fused in one launch:
// X is read once, Y and the per-sample ladj are written once.
//
// Per pair p (the register tile holds y, the previous Johnson output, on entry -- X itself for p = 0):
//   dot = vh'y,  vh = v sqrt(2/v'v)                 householder_trafo! (householder_trafo.jl:8-11)
//   z   = (y - dot vh)/lambda - xi/lambda           the reflection's output, then (x - xi)/lambda as
//                                                    fma(x, 1/lambda, -xi/lambda) (johnson_trafo.jl:30)
//   L_p = asinh(z)/ln2                              asinh2 (enf_frag.h): log2(|z| + sqrt(q)),
//                                                    q = 1 + z^2, or the Taylor form for |z| < 1/8
//   ladj += log|delta/lambda| - log(q)/2            johnson_trafo.jl:41; the constant part once per
//                                                    column (ctot), -1/2 log2 of the product of the q
//                                                    of a lane's 8 rows of one column
//   y   = gamma_p + delta'_p L_p                    at the end of the pair, delta' = delta*ln2
// so the last pair leaves the output in the tile. y is formed explicitly, as the reference rounds it,
// before the next reflection: folding gamma and delta' into the next pair's constants (round 1) saves one
// FMA per element but adds terms that the reference has already cancelled, and gave up to 16x the
// reference's error on elements where y cancels (tests/test_gpu_fp32_accuracy.py per-element test).
// Per element and pair: 4 FMAs (dot, 2 for z, y), q, sqrt, |z| + s, log2, the small-|z| polynomial
// (3) and its branch-free merge (4 full-rate ops), 7/8 multiply for the ladj product.
//
// Parameter records (LDS, built in double in each block's prologue): per pair and row
// {delta', gamma, vh, 1/lambda, -xi/lambda, vh/lambda}; record p's {delta', gamma} slots hold pair p-1's
// (read at the end of pair p-1, which applies them; record 0's {1, 0} is not used), record n holds
// {delta'_n, gamma_n}.
//
// Fast-path guard: the product of 8 q stays finite unless |z| is large (about 2^8 on every row),
// infinite or NaN; then the lanes of that column redo the whole program from X with the exact-range
// elementwise form (johnson_fwd_f32_slow in enf_frag.h: asinh finite up to FLT_MAX, ladj -Inf where
// the reference's fp32 1 + z^2 overflows).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "enf_frag.h"
#include "enf_internal.h"

namespace enf {

constexpr int kHjMaxPairs = 8;
constexpr int kHjW = 6;  // record parameters per row

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
// LDS: [per pair {hs, cl} + ctot: doubles][ladj staging: 4 waves x kStagePerWave floats][records]
constexpr size_t kHjScratch = ((2 * kHjMaxPairs + 1) * sizeof(double) + 15) / 16 * 16;
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
// of each FMA (delta', vh, 1/lambda, vh/lambda) is therefore stored one slot rotated within its
// 16-byte vector: row e uses slot hj_rot(e), an odd register distance from x[e]'s.
__host__ __device__ constexpr int hj_rot(int e) { return (e & ~3) | ((e + 1) & 3); }
enum : int { HJ_DP = 0, HJ_GP = 1, HJ_VH = 2, HJ_IL = 3, HJ_NXI = 4, HJ_RR = 5 };
__host__ __device__ constexpr bool hj_rotated(int q) { return q == HJ_DP || q == HJ_VH || q == HJ_IL || q == HJ_RR; }

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
      const float v = fmaf((float)kLn2, stage[c], ctot) + old[k];
      const int64_t col = col0 + c;
      if ((!TAIL && ENF_INB(col < a.N, "hj ladj", col, a.N)) || (TAIL && col < a.N)) ladj[col] = v;
    }
  }
}

// Records, pair p < n: [group g][param q][R values, value 4h+e = row h*D/NF+4g+e, rotated slot for
// the multipliers]; record n: {delta'_{n-1}, gamma_{n-1}} (the output). A lane reads each parameter
// of its rows with NF 16-byte LDS reads.
template <int D, int R, int AS>
__device__ void build_hj_program(const HJArgs& a, int n, float* __restrict__ rec, double* __restrict__ scr,
                                 float* ctot) {
  // AS == 2 (asinh2_med3): z is carried as sqrt(K) z, so the three z records are scaled by sqrt(K)
  const double zs = AS == 2 ? kAsinhSqrtK : 1.0;
  constexpr int NF = R / 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // pass 1 (one wave per pair): v'v and the constant ladj part sum_d log|delta/lambda|
  // (johnson_trafo.jl:41) in double
  for (int p = wave; p < n; p += nw) {
    const float* v = a.v[p];
    double vv = 0.0, cl = 0.0;
    for (int d = lane; d < a.dreal; d += 64) {  // the batch's rows (padded rows: neutral records below)
      const double vd = v[d];
      vv += vd * vd;
      cl += log(fabs((double)a.d[p][d])) - log(fabs((double)a.lam[p][d]));
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
  // pass 2: records
  for (int i = threadIdx.x; i < (n + 1) * D; i += blockDim.x) {
    const int p = i / D, d = i % D;
    const int h = d / (D / NF), w = d % (D / NF), g = w / 4, e = w % 4;
    float* r = rec + (size_t)p * kHjW * D + g * kHjW * R + 4 * h;
    double q[kHjW] = {0, 0, 0, 0, 0, 0};
    // a padded row (d >= dreal): vh = 0, 1/lambda = 1, -xi/lambda = 0, gamma = 0 -- its zeros stay zero,
    // with q = 1 (ladj 0); its ladj constant is not in ctot (pass 1)
    const bool real = d < a.dreal;
    q[HJ_DP] = p > 0 && real ? (double)a.d[p - 1][d] * kLn2 : 1.0;
    q[HJ_GP] = p > 0 && real ? (double)a.g[p - 1][d] : 0.0;
    q[HJ_IL] = 1.0;
    if (p < n && real) {
      const double vh = (double)a.v[p][d] * scr[2 * p];
      const double il = zs / (double)a.lam[p][d];
      q[HJ_VH] = vh;
      q[HJ_IL] = il;
      q[HJ_NXI] = -(double)a.xi[p][d] * il;
      q[HJ_RR] = vh * il;  // sqrt(K) vh / lambda
    }
#pragma unroll
    for (int k = 0; k < kHjW; ++k) r[k * R + (hj_rotated(k) ? hj_rot(e) : e)] = (float)q[k];
  }
  if (threadIdx.x == 0) {
    double c = 0.0;
    for (int p = 0; p < n; ++p) c += scr[2 * p + 1];
    // AS == 2: the fast form sums -log2(q')/2 = -log2(q)/2 - log2(K)/2 per element (ln2 * acc)
    if (AS == 2) c += 0.5 * D * n * log(kAsinhK);
    *ctot = (float)c;
  }
  __syncthreads();
}

// One pair's parameters of the lane's rows (6 x R values): the first three are read at the end of
// the previous pair, the last three at the start of the pair (they are needed after the dot).
template <int R>
struct HJParams {
  float v[kHjW][R];
  template <int Q0, int Q1>
  __device__ __forceinline__ void load(const float* r) {
#pragma unroll
    for (int k = Q0; k < Q1; ++k)
#pragma unroll
      for (int h = 0; h < R / 4; ++h) lds_vec<float, 4>(r + k * R + 4 * h, *reinterpret_cast<float(*)[4]>(&v[k][4 * h]));
  }
  __device__ __forceinline__ float m(int k, int e) const { return v[k][hj_rotated(k) ? hj_rot(e) : e]; }
};

// Householder dot of every column of the tile: two independent partial chains per column (even
// and odd rows) over the lane's R rows, then log2(G) DPP stages across the G lanes of the column.
// (Q: the record slot of vh in the parameter set P)
template <int D, int R, int U, int Q = HJ_VH, typename P = HJParams<R>>
__device__ __forceinline__ void hj_dots(const float (&y)[U][R], const P& prm, float (&dot)[U]) {
  constexpr int G = HJLay<D, R, U>::G;
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

// The dot and z of one pair, in place on the tile (x: the pair's input y on entry, z on exit).
// In the reference's operation order: the reflection's output y - vh (vh'y), then (. - xi)/lambda as
// fma(., 1/lambda, -xi/lambda) (the records' vh/lambda slot is not read).
template <int D, int R, int U, bool RL = true>
__device__ __forceinline__ void hj_pair_z(float (&x)[U][R], const float* r, HJParams<R>& prm) {
  if constexpr (RL) prm.template load<HJ_IL, HJ_RR>(r);
  float dot[U];
  hj_dots<D, R, U>(x, prm, dot);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) x[u][e] = fmaf(-dot[u], prm.m(HJ_VH, e), x[u][e]);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) x[u][e] = fmaf(x[u][e], prm.m(HJ_IL, e), prm.m(HJ_NXI, e));
}

// One pair (reflection + Johnson) on the register tile, fast form. x holds L (pair 0: the input x)
// on entry and the new L on exit; r points at the lane's record group of this pair and is advanced
// to the next record (whose first three parameters are read at the end). Returns the largest
// product of q = 1 + z^2 over a lane's R rows of one column (+Inf / NaN: the fast form is not valid
// for the tile). AS selects the asinh form: 1 = the mask-first merge asinh2_mask / asinh2_pick (the
// product), and in the diagnostics build only 3 = the same merge with its mask taken from the log2
// (asinh2_merge), 2 = asinh2_med3 (z' = sqrt(K) z, enf_frag.h) and 0 = round 1's absolute-error form.
// The Johnson part of one pair (AS = 1 form) on ONE slab of the tile (VAR bit 1, diagnostics build):
// the temporaries of one slab only, for a lower register count (occupancy 5).
template <int R, bool LADJ>
__device__ __forceinline__ float hj_johnson_slab(float (&x)[R], float& acc, uint32_t csign) {
  float q[R], t[R];
  uint32_t msel[R];
#pragma unroll
  for (int e = 0; e < R; ++e) q[e] = fmaf(x[e], x[e], 1.0f);
#pragma unroll
  for (int e = 0; e < R; ++e) msel[e] = asinh2_mask(q[e], csign);
  __builtin_amdgcn_s_setprio(3);  // the wave-priority schedule of hj_pair_fast
  if constexpr (R == 8) {
    sqrt8(t, q);
  } else {
#pragma unroll
    for (int e = 0; e < R; ++e) t[e] = hw_sqrt(q[e]);
  }
  __builtin_amdgcn_s_setprio(0);
  const float pr = prod_tree<R>(q);
#pragma unroll
  for (int e = 0; e < R; ++e) q[e] = asinh2_small(x[e], q[e]);
#pragma unroll
  for (int e = 0; e < R; ++e) t[e] = fabsf(x[e]) + t[e];
  __builtin_amdgcn_s_setprio(3);
  if constexpr (R == 8) {
    log2_8_inplace(t);
  } else {
#pragma unroll
    for (int e = 0; e < R; ++e) t[e] = hw_log2(t[e]);
  }
  __builtin_amdgcn_s_setprio(0);
  if (LADJ) acc = fmaf(-0.5f, hw_log2(pr), acc);
#pragma unroll
  for (int e = 0; e < R; ++e) x[e] = asinh2_pick(q[e], t[e], msel[e]);
  return pr;
}

// VAR (diagnostics build only): bit 1 = the Johnson part slab by slab (hj_johnson_slab); bit 2 = no
// per-pair record reads (every pair uses the records loaded before the pair loop: WRONG results, a
// timing probe of the LDS record traffic).
template <int D, int R, int U, bool LADJ, int AS = 1, int VAR = 0>
__device__ __forceinline__ float hj_pair_fast(float (&x)[U][R], float (&acc)[U], const float*& r, HJParams<R>& prm,
                                              uint32_t csign) {
  constexpr bool RL = !(VAR & 2);
  // VAR bit 128 (diagnostics A/B): priority 2 through the reflection (dot, DPP reduction, z), 3 for the
  // transcendental groups, 0 for the rest
  if constexpr ((VAR & 128) != 0) __builtin_amdgcn_s_setprio(2);
  hj_pair_z<D, R, U, RL>(x, r, prm);
  if constexpr ((VAR & 1) && AS == 1) {
    float pr1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) pr1[u] = hj_johnson_slab<R, LADJ>(x[u], acc[u], csign);
    r += kHjW * D;
    if constexpr (RL) prm.template load<0, HJ_IL>(r);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < R; ++e) x[u][e] = fmaf(x[u][e], prm.m(HJ_DP, e), prm.m(HJ_GP, e));
    float m1 = pr1[0];
#pragma unroll
    for (int u = 1; u < U; ++u) m1 = fmaxf(m1, pr1[u]);
    return m1;
  }
  // stage by stage over the whole tile (U*R independent chains per stage)
  float q[U][R], t[U][R], pr[U];
  uint32_t msel[U][R];  // AS == 1: the select mask of asinh2_pick, from q (before the transcendentals)
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) q[u][e] = fmaf(x[u][e], x[u][e], AS == 2 ? (float)kAsinhK : 1.0f);
  if constexpr (AS == 1) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < R; ++e) msel[u][e] = asinh2_mask(q[u][e], csign);
  }
  // Wave priority 3 while a wave issues its sqrt / log2 group, 0 otherwise (round 3, last session): the SIMD's
  // arbiter then issues the transcendentals of the waves in that phase first and fills the transcendental
  // pipe's busy cycles with the other waves' FMAs, instead of picking by age. 0.682 / 0.683 / 0.686 vs
  // 0.725 / 0.721 / 0.723 ms streaming, 0.532 / 0.548 / 0.553 vs 0.614 / 0.609 / 0.597 ms compute-only
  // (profiles/r03_setprio_ab.jsonl). VAR bit 4 (diagnostics A/B): the previous schedule without it; bit 8:
  // the priorities the other way round (slower).
  // (bits 16 / 32: only around the sqrt / only around the log2 group; 64: also around the ladj's log2)
  constexpr bool PRIO = (VAR & 4) == 0 && (VAR & 8) == 0;
  constexpr bool PS = PRIO && (VAR & 32) == 0, PL = PRIO && (VAR & 16) == 0;
  if constexpr ((VAR & 128) != 0) __builtin_amdgcn_s_setprio(0);
  if constexpr (PS) __builtin_amdgcn_s_setprio(3);
  if constexpr ((VAR & 8) != 0) __builtin_amdgcn_s_setprio(0);
  if constexpr (R == 8) {
#pragma unroll
    for (int u = 0; u < U; ++u) sqrt8(t[u], q[u]);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < R; ++e) t[u][e] = hw_sqrt(q[u][e]);
  }
  if constexpr (PS) __builtin_amdgcn_s_setprio(0);
  if constexpr ((VAR & 8) != 0) __builtin_amdgcn_s_setprio(2);
#pragma unroll
  for (int u = 0; u < U; ++u) pr[u] = prod_tree<R>(q[u]);
  if constexpr (AS > 0) {  // small |z|: the Taylor form (enf_frag.h) in place of q
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < R; ++e)
        q[u][e] = AS == 2 ? asinh2_small_k(x[u][e], q[u][e]) : asinh2_small(x[u][e], q[u][e]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) t[u][e] = fabsf(x[u][e]) + t[u][e];
  if constexpr (PL) __builtin_amdgcn_s_setprio(3);
  if constexpr ((VAR & 8) != 0) __builtin_amdgcn_s_setprio(0);
  if constexpr (R == 8) {
#pragma unroll
    for (int u = 0; u < U; ++u) log2_8_inplace(t[u]);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < R; ++e) t[u][e] = hw_log2(t[u][e]);
  }
  if constexpr (PL && (VAR & 64) == 0) __builtin_amdgcn_s_setprio(0);
  if constexpr ((VAR & 8) != 0) __builtin_amdgcn_s_setprio(2);
  if (LADJ)
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = fmaf(-0.5f, hw_log2(pr[u]), acc[u]);
  if constexpr (PL && (VAR & 64) != 0) __builtin_amdgcn_s_setprio(0);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) {
      if constexpr (AS == 2)
        x[u][e] = asinh2_med3(q[u][e], t[u][e]);
      else if constexpr (AS == 1)
        x[u][e] = asinh2_pick(q[u][e], t[u][e], msel[u][e]);
      else if constexpr (AS == 3)
        x[u][e] = asinh2_merge(x[u][e], q[u][e], t[u][e], csign);
      else
        x[u][e] = copysignf(t[u][e], x[u][e]);
    }
  r += kHjW * D;
  if constexpr (RL) prm.template load<0, HJ_IL>(r);
  // y_p = gamma_p + delta'_p L_p: the next record's {delta', gamma} slots (record n: the output's)
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) x[u][e] = fmaf(x[u][e], prm.m(HJ_DP, e), prm.m(HJ_GP, e));
  float m = pr[0];
#pragma unroll
  for (int u = 1; u < U; ++u) m = fmaxf(m, pr[u]);
  return m;
}

// The same pair in the exact-range elementwise form (johnson_fwd_f32_slow): asinh finite up to
// FLT_MAX, ladj -Inf where the reference's fp32 1 + z^2 overflows.
// (AS == 2: the records give sqrt(K) z; z is unscaled here, and the ladj carries the fast form's
// -log2(K)/2 per element that the column constant cancels.)
template <int D, int R, int U, bool LADJ, int AS>
__device__ __forceinline__ void hj_pair_exact(float (&x)[U][R], float (&acc)[U], const float*& r, HJParams<R>& prm) {
  hj_pair_z<D, R, U>(x, r, prm);
  constexpr float halflog2k = 3.4396521971792485e-07f;  // log2(K)/2
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) {
      const YL yl = johnson_fwd_f32_slow(AS == 2 ? x[u][e] * (float)kAsinhRSqrtK : x[u][e], 0.f, 1.f);
      x[u][e] = yl.y;
      if (LADJ) acc[u] += AS == 2 ? yl.l - halflog2k : yl.l;
    }
  r += kHjW * D;
  prm.template load<0, HJ_IL>(r);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) x[u][e] = fmaf(x[u][e], prm.m(HJ_DP, e), prm.m(HJ_GP, e));
}

template <int D, int R, int U, int LM, int AS = 1, int VAR = 0, bool PAD = false>
struct HJBody {
  const HJArgs& a;
  const float* rec;  // this lane's record group
  float ctot;
  float* stage;
  int n;

  template <bool TAIL, int DBG>
  __device__ __forceinline__ void tile(int64_t col0, float (&x)[U][R], const float (&old)[HJLay<D, R, U>::NLS]) {
    constexpr bool LADJ = LM > 0;
    float acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = 0.f;
    const float* r = rec;
    HJParams<R> prm;
    prm.template load<0, HJ_IL>(r);
    if constexpr ((VAR & 2) != 0) prm.template load<HJ_IL, HJ_RR>(r);
    const uint32_t csign = sign_mask_vgpr();
    // branch-free pair loop; a tile with a product overflow (|z| large, Inf, NaN) is redone below
    float m = 0.f;
    for (int p = 0; p < n; ++p) m = fmaxf(m, hj_pair_fast<D, R, U, LADJ, AS, VAR>(x, acc, r, prm, csign));
    // column-uniform: the exact form's dot products read every lane of a column (DPP)
    m = group_max<HJLay<D, R, U>::G>(m);
    if (__builtin_expect(!(m <= FLT_MAX), 0)) {
      hj_load<D, R, U, TAIL, DBG, PAD>(a, col0, x);
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = 0.f;
      r = rec;
      prm.template load<0, HJ_IL>(r);
      for (int p = 0; p < n; ++p) hj_pair_exact<D, R, U, LADJ, AS>(x, acc, r, prm);
    }
    // (y_n = gamma_n + delta'_n L_n was formed at the end of the last pair)
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

template <int D, int R, int U, int LM, int OCC, int DBG, int AS = 1, int VAR = 0, bool PAD = false>
__global__ __launch_bounds__(256, OCC) void flow_hj_kernel(HJArgs a) {
  const int n = a.n;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* scr = reinterpret_cast<double*>(smem);
  float* ctotp = reinterpret_cast<float*>(scr + 2 * kHjMaxPairs);
  float* stage = reinterpret_cast<float*>(smem + kHjScratch) + (threadIdx.x >> 6) * kStagePerWave;
  float* rec = reinterpret_cast<float*>(smem + kHjHeader);
  build_hj_program<D, R, AS>(a, n, rec, scr, ctotp);
  constexpr int G = HJLay<D, R, U>::G;
  HJBody<D, R, U, LM, AS, VAR, PAD> body{a, rec + ((threadIdx.x & 63) % G) * kHjW * R, *ctotp, stage, n};
  hj_stream<D, R, U, LM, DBG, PAD>(a, body);
}

// ---------------------------------------------------------------------------------------------------
// The inverse program (round 4): inverse(J_n o H_n o ... o J_1 o H_1) = H_1 o J_1^-1 o ... o H_n o J_n^-1
// (src/johnson_trafo.jl:82 inverse(JohnsonTrafo) = JohnsonTrafoInv, src/householder_trafo.jl:153-154 a single
// reflection is its own inverse), i.e. the layers J^-1, H, J^-1, H, ... applied in this order, fp32, the
// layouts of the forward program (D = 32 / 64 / 128, padded or not), fused in one launch. Per pair p:
//   w   = (y - gamma)/delta                  as fma(y, 1/delta, -gamma/delta)       (johnson_trafo.jl:36)
//   sh  = sinh(w): |w| < 1/2: w (1 + w^2/6 + w^4/120 + w^6/5040) (truncation < 1e-8 relative),
//         else (E - 1/E)/2, E = exp2(w log2 e) -- both odd in w, merged branch-free by a mask from w^2
//   x   = lambda sh + xi                      the JohnsonTrafoInv output              (johnson_trafo.jl:36)
//   ladj += -log|delta/lambda| + log(1 + sh^2)/2: the reference's -johnsontrafo_ladj of the output
//         (johnson_trafo.jl:103-104), whose (x - xi)/lambda is sh up to the rounding of x; the constant part
//         once per column (ctot), +1/2 log2 of the product of the q = 1 + sh^2 of a lane's 8 rows
//   dot = vh'x, x -= dot vh                   householder_trafo! (householder_trafo.jl:8-11)
// Records per pair and row {1/delta, -gamma/delta, lambda, xi, vh} (built in double); the multipliers of tile
// registers one slot rotated (hj_rot). A tile whose q product overflows (|sh| ~ 2^16 on every row, Inf, NaN)
// is redone from X elementwise (exact-range sinh, log2 per element: ladj +Inf where the reference's fp32
// 1 + z^2 overflows).
constexpr int kHjiW = 5;
enum : int { HI_ID = 0, HI_NG = 1, HI_LM = 2, HI_XI = 3, HI_VH = 4 };
__host__ __device__ constexpr bool hi_rotated(int q) { return q == HI_ID || q == HI_LM || q == HI_VH; }
static size_t hji_lds_bytes(int D, int n) { return kHjHeader + (size_t)n * kHjiW * D * sizeof(float); }

template <int R>
struct HJIParams {
  float v[kHjiW][R];
  __device__ __forceinline__ void load(const float* r) {
#pragma unroll
    for (int k = 0; k < kHjiW; ++k)
#pragma unroll
      for (int h = 0; h < R / 4; ++h) lds_vec<float, 4>(r + k * R + 4 * h, *reinterpret_cast<float(*)[4]>(&v[k][4 * h]));
  }
  __device__ __forceinline__ float m(int k, int e) const { return v[k][hi_rotated(k) ? hj_rot(e) : e]; }
};

template <int D, int R>
__device__ void build_hji_program(const HJArgs& a, int n, float* __restrict__ rec, double* __restrict__ scr,
                                  float* ctot) {
  constexpr int NF = R / 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int p = wave; p < n; p += nw) {  // v'v and sum_d log|delta/lambda| (johnson_trafo.jl:41) in double
    const float* v = a.v[p];
    double vv = 0.0, cl = 0.0;
    for (int d = lane; d < a.dreal; d += 64) {
      const double vd = v[d];
      vv += vd * vd;
      cl += log(fabs((double)a.d[p][d])) - log(fabs((double)a.lam[p][d]));
    }
    for (int m = 32; m >= 1; m >>= 1) {
      vv += __shfl_xor(vv, m);
      cl += __shfl_xor(cl, m);
    }
    if (lane == 0) {
      scr[2 * p] = sqrt(2.0 / vv);
      scr[2 * p + 1] = cl;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n * D; i += blockDim.x) {
    const int p = i / D, d = i % D;
    const int h = d / (D / NF), w = d % (D / NF), g = w / 4, e = w % 4;
    float* r = rec + (size_t)p * kHjiW * D + g * kHjiW * R + 4 * h;
    // a padded row (d >= dreal): w = 0, sh = 0, x = 0, vh = 0 -- its zeros stay zero with q = 1 (ladj 0)
    double q[kHjiW] = {1.0, 0.0, 1.0, 0.0, 0.0};
    if (d < a.dreal) {
      const double id = 1.0 / (double)a.d[p][d];
      q[HI_ID] = id;
      q[HI_NG] = -(double)a.g[p][d] * id;
      q[HI_LM] = (double)a.lam[p][d];
      q[HI_XI] = (double)a.xi[p][d];
      q[HI_VH] = (double)a.v[p][d] * scr[2 * p];
    }
#pragma unroll
    for (int k = 0; k < kHjiW; ++k) r[k * R + (hi_rotated(k) ? hj_rot(e) : e)] = (float)q[k];
  }
  if (threadIdx.x == 0) {
    double c = 0.0;
    for (int p = 0; p < n; ++p) c -= scr[2 * p + 1];  // -johnsontrafo_ladj: -log|delta/lambda|
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

// One pair (J^-1, H) on the register tile, fast form: returns the largest q product of a lane's rows.
template <int D, int R, int U, bool LADJ>
__device__ __forceinline__ float hji_pair_fast(float (&x)[U][R], float (&acc)[U], const float*& r) {
  HJIParams<R> prm;
  prm.load(r);
  r += kHjiW * D;
  float w[U][R], E[U][R], rE[U][R], pr[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) {
      w[u][e] = fmaf(x[u][e], prm.m(HI_ID, e), prm.m(HI_NG, e));
      E[u][e] = w[u][e] * (float)kLog2e;
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
      const float sh = asinh2_pick(w[u][e], (E[u][e] - rE[u][e]) * 0.5f, msk[u][e]);
      q[u][e] = fmaf(sh, sh, 1.0f);
      x[u][e] = fmaf(prm.m(HI_LM, e), sh, prm.m(HI_XI, e));
    }
    pr[u] = prod_tree<R>(q[u]);
    if (LADJ) acc[u] = fmaf(0.5f, hw_log2(pr[u]), acc[u]);
  }
  float dot[U];
  hj_dots<D, R, U, HI_VH>(x, prm, dot);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) x[u][e] = fmaf(-dot[u], prm.m(HI_VH, e), x[u][e]);
  float m = pr[0];
#pragma unroll
  for (int u = 1; u < U; ++u) m = fmaxf(m, pr[u]);
  return m;
}

// The same pair elementwise over the whole fp32 range: sinh finite up to |w| ~ 89.4 (E/2 formed as
// exp2(|w| log2 e - 1)), the ladj's log2 per element (+Inf where 1 + sh^2 overflows, as the reference's).
template <int D, int R, int U, bool LADJ>
__device__ __forceinline__ void hji_pair_exact(float (&x)[U][R], float (&acc)[U], const float*& r) {
  HJIParams<R> prm;
  prm.load(r);
  r += kHjiW * D;
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) {
      const float w = fmaf(x[u][e], prm.m(HI_ID, e), prm.m(HI_NG, e));
      const float aw = fabsf(w);
      const float h = hw_exp2(fmaf(aw, (float)kLog2e, -1.0f));
      const float big = copysignf(fmaf(-0.25f, hw_rcp(h), h), w);
      const float sh = aw < 0.5f ? sinh_small(w, w * w) : big;
      x[u][e] = fmaf(prm.m(HI_LM, e), sh, prm.m(HI_XI, e));
      if (LADJ) acc[u] += 0.5f * hw_log2(fmaf(sh, sh, 1.0f));
    }
  float dot[U];
  hj_dots<D, R, U, HI_VH>(x, prm, dot);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) x[u][e] = fmaf(-dot[u], prm.m(HI_VH, e), x[u][e]);
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
    constexpr bool LADJ = LM > 0;
    float acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = 0.f;
    const float* r = rec;
    float m = 0.f;
    for (int p = 0; p < n; ++p) m = fmaxf(m, hji_pair_fast<D, R, U, LADJ>(x, acc, r));
    m = group_max<HJLay<D, R, U>::G>(m);
    if (__builtin_expect(!(m <= FLT_MAX), 0)) {
      hj_load<D, R, U, TAIL, DBG, PAD>(a, col0, x);
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = 0.f;
      r = rec;
      for (int p = 0; p < n; ++p) hji_pair_exact<D, R, U, LADJ>(x, acc, r);
    }
    hj_store<D, R, U, LM, TAIL, DBG, PAD>(a, ctot, col0, x, acc, old, stage);
  }
};

template <int D, int R, int U, int LM, bool PAD>
__global__ __launch_bounds__(256, 4) void flow_hji_kernel(HJArgs a) {
  const int n = a.n;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* scr = reinterpret_cast<double*>(smem);
  float* ctotp = reinterpret_cast<float*>(scr + 2 * kHjMaxPairs);
  float* stage = reinterpret_cast<float*>(smem + kHjScratch) + (threadIdx.x >> 6) * kStagePerWave;
  float* rec = reinterpret_cast<float*>(smem + kHjHeader);
  build_hji_program<D, R>(a, n, rec, scr, ctotp);
  constexpr int G = HJLay<D, R, U>::G;
  HJIBody<D, R, U, LM, PAD> body{a, rec + ((threadIdx.x & 63) % G) * kHjiW * R, *ctotp, stage, n};
  hj_stream<D, R, U, LM, 0, PAD>(a, body);
}

#if ENF_DIAG
// ---------------------------------------------------------------------------------------------------
// Wave-specialised form of the same program (round 3): the transcendentals on waves of their own.
//
// On gfx950 a v_sqrt / v_log interleaved with a wave's own FMAs costs ~5.5 ns of SIMD time instead of the
// ~3.7 ns it costs in a run of transcendentals (tools/microbench21: 224 FMAs + 32 transcendentals per wave,
// 416 ns per wave-iteration vs 240 + 118 alone), while transcendentals issued by OTHER waves of the SIMD
// largely overlap a wave's FMA stream (tools/microbench22: two FMA waves + two transcendental waves per SIMD
// 1.27 ms vs 1.67 ms for the same work mixed in every wave). So a block of 16 waves splits each pair:
//  * F waves (0-7, two per SIMD) own the tiles: dot, reflection and z of pair p; later the small-|z| form,
//    the merge and y = gamma + delta' L of pair p (the shipped kernel's operations, in its order);
//  * T waves (8-15, two per SIMD; T wave 8 + f serves F wave f) take z through LDS and return
//    t = log2(|z| + sqrt(1 + z^2)); they also keep the ladj (the -1/2 log2 of the q product of a lane's 8
//    rows, one log2 per 8 rows, as before) and store it, and stage the next tiles' X through LDS.
// Every F wave keeps two tiles in flight (slots A and B, one step apart), so that while the T wave works on
// one slot's transcendentals the F wave works on the other slot. Steps are paced by one block barrier; a
// step moves 16 values per lane each way. Identical arithmetic to flow_hj_kernel (AS = 1), so identical
// results; the exact-range redo of a tile whose q product overflows is run by its F wave.
// MEASURED AND REJECTED (diagnostics build only, ENF_HJ_SPEC=1): bit-identical outputs but 0.97 vs 0.78 ms at
// D = 32 and 0.99 vs 0.80 ms at D = 64 (profiles/r03_hjs_spec_ab.jsonl) -- one block barrier per step puts all
// F waves of a SIMD in the same phase, so the LDS round trips and the dot's DPP chain of each step are exposed
// instead of hidden behind the other waves' work; the synthetic form of the same pacing
// (tools/microbench23: 975 ns per step against 888 for the mixed stream) showed the same.
constexpr int kHjSpecDefault = 0;         // product default of ENF_HJ_SPEC (dispatch_hj)
constexpr int kHjsF = 8;                  // F waves per block; T waves kHjsF .. 2 kHjsF - 1
constexpr int kHjsSlot = 64 * 16;         // floats of one slot: 16 values per lane
constexpr size_t kHjsStage = (size_t)2 * kHjsF * kStagePerWave * sizeof(float);
constexpr size_t kHjsFlags = 16 * sizeof(int);  // overflow flag per F wave and slot
constexpr size_t kHjsExch = (size_t)kHjsF * 2 * kHjsSlot * sizeof(float);  // z / t exchange
constexpr size_t kHjsXArea = kHjsExch;                                      // next tiles' X
static size_t hjs_lds_bytes(int D, int n) {
  return kHjScratch + kHjsStage + kHjsFlags + kHjsExch + kHjsXArea + (size_t)(n + 1) * kHjW * D * sizeof(float);
}

// LDS slot of one lane: 16 values in 4 16-byte vectors at a stride of 1 KiB (conflict-free b128 access)
template <int R, int U>
__device__ __forceinline__ void slot_write(float* __restrict__ slot, int lane, const float (&v)[U][R]) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int h = 0; h < R / 4; ++h) {
      u32x4 w;
      __builtin_memcpy(&w, &v[u][4 * h], 16);
      *reinterpret_cast<u32x4*>(slot + (u * (R / 4) + h) * 256 + 4 * lane) = w;
    }
}
template <int R, int U>
__device__ __forceinline__ void slot_read(const float* __restrict__ slot, int lane, float (&v)[U][R]) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int h = 0; h < R / 4; ++h) {
      const u32x4 w = *reinterpret_cast<const u32x4*>(slot + (u * (R / 4) + h) * 256 + 4 * lane);
      __builtin_memcpy(&v[u][4 * h], &w, 16);
    }
}

// F: y of pair p - 1 from the T wave's t (x holds that pair's z on entry), record r = record p
template <int R, int U>
__device__ __forceinline__ void hjs_merge(float (&x)[U][R], const float (&t)[U][R], const HJParams<R>& prm,
                                          uint32_t csign) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) {
      const float q = fmaf(x[u][e], x[u][e], 1.0f);
      const uint32_t m = asinh2_mask(q, csign);
      const float L = asinh2_pick(asinh2_small(x[u][e], q), t[u][e], m);
      x[u][e] = fmaf(L, prm.m(HJ_DP, e), prm.m(HJ_GP, e));
    }
}

// Y of a finished tile (F wave); the ladj is the T wave's
template <int D, int R, int U>
__device__ __forceinline__ void hjs_store_y(const HJArgs& a, int64_t col0, const float (&x)[U][R]) {
  using L = HJLay<D, R, U>;
  const int lane = threadIdx.x & 63;
  float* __restrict__ Y = (float*)a.Y;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t c = L::col(col0, u, lane);
#pragma unroll
    for (int h = 0; h < L::NF; ++h) {
      u32x4 v4;
      __builtin_memcpy(&v4, &x[u][4 * h], 16);
      if (ENF_INB(c < a.N, "hjs store Y", c, a.N))
        __builtin_nontemporal_store(v4, reinterpret_cast<u32x4*>(Y + c * D + L::row(h, lane)));
    }
  }
}

template <int D, int LM>
__global__ __launch_bounds__(1024, 1) void flow_hjs_kernel(HJArgs a) {
  constexpr int R = 8, U = 2;
  using L = HJLay<D, R, U>;
  constexpr int G = L::G;
  const int n = a.n;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* scr = reinterpret_cast<double*>(smem);
  float* ctotp = reinterpret_cast<float*>(scr + 2 * kHjMaxPairs);
  unsigned char* p0 = smem + kHjScratch;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  float* stage = reinterpret_cast<float*>(p0) + wave * kStagePerWave;
  int* flags = reinterpret_cast<int*>(p0 + kHjsStage);
  float* exch = reinterpret_cast<float*>(p0 + kHjsStage + kHjsFlags);
  float* xarea = exch + kHjsF * 2 * kHjsSlot;
  float* rec = xarea + kHjsF * 2 * kHjsSlot;
  const bool isF = wave < kHjsF;
  const int f = isF ? wave : wave - kHjsF;
  float* ex[2] = {exch + (2 * f) * kHjsSlot, exch + (2 * f + 1) * kHjsSlot};
  float* xa[2] = {xarea + (2 * f) * kHjsSlot, xarea + (2 * f + 1) * kHjsSlot};

  constexpr int64_t CT = L::TC;
  const int64_t ntiles = a.N / CT;
  const int64_t stride = (int64_t)gridDim.x * kHjsF;
  const int64_t g = (int64_t)blockIdx.x * kHjsF + f;  // this F wave's (or its partner's) tile stream
  const int64_t K = g < ntiles ? (ntiles - 1 - g) / stride + 1 : 0;
  const int64_t g0 = (int64_t)blockIdx.x * kHjsF;
  const int64_t Kmax = g0 < ntiles ? (ntiles - 1 - g0) / stride + 1 : 0;
  auto tile_col = [&](int64_t k) { return (g + k * stride) * CT; };

  // T waves: the first tile of each slot, loaded before the prologue
  float xt[2][U][R];
  if (!isF) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (s < K) hj_load<D, R, U, false, 0>(a, tile_col(s), xt[s]);
  }
  build_hj_program<D, R, 1>(a, n, rec, scr, ctotp);  // ends with a block barrier
  const float ctot = *ctotp;
  const float* recl = rec + (lane % G) * kHjW * R;
  if (!isF) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (s < K) slot_write<R, U>(xa[s], lane, xt[s]);
    if (lane < 2) flags[2 * f + lane] = 0;
  }
  __syncthreads();

  // steps: slot A (X = 0) holds tiles 0, 2, 4, ... of the stream and gets F steps 0, 2, 4, ...; slot B tiles
  // 1, 3, ... and steps 1, 3, ...; a tile takes n F steps (pair p's z phase, merged with pair p - 1's y),
  // its last y comes with the first step of the slot's next tile. T processes at step s the slot F touched
  // at step s - 1.
  const int64_t nA = (Kmax + 1) / 2, nB = Kmax / 2;
  const int64_t S = Kmax == 0 ? 0 : ((2 * n * nA > 2 * n * nB + 1) ? 2 * n * nA : 2 * n * nB + 1) + 1;
  const uint32_t csign = sign_mask_vgpr();
  float x[2][U][R];        // F: the two slots' tiles (z after a z phase, y after a merge)
  float acc[2][U] = {};    // T: ladj partials of the two slots' tiles
  float mx[2] = {0.f, 0.f};  // T: largest q product of the slot's tile
  HJParams<R> prm;

  auto f_step = [&](auto XC, int64_t s) {
    constexpr int X = decltype(XC)::value;
    if (s < X) return;
    const int64_t q = (s - X) >> 1;
    const int64_t j = q / n;
    const int p = (int)(q - j * n);
    const int64_t k = 2 * j + X;
    if (p == 0 && j > 0 && k - 2 < K) {
      // the slot's previous tile: its last y (record n), or the exact-range redo from X
      const int64_t c0 = tile_col(k - 2);
      if (flags[2 * f + X] == 0) {
        float t[U][R];
        slot_read<R, U>(ex[X], lane, t);
        prm.template load<0, HJ_IL>(recl + n * kHjW * D);
        hjs_merge<R, U>(x[X], t, prm, csign);
        hjs_store_y<D, R, U>(a, c0, x[X]);
      } else {
        float old[L::NLS];
        hj_load<D, R, U, false, 0>(a, c0, x[X]);
        hj_load_old<D, R, U, LM>(a, c0, old, false);
        float accx[U];
#pragma unroll
        for (int u = 0; u < U; ++u) accx[u] = 0.f;
        const float* r = recl;
        HJParams<R> pe;
        pe.template load<0, HJ_IL>(r);
        for (int pp = 0; pp < n; ++pp) hj_pair_exact<D, R, U, LM != 0, 1>(x[X], accx, r, pe);
        hj_store<D, R, U, LM, false, 0>(a, ctot, c0, x[X], accx, old, stage);
      }
    }
    if (k >= K) return;
    const float* rp = recl + p * kHjW * D;
    prm.template load<0, HJ_IL>(rp);
    if (p == 0) {
      slot_read<R, U>(xa[X], lane, x[X]);
    } else {
      float t[U][R];
      slot_read<R, U>(ex[X], lane, t);
      hjs_merge<R, U>(x[X], t, prm, csign);
    }
    hj_pair_z<D, R, U>(x[X], rp, prm);
    slot_write<R, U>(ex[X], lane, x[X]);
  };

  auto t_step = [&](auto YC, int64_t s) {
    constexpr int Y = decltype(YC)::value;
    if (s < Y + 1) return;
    const int64_t q = (s - 1 - Y) >> 1;
    const int64_t j = q / n;
    const int p = (int)(q - j * n);
    const int64_t k = 2 * j + Y;
    if (k >= K) return;
    if (p == 0 && k + 2 < K) hj_load<D, R, U, false, 0>(a, tile_col(k + 2), xt[Y]);  // the slot's next tile
    float z[U][R], t[U][R];
    slot_read<R, U>(ex[Y], lane, z);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float qv[R];
#pragma unroll
      for (int e = 0; e < R; ++e) qv[e] = fmaf(z[u][e], z[u][e], 1.0f);
      sqrt8(t[u], qv);
      const float pr = prod_tree<R>(qv);
#pragma unroll
      for (int e = 0; e < R; ++e) t[u][e] = fabsf(z[u][e]) + t[u][e];
      log2_8_inplace(t[u]);
      if (LM > 0) acc[Y][u] = fmaf(-0.5f, hw_log2(pr), acc[Y][u]);
      mx[Y] = fmaxf(mx[Y], pr);
    }
    slot_write<R, U>(ex[Y], lane, t);
    if (p == n - 1) {
      // tile done: the F wave redoes it in the exact form when some q product overflowed (+Inf / NaN)
      const bool ovf = __any(!(mx[Y] <= FLT_MAX));
      if (lane == 0) flags[2 * f + Y] = ovf ? 1 : 0;
      if (LM > 0 && !ovf) {
        const int64_t c0 = tile_col(k);
        float old[L::NLS];
        hj_load_old<D, R, U, LM>(a, c0, old, false);
        float* __restrict__ ladj = (float*)a.ladj;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const float tot = group_sum<G>(acc[Y][u]);
          if ((lane % G) == 0) stage[u * L::CPS + lane / G] = tot;
        }
#pragma unroll
        for (int kk = 0; kk < L::NLS; ++kk) {
          const int c = kk * 64 + (L::TC >= 64 ? lane : lane % L::TC);
          const float v = fmaf((float)kLn2, stage[c], ctot) + old[kk];
          if (ENF_INB(c0 + c < a.N, "hjs ladj", c0 + c, a.N)) ladj[c0 + c] = v;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc[Y][u] = 0.f;
      mx[Y] = 0.f;
      if (k + 2 < K) slot_write<R, U>(xa[Y], lane, xt[Y]);  // waits for the load issued at p == 0
    }
  };

  // one loop per role (wave-uniform branch; both execute the same S barriers), so that neither keeps the
  // other's registers live
  if (isF) {
    for (int64_t s = 0; s < S; s += 2) {
      f_step(std::integral_constant<int, 0>{}, s);
      __syncthreads();
      if (s + 1 < S) {
        f_step(std::integral_constant<int, 1>{}, s + 1);
        __syncthreads();
      }
    }
  } else {
    for (int64_t s = 0; s < S; s += 2) {
      t_step(std::integral_constant<int, 1>{}, s);
      __syncthreads();
      if (s + 1 < S) {
        t_step(std::integral_constant<int, 0>{}, s + 1);
        __syncthreads();
      }
    }
  }
  // the ragged last tile: one F wave, whole program in its own registers (flow_hj_kernel's tail path)
  if (isF && ntiles * CT < a.N && g == ntiles % stride) {
    HJBody<D, R, U, LM, 1, 0> body{a, recl, ctot, stage, n};
    const int64_t c0 = ntiles * CT;
    float xt0[U][R], old[L::NLS];
    hj_load<D, R, U, true, 0>(a, c0, xt0);
    hj_load_old<D, R, U, LM>(a, c0, old, true);
    body.template tile<true, 0>(c0, xt0, old);
  }
}
#endif  // ENF_DIAG

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


#if ENF_DIAG
// one block of 16 waves per CU
template <int D, int LM>
static hipError_t launch_hjs(const HJArgs& h, hipStream_t st, const DeviceInfo& dev) {
  const size_t lds = hjs_lds_bytes(D, h.n);
  const void* k = reinterpret_cast<const void*>(&flow_hjs_kernel<D, LM>);
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  int64_t blocks = dev.num_cu;
  const int64_t need = (h.N + (int64_t)HJLay<D, 8, 2>::TC * kHjsF - 1) / ((int64_t)HJLay<D, 8, 2>::TC * kHjsF);
  if (blocks > need) blocks = need > 0 ? need : 1;
  hipLaunchKernelGGL((flow_hjs_kernel<D, LM>), dim3((unsigned)blocks), dim3(1024), lds, st, h);
  return hipGetLastError();
}
#endif

template <int D, int R, int U, int LM, int OCC = 1, int DBG = 0, int AS = 1, int VAR = 0, bool PAD = false>
static hipError_t launch_hj(const HJArgs& h, hipStream_t st, const DeviceInfo& dev) {
  const size_t lds = hj_lds_bytes(D, h.n);
  const void* k = reinterpret_cast<const void*>(&flow_hj_kernel<D, R, U, LM, OCC, DBG, AS, VAR, PAD>);
  int64_t blocks = 0;
  hipError_t e = frag_grid(k, h.N, (int64_t)HJLay<D, R, U>::TC * 4, lds, dev, &blocks);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((flow_hj_kernel<D, R, U, LM, OCC, DBG, AS, VAR, PAD>), dim3((unsigned)blocks), dim3(256), lds, st, h);
  return hipGetLastError();
}

// R = 8 rows per lane, U = 2 slabs (16 values per lane). Diagnostics build only (ENF_DIAG):
// ENF_DEBUG_MODE 1/2 (synthesized tile / no stores), ENF_HJ_ASINH = 0/2 (round 1's asinh form / the
// one-med3 clamp asinh2_med3 in place of the four-op merge: 9% faster, rejected for its coherent bias,
// DESIGN.md §3).
template <int DBG, int LM>
static hipError_t launch_hj_as(int as, const HJArgs& a, hipStream_t st, const DeviceInfo& dev) {
  if (as == 0) return launch_hj<32, 8, 2, LM, 4, DBG, 0>(a, st, dev);
  if (as == 2) return launch_hj<32, 8, 2, LM, 4, DBG, 2>(a, st, dev);
  if (as == 3) return launch_hj<32, 8, 2, LM, 4, DBG, 3>(a, st, dev);
  return launch_hj<32, 8, 2, LM, 4, DBG, 1>(a, st, dev);
}
template <int LM>
static hipError_t dispatch_hj(const HJArgs& a, int D, int dbg, hipStream_t st, const DeviceInfo& dev) {
  (void)dbg;
  // padded layout (round 3): D = 24 / 100 / 36 ... on the next power of two, rows past a.dreal inert
  if (a.dreal != D) {
    if (D == 32) return launch_hj<32, 8, 2, LM, 4, 0, 1, 0, true>(a, st, dev);
    if (D == 64) return launch_hj<64, 8, 2, LM, 4, 0, 1, 0, true>(a, st, dev);
    return launch_hj<128, 8, 2, LM, 4, 0, 1, 0, true>(a, st, dev);
  }
  if (D == 128) return launch_hj<128, 8, 2, LM, 4>(a, st, dev);
  // ENF_HJ_SPEC (diagnostics build): 1 = the wave-specialised kernel (flow_hjs_kernel, rejected), 0 = flow_hj_kernel
#if ENF_DIAG
  static const int spec = ENF_KNOB("ENF_HJ_SPEC", kHjSpecDefault);
  if (spec && dbg == 0) return D == 32 ? launch_hjs<32, LM>(a, st, dev) : launch_hjs<64, LM>(a, st, dev);
#endif
  if (D == 32) {
#if ENF_DIAG
    if constexpr (LM == 1) {
      static const int as = ENF_KNOB("ENF_HJ_ASINH", 1);
      // ENF_HJ_VAR: 1 = Johnson part slab by slab at occupancy 5, 3 = the same without per-pair record
      // reads, 2 = no per-pair record reads (timing probes; 2 and 3 give wrong results)
      static const int var = ENF_KNOB("ENF_HJ_VAR", 0);
      if (dbg == 0 && var == 1) return launch_hj<32, 8, 2, 1, 5, 0, 1, 1>(a, st, dev);
      if (dbg == 0 && var == 2) return launch_hj<32, 8, 2, 1, 4, 0, 1, 2>(a, st, dev);
      if (dbg == 0 && var == 3) return launch_hj<32, 8, 2, 1, 5, 0, 1, 3>(a, st, dev);
      // 4: without the s_setprio around the transcendental groups (the schedule before), 8: priorities reversed
      if (dbg == 0 && var == 4) return launch_hj<32, 8, 2, 1, 4, 0, 1, 4>(a, st, dev);
      if (dbg == 0 && var == 8) return launch_hj<32, 8, 2, 1, 4, 0, 1, 8>(a, st, dev);
      if (dbg == 0 && var == 16) return launch_hj<32, 8, 2, 1, 4, 0, 1, 16>(a, st, dev);
      if (dbg == 0 && var == 32) return launch_hj<32, 8, 2, 1, 4, 0, 1, 32>(a, st, dev);
      if (dbg == 0 && var == 64) return launch_hj<32, 8, 2, 1, 4, 0, 1, 64>(a, st, dev);
      if (dbg == 0 && var == 128) return launch_hj<32, 8, 2, 1, 4, 0, 1, 128>(a, st, dev);
      if (dbg == 0 && var == 192) return launch_hj<32, 8, 2, 1, 4, 0, 1, 192>(a, st, dev);
      if (dbg == 2 && var == 4) return launch_hj<32, 8, 2, 1, 4, 2, 1, 4>(a, st, dev);
      if (dbg == 2 && var == 8) return launch_hj<32, 8, 2, 1, 4, 2, 1, 8>(a, st, dev);
      if (dbg == 2 && var == 1) return launch_hj<32, 8, 2, 1, 5, 2, 1, 1>(a, st, dev);
      if (dbg == 1) return launch_hj_as<1, 1>(as, a, st, dev);
      if (dbg == 2) return launch_hj_as<2, 1>(as, a, st, dev);
      if (dbg == 8) return launch_hj_as<8, 1>(as, a, st, dev);
      if (dbg == 9) return launch_hj_as<9, 1>(as, a, st, dev);
      return launch_hj_as<0, 1>(as, a, st, dev);
    }
#endif
    return launch_hj<32, 8, 2, LM, 4>(a, st, dev);
  }
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
  const size_t lds = hji_lds_bytes(D, h.n);
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
