// enf_frag.h -- device building blocks shared by the fused flow kernels (enf_flow.hip: step-table
// interpreter; enf_flow_hj.hip: compiled (Householder o Johnson)^n program): hardware math, DPP group
// sums, the 16-byte fragment layout of a column-major D x N batch, tile loads/stores and the
// software-pipelined persistent tile loop.
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <type_traits>

#include "enf_internal.h"

namespace enf {

// ------------------------------------------------------------------------------------------
// device math
// ------------------------------------------------------------------------------------------
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr double kLn2 = 0.69314718055994530942;
constexpr double kLog2e = 1.44269504088896340736;

__device__ __forceinline__ float hw_log2(float x) { return __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float hw_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float hw_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float hw_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// Eight independent transcendentals issued back to back (one inline-asm block the scheduler cannot
// interleave). On gfx950 a v_sqrt/v_log costs ~3.4 ns of SIMD issue when transcendentals come in runs
// and ~5 ns when the compiler spreads them between dependent full-rate instructions (pair loop of the
// compiled (J o H)^n program replayed register-only: tools/replay_loop.py, profiles/r02_*). The
// trailing s_nop 0 is the one wait state a VALU reading a transcendental's result needs on gfx950,
// which the compiler's hazard recognizer cannot see inside asm.
#define ENF_TRANS8(OP, o, i)                                                                          \
  asm(OP " %0, %8\n" OP " %1, %9\n" OP " %2, %10\n" OP " %3, %11\n" OP " %4, %12\n" OP " %5, %13\n" OP \
      " %6, %14\n" OP " %7, %15\ns_nop 0"                                                             \
      : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]), "=&v"(o[7]) \
      : "v"(i[0]), "v"(i[1]), "v"(i[2]), "v"(i[3]), "v"(i[4]), "v"(i[5]), "v"(i[6]), "v"(i[7]))
__device__ __forceinline__ void sqrt8(float (&o)[8], const float (&i)[8]) { ENF_TRANS8("v_sqrt_f32", o, i); }
__device__ __forceinline__ void exp2_8(float (&o)[8], const float (&i)[8]) { ENF_TRANS8("v_exp_f32", o, i); }
__device__ __forceinline__ void rcp8(float (&o)[8], const float (&i)[8]) { ENF_TRANS8("v_rcp_f32", o, i); }
__device__ __forceinline__ void log2_8_inplace(float (&x)[8]) {
  asm("v_log_f32 %0, %0\nv_log_f32 %1, %1\nv_log_f32 %2, %2\nv_log_f32 %3, %3\nv_log_f32 %4, %4\n"
      "v_log_f32 %5, %5\nv_log_f32 %6, %6\nv_log_f32 %7, %7\ns_nop 0"
      : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
}

// DPP cross-lane sum over aligned groups of G lanes (G <= 64, power of two). All 64 lanes must
// be active. quad_perm(1,0,3,2) = 0xB1, quad_perm(2,3,0,1) = 0x4E, row_half_mirror = 0x141,
// row_mirror = 0x140: after the quad steps every lane of a quad holds the quad sum, so a
// mirror partner always lies in the other quad / half-row.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL,
                                                               0xF, 0xF, false));
}
// (mov_dpp with bound_ctrl: every lane of these patterns reads a lane of its own row, so no `old` value is
// needed and none is materialised -- update_dpp(0, ...) cost two v_mov of zero per stage; round 4)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int CTRL, typename T>
__device__ __forceinline__ T dpp(T x) {
  if constexpr (std::is_same_v<T, float>) return dpp_f<CTRL>(x);
  else return dpp_d<CTRL>(x);
}
template <int G, typename T>
__device__ __forceinline__ T group_sum(T x) {
  if constexpr (G >= 2) x += dpp<0xB1>(x);
  if constexpr (G >= 4) x += dpp<0x4E>(x);
  if constexpr (G >= 8) x += dpp<0x141>(x);
  if constexpr (G >= 16) x += dpp<0x140>(x);
  if constexpr (G >= 32) x += __shfl_xor(x, 16);
  if constexpr (G >= 64) x += __shfl_xor(x, 32);
  return x;
}

// DPP max over aligned groups of G lanes (as group_sum)
template <int G>
__device__ __forceinline__ float group_max(float x) {
  if constexpr (G >= 2) x = fmaxf(x, dpp<0xB1>(x));
  if constexpr (G >= 4) x = fmaxf(x, dpp<0x4E>(x));
  if constexpr (G >= 8) x = fmaxf(x, dpp<0x141>(x));
  if constexpr (G >= 16) x = fmaxf(x, dpp<0x140>(x));
  if constexpr (G >= 32) x = fmaxf(x, __shfl_xor(x, 16));
  if constexpr (G >= 64) x = fmaxf(x, __shfl_xor(x, 32));
  return x;
}

// ------------------------------------------------------------------------------------------
// per-element transforms. acc is the running per-lane ladj partial of one column, in units of
// log2 (fp32) or natural log (fp64): ladj = C_total + UNIT * acc.
// ------------------------------------------------------------------------------------------
template <typename T>
struct Unit;
template <>
struct Unit<float> { static constexpr float v = (float)kLn2; };
template <>
struct Unit<double> { static constexpr double v = 1.0; };

// asinh(z)/ln2 in fp32 with a small relative error everywhere (johnson_trafo.jl:31 computes
// asinh in the data precision; Julia's asinh(::Float32) is accurate to a few ulp). The fast form
// log2(|z| + sqrt(q)), q = 1 + z^2, loses the low bits of |z| when |z| + sqrt(q) rounds near 1:
// relative error ~1.5e-7/|z| (1e-4 at |z| ~ 2^-12, where the rounding of q drops the z^2/2 term
// that cancels log's -t^2/2). Below kAsinhSmall the Taylor series to z^5 written in q replaces it:
//   asinh z = z (1 - u/6 + 3u^2/40),  u = q - 1,  i.e. z (A0 + A1 q + A2 q^2)
// (max relative error 2.4e-7 on |z| < 1/8; the log form is within 1e-6 on |z| >= 1/8; a tile of
// z ~ N(0,1) values: tools/asinh32_err.py). Signed zeros pass through z * p.
constexpr float kAsinhSmall = 0.125f;
constexpr double kAsinhA2 = 3.0 / 40.0, kAsinhA1 = -1.0 / 6.0 - 2.0 * kAsinhA2, kAsinhA0 = 1.0 + 1.0 / 6.0 + kAsinhA2;
__device__ __forceinline__ float asinh2_small(float z, float q) {
  return z * fmaf(q, fmaf(q, (float)(kAsinhA2 * kLog2e), (float)(kAsinhA1 * kLog2e)), (float)(kAsinhA0 * kLog2e));
}
// Branch-free merge of the two forms, given t = log2(|z| + sqrt(q)) >= 0 and the small form S:
//   asinh(z)/ln2 = |z| < kAsinhSmall ? S : copysign(t, z)
// in four full-rate VALU instructions on gfx950 and no compare / select / copysign (v_cmp, v_cndmask
// and v_bfi each issue at half rate there; tools/microbench5-9, profiles/r02_microbench_issue_costs.txt):
//   T' = t | (z & 0x80000000)            v_bitop3_b32 0xF8 (sign constant in a VGPR, csign)
//   M  = (t - kAsinhSmallL2) >> 31        v_subrev_f32 (literal) + v_ashrrev_i32: all ones iff |z| < T
//                                         (t is monotone in |z|; log2(T + sqrt(1 + T^2)) = asinh(T)/ln2)
//   L  = M ? S : T'                       v_bitop3_b32 0xE4
// S = z * p with p > 0 for every q carries z's sign. NaN z gives NaN t and NaN S: NaN either way.
// (A plain ?: on values computed only for it was also turned by hipcc 7.2 into an exec-masked branch
// around one element's sqrt/log.)
constexpr float kAsinhSmallL2 = 0.17987053f;  // asinh(1/8)/ln2 (mpmath: 0.1798705244977...)
__device__ __forceinline__ uint32_t sign_mask_vgpr() {
  uint32_t c;
  asm volatile("v_mov_b32 %0, 0x80000000" : "=v"(c));  // a VGPR operand: an SGPR source halves the issue rate
  return c;
}
__device__ __forceinline__ float asinh2_merge(float z, float small, float t, uint32_t csign) {
  const uint32_t ts = __builtin_amdgcn_bitop3_b32(__builtin_bit_cast(uint32_t, t), __builtin_bit_cast(uint32_t, z),
                                                 csign, 0xF8);
  const uint32_t m = (uint32_t)(__builtin_bit_cast(int32_t, t - kAsinhSmallL2) >> 31);
  return __builtin_bit_cast(float, __builtin_amdgcn_bitop3_b32(__builtin_bit_cast(uint32_t, small), ts, m, 0xE4));
}
// Mask-first form of the same merge (round 2): the select mask is taken from q, not from t, so it
// issues while the sqrt / log2 of the tile are in flight and ONE instruction follows the log2:
//   M = ((bits(q) - bits(1 + 1/64)) >> 31) | 0x80000000    v_sub_u32 + v_ashrrev_i32 + v_or_b32
//   L = M ? S : t  (bitwise)                                v_bitop3_b32 0xE4
// q >= 1, so the integer difference is negative exactly when q < 1 + 1/64, i.e. |z| < 1/8 (up to the
// rounding of q, where both forms are accurate). M's sign bit is always set, so the sign bit comes
// from S = z * p (p > 0), which is z's sign: the log side needs no separate copysign. NaN q (NaN z)
// leaves M's low bits clear (+NaN) or set (-NaN) and either way returns a NaN.
constexpr uint32_t kAsinhSmallQBits = 0x3F820000u;  // 1 + 1/64 = q at |z| = 1/8
__device__ __forceinline__ uint32_t asinh2_mask(float q, uint32_t csign) {
  const int32_t d = (int32_t)(__builtin_bit_cast(uint32_t, q) - kAsinhSmallQBits);
  return (uint32_t)(d >> 31) | csign;
}
__device__ __forceinline__ float asinh2_pick(float small, float t, uint32_t M) {
  return __builtin_bit_cast(float, __builtin_amdgcn_bitop3_b32(__builtin_bit_cast(uint32_t, small),
                                                               __builtin_bit_cast(uint32_t, t), M, 0xE4));
}
// the full fp32 form given q = fma(z, z, 1) and s = sqrt(q): asinh(z)/ln2
__device__ __forceinline__ float asinh2_f32(float z, float q, float s, uint32_t csign) {
  return asinh2_pick(asinh2_small(z, q), hw_log2(fabsf(z) + s), asinh2_mask(q, csign));
}

// The same two forms merged by one clamp -- a measured and REJECTED alternative, kept in the
// diagnostics build of the compiled (J o H)^n program only (enf_flow_hj.hip AS = 2, ENF_HJ_ASINH=2):
// 0.743 vs 0.818 ms on the headline flow, but the bias b below is coherent (the same sign as z on
// every element that takes the log side), so through four pairs and the reflections' dot products it
// accumulates to up to 2.6x the per-element bound of tests/test_gpu_fp32_accuracy.py (errors ~2e-5 of
// the element's scale, where the merge form stays within it; profiles/r02_asinh_med3_ab.txt).
//   asinh(z)/ln2 = med3(S, -t', t'),  t' = t + b
// The Taylor form S truncated after its positive z^5 term lies above asinh|z| for every z > 0 (odd:
// below for z < 0) and grows like z^5, while the log form t carries an absolute error below ~2.2e-7
// (log2 units; w = |z| + sqrt(q) rounds near 1 for small |z|). With the bias b above that error the
// clamp returns S exactly where S < t' -- the accurate small-|z| side -- and +-t' elsewhere: S is chosen
// for |z| < ~0.17, where its truncation error (~5 z^7/112) is below b. One v_med3_f32 (half rate) in
// place of the merge's four full-rate operations; the price is the bias b on the log side, a relative
// error below 2e-6 near the crossover and below 4e-7 for |z| > 1 (tools/asinh32_err.py, 4M z over
// 1e-30..1e3). The bias costs no instruction: the program carries z' = sqrt(K) z (its records for z
// are scaled), so q' = z'^2 + K = K q, sqrt(q') = sqrt(K) s and log2(|z'| + sqrt(q')) = t + log2(K)/2,
// i.e. b = log2(K)/2 with K = 1 + 2^-21 (b = 3.44e-7); the Taylor coefficients absorb sqrt(K) and K,
// and the ladj's log2 q' = log2 q + log2 K is corrected in the column constant.
constexpr double kAsinhK = 1.0 + 1.0 / 2097152.0;   // 1 + 2^-21, exact in fp32
constexpr double kAsinhSqrtK = 1.0000002384185507;  // sqrt(K)
constexpr double kAsinhRSqrtK = 0.9999997615815062; // 1/sqrt(K)
__device__ __forceinline__ float asinh2_small_k(float zk, float qk) {
  // z (A0 + A1 q + A2 q^2) / ln2 with z = zk / sqrt(K), q = qk / K
  constexpr double rk = kAsinhRSqrtK * kLog2e;
  return zk * fmaf(qk, fmaf(qk, (float)(kAsinhA2 * rk / (kAsinhK * kAsinhK)), (float)(kAsinhA1 * rk / kAsinhK)),
                   (float)(kAsinhA0 * rk));
}
__device__ __forceinline__ float asinh2_med3(float small, float tb) { return __builtin_amdgcn_fmed3f(small, -tb, tb); }

// fp32 robust Johnson element (huge |z|, Inf, NaN): the rare path of the fragment kernel and the
// generic kernel's form. asinh stays finite for |z| up to FLT_MAX; log(1+z^2) overflows to +Inf
// exactly where the reference's fp32 `1 + ((x-xi)/lambda)^2` does (johnson_trafo.jl:41), so
// the ladj is -Inf there, as in the reference.
struct YL { float y, l; };
__device__ __forceinline__ YL johnson_fwd_f32_slow(float z, float g, float d2) {
  const float t = fabsf(z);
  const float q = fmaf(z, z, 1.0f);
  const float L = t > 1e18f ? copysignf(hw_log2(t) + 1.0f, z)  // log2(2|z|) when huge
                            : asinh2_f32(z, q, hw_sqrt(q), sign_mask_vgpr());
  return {fmaf(d2, L, g), -0.5f * hw_log2(q)};  // ladj part in log2 units
}

// ------------------------------------------------------------------------------------------
// the fragment kernel
// ------------------------------------------------------------------------------------------
template <typename T, int D>
struct Frag {
  static constexpr int V = 16 / (int)sizeof(T);        // elements per 16-B fragment
  static constexpr int G = D >= V ? D / V : 1;         // lanes per column
  static constexpr int CPF = D >= V ? 1 : V / D;       // columns per fragment
  static constexpr int SEG = D >= V ? V : D;           // elements of one column in a fragment
  static constexpr int COLS_PER_INSTR = 64 / G * CPF;  // columns per wave-instruction
  static_assert(D >= V ? (D % V == 0 && G <= 64) : (V % D == 0), "unsupported D");
};

// fragment u of this lane holds rows r0 .. r0+SEG-1 of columns colf(u) .. colf(u)+CPF-1
template <typename T, int D>
__device__ __forceinline__ int64_t frag_col(int64_t col0, int u, int lane) {
  using F = Frag<T, D>;
  return col0 + (int64_t)u * F::COLS_PER_INSTR + (lane / F::G) * F::CPF;
}

// One wave tile = U fully coalesced 1-KiB wave-instructions (ldx == D, 16-B aligned).
// DBG (diagnostic builds only, ENF_DEBUG_MODE): 1 = synthesize the tile instead of loading it,
// 2 = also skip the stores (compute-only timing).
// PAD (padded fragment path, frag_pad_dim): D is the power-of-two layout, the columns are a.D < D rows
// apart, and a lane whose rows start at or past a.D holds zeros and stores nothing.
template <typename T, int D, int U, bool TAIL, int DBG = 0, bool PAD = false>
__device__ __forceinline__ void load_tile(const FlowArgs& a, int64_t col0, T (&x)[U][Frag<T, D>::V]) {
  using F = Frag<T, D>;
  constexpr int V = F::V, G = F::G, SEG = F::SEG;
  const int lane = threadIdx.x & 63;
  const int r0 = D >= V ? V * (lane % G) : 0;
  const int64_t ld = PAD ? (int64_t)a.D : (int64_t)D;
  const bool live = !PAD || r0 < a.D;
  const T* __restrict__ X = (const T*)a.X;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t cf = frag_col<T, D>(col0, u, lane);
    const int64_t eoff = cf * ld + r0;
    if (DBG >= 1) {
#pragma unroll
      for (int e = 0; e < V; ++e) x[u][e] = (T)(lane + 3 * u + e) * (T)0.03125 - (T)1;
    } else if (!TAIL) {
      if (live && (!PAD || ENF_INB(eoff + V <= a.N * a.ldx, "frag load X", eoff, a.N * a.ldx))) {
        const u32x4 v4 = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(X + eoff));
        __builtin_memcpy(&x[u][0], &v4, 16);
      } else {
#pragma unroll
        for (int e = 0; e < V; ++e) x[u][e] = (T)0;
      }
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) x[u][e] = (live && (cf + e / SEG) < a.N) ? X[eoff + e] : (T)0;
    }
  }
}

// 16-byte LDS read of V parameter values
template <typename T, int V>
__device__ __forceinline__ void lds_vec(const T* __restrict__ p, T (&v)[V]) {
  static_assert(V * sizeof(T) == 16, "16-byte vectors");
  const u32x4 w = *reinterpret_cast<const u32x4*>(p);
  __builtin_memcpy(&v[0], &w, 16);
}

// Run the step program on one wave tile held in registers (x), then store Y and ladj.
// ladj output of a wave tile. G == 1: a lane owns whole columns (CPF per fragment) and stores
// them as one CPF-vector per fragment. G > 1: column totals are staged through the wave's LDS
// slots and written by NLS = ceil(TC/64) full-wave stores (TC = columns per tile; when TC < 64
// the upper lanes store duplicates of the same values to the same addresses, so no lane mask
// and no branch is needed: the vmcnt accounting of the tile loop stays static).
template <typename T, int D, int U>
struct LadjOut {
  using F = Frag<T, D>;
  static constexpr int TC = F::COLS_PER_INSTR * U;
  static constexpr int NLS = F::G == 1 ? U : (TC + 63) / 64;
  static constexpr int W = F::G == 1 ? F::CPF : 1;  // values per lane per store
  __device__ static __forceinline__ int64_t col(int64_t col0, int k, int lane) {
    if constexpr (F::G == 1) return frag_col<T, D>(col0, k, lane);
    else return col0 + (int64_t)k * 64 + (TC >= 64 ? lane : lane % TC);
  }
};

// LM: 0 no ladj, 1 write ladj, 2 add to ladj (accumulate_ladj)
template <typename T, int D, int U, int LM>
__device__ __forceinline__ void load_ladj_old(const FlowArgs& a, int64_t col0, T (&old)[LadjOut<T, D, U>::NLS][LadjOut<T, D, U>::W]) {
  using LO = LadjOut<T, D, U>;
  const int lane = threadIdx.x & 63;
  const T* __restrict__ ladj = (const T*)a.ladj;
#pragma unroll
  for (int k = 0; k < LO::NLS; ++k)
#pragma unroll
    for (int w = 0; w < LO::W; ++w) old[k][w] = LM == 2 ? ladj[LO::col(col0, k, lane) + w] : (T)0;
}

// register tile types (aliases avoid a clang parse ambiguity of T (&x)[U][Frag<T, D>::V] params)
template <typename T, int D, int U>
using Tile = T[U][Frag<T, D>::V];
template <typename T, int D, int U>
using Acc = T[U][Frag<T, D>::CPF];
#define ENF_FRAG_CONSTS                                   \
  using F = Frag<T, D>;                                   \
  constexpr int V = F::V, G = F::G, CPF = F::CPF, SEG = F::SEG; \
  (void)V; (void)G; (void)CPF; (void)SEG;

// ---- step bodies: one transform applied to the wave tile x (U fragments of V values per lane).
// r points at this lane's record group ([param][element], 16-byte vectors). acc: ladj partials.
// Column dot products of all U*CPF column segments of the tile with the lane's 16-byte vector v,
// reduced over the G lanes of each column. Every stage runs across all segments before the next
// one (U*CPF independent chains), so neither the FMA chain nor the DPP stages stall the wave.
template <typename T, int D, int U>
__device__ __forceinline__ void tile_dots(const Tile<T, D, U>& x, const T (&v)[Frag<T, D>::V],
                                          T (&dot)[U][Frag<T, D>::CPF]) {
  ENF_FRAG_CONSTS
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int c = 0; c < CPF; ++c) dot[u][c] = v[c * SEG] * x[u][c * SEG];
#pragma unroll
  for (int e = 1; e < SEG; ++e)
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < CPF; ++c) dot[u][c] = fma(v[c * SEG + e], x[u][c * SEG + e], dot[u][c]);
  if constexpr (G >= 2) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u][0] += dpp<0xB1>(dot[u][0]);
  }
  if constexpr (G >= 4) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u][0] += dpp<0x4E>(dot[u][0]);
  }
  if constexpr (G >= 8) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u][0] += dpp<0x141>(dot[u][0]);
  }
  if constexpr (G >= 16) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u][0] += dpp<0x140>(dot[u][0]);
  }
  if constexpr (G >= 32) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u][0] += __shfl_xor(dot[u][0], 16);
  }
  if constexpr (G >= 64) {
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u][0] += __shfl_xor(dot[u][0], 32);
  }
}

// ---- tile epilogue: store Y and the ladj
template <typename T, int D, int U, int LM, bool TAIL, int DBG, bool PAD = false>
__device__ __forceinline__ void store_tile(const FlowArgs& a, T ctot, int64_t col0, Tile<T, D, U>& x,
                                           Acc<T, D, U>& acc,
                                           const T (&old)[LadjOut<T, D, U>::NLS][LadjOut<T, D, U>::W],
                                           T* __restrict__ stage) {
  ENF_FRAG_CONSTS
  constexpr bool LADJ = LM > 0;
  const int lane = threadIdx.x & 63;
  T* __restrict__ Y = (T*)a.Y;
  const int64_t N = a.N;
  const int r0 = D >= V ? V * (lane % G) : 0;
  const int64_t ld = PAD ? (int64_t)a.D : (int64_t)D;
  const bool live = !PAD || r0 < a.D;
  int64_t colf[U];
#pragma unroll
  for (int u = 0; u < U; ++u) colf[u] = frag_col<T, D>(col0, u, lane);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t eoff = colf[u] * ld + r0;
    if (DBG == 2) {
      if (x[u][0] == (T)1234.5) Y[eoff] = x[u][1];  // keeps the compute alive, never true in practice
    } else if (!TAIL) {
      if (live && (!PAD || ENF_INB(eoff + V <= a.N * a.ldy, "frag store Y", eoff, a.N * a.ldy))) {
        u32x4 v4;
        __builtin_memcpy(&v4, &x[u][0], 16);
        __builtin_nontemporal_store(v4, reinterpret_cast<u32x4*>(Y + eoff));
      }
    } else if (live) {
#pragma unroll
      for (int e = 0; e < V; ++e)
        if (colf[u] + e / SEG < N) Y[eoff + e] = x[u][e];
    }
  }
  if constexpr (LADJ) {
    using LO = LadjOut<T, D, U>;
    T* __restrict__ ladj = (T*)a.ladj;
    if constexpr (G == 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int c = 0; c < CPF; ++c) {
          const int64_t col = colf[u] + c;
          const T v = fma(Unit<T>::v, acc[u][c], ctot) + old[u][c];
          if (!TAIL) {
            if (!PAD || ENF_INB(col < N, "frag ladj", col, N)) ladj[col] = v;
          } else if (col < N) {
            ladj[col] = v;
          }
        }
      }
    } else {
      // group totals -> the wave's LDS slots (leaders only) -> full-wave coalesced stores
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const T tot = group_sum<G>(acc[u][0]);
        if ((lane % G) == 0) stage[u * F::COLS_PER_INSTR + lane / G] = tot;
      }
#pragma unroll
      for (int k = 0; k < LO::NLS; ++k) {
        const int c = k * 64 + (LO::TC >= 64 ? lane : lane % LO::TC);
        const T v = fma(Unit<T>::v, stage[c], ctot) + old[k][0];
        const int64_t col = col0 + c;
        if (!TAIL) {
          if (!PAD || ENF_INB(col < N, "frag ladj staged", col, N)) ladj[col] = v;
        } else if (col < N) {
          ladj[col] = v;
        }
      }
    }
  }
}

// Persistent, software-pipelined tile loop over the N columns: wave w processes tiles w, w + nwaves,
// ...; the next tile's loads are in flight while this tile computes. Memory operations per iteration
// are branch-free and in a fixed order (old ladj, prefetch, stores): past the last tile the prefetch
// re-reads the current tile instead of being skipped, so the compiler's vmcnt waits only ever cover
// the current tile. The first half-iteration is peeled so that the loop header is reached from the
// entry and from the back edge with the same outstanding memory operations (the previous tile's
// stores behind the current tile's loads). The ragged last tile (N not a multiple of the tile) is
// processed by one wave with masked loads and stores.
// Body::tile<TAIL, DBG>(col0, x, old) runs the flow on one register tile and stores it. pro() -- the
// block prologue, with its barrier -- runs exactly once per wave, after the wave's first tile loads
// are issued, so their HBM latency overlaps it.
template <typename T, int D, int U, int LM, int DBG, bool PAD = false, typename Body, typename Pro>
__device__ __forceinline__ void frag_stream(const FlowArgs& a, Body& body, Pro&& pro) {
  using F = Frag<T, D>;
  using LO = LadjOut<T, D, U>;
  static_assert(F::G == 1 || LO::TC <= kStagePerWave, "ladj staging area too small");
  constexpr int64_t COLS_PER_TILE = (int64_t)F::COLS_PER_INSTR * U;
  const int64_t ntiles_full = a.N / COLS_PER_TILE;
  // wave-uniform tile indices (readfirstlane: scalar registers, uniform branches)
  const int64_t wave_id = (int64_t)blockIdx.x * (blockDim.x >> 6) +
                          __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  using XT = T[U][F::V];
  using OT = T[LO::NLS][LO::W];
  XT xa, xb;
  OT old;
  const int64_t t = wave_id;
  if (t < ntiles_full) {
    load_tile<T, D, U, false, DBG, PAD>(a, t * COLS_PER_TILE, xa);
    int64_t t1 = t + nwaves;
    load_ladj_old<T, D, U, LM>(a, t * COLS_PER_TILE, old);
    load_tile<T, D, U, false, DBG, PAD>(a, (t1 < ntiles_full ? t1 : t) * COLS_PER_TILE, xb);
    pro();
    body.template tile<false, DBG>(t * COLS_PER_TILE, xa, old);
    while (t1 < ntiles_full) {
      const int64_t t2 = t1 + nwaves;
      load_ladj_old<T, D, U, LM>(a, t1 * COLS_PER_TILE, old);
      load_tile<T, D, U, false, DBG, PAD>(a, (t2 < ntiles_full ? t2 : t1) * COLS_PER_TILE, xa);
      body.template tile<false, DBG>(t1 * COLS_PER_TILE, xb, old);
      if (t2 >= ntiles_full) break;
      const int64_t t3 = t2 + nwaves;
      load_ladj_old<T, D, U, LM>(a, t2 * COLS_PER_TILE, old);
      load_tile<T, D, U, false, DBG, PAD>(a, (t3 < ntiles_full ? t3 : t2) * COLS_PER_TILE, xb);
      body.template tile<false, DBG>(t2 * COLS_PER_TILE, xa, old);
      t1 = t3;
    }
  } else {
    pro();
  }
  if (ntiles_full * COLS_PER_TILE < a.N && wave_id == ntiles_full % nwaves) {
    const int64_t c0 = ntiles_full * COLS_PER_TILE;
    load_tile<T, D, U, true, 0, PAD>(a, c0, xa);
    // tail: old ladj only for existing columns
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < LO::NLS; ++k)
#pragma unroll
      for (int w = 0; w < LO::W; ++w) {
        const int64_t c = LO::col(c0, k, lane) + w;
        old[k][w] = (LM == 2 && c < a.N) ? ((const T*)a.ladj)[c] : (T)0;
      }
    body.template tile<true, 0>(c0, xa, old);
  }
}

// Grid of a persistent fragment kernel: one block (4 waves) per 4 wave tiles, capped at the
// resident blocks per CU (hipOccupancy; ENF_BLOCKS_PER_CU lowers it for tuning) times the CUs.
hipError_t frag_grid(const void* kernel, int64_t N, int64_t cols_per_block, size_t lds, const DeviceInfo& dev,
                     int64_t* blocks);

}  // namespace enf
