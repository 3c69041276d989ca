// enf_train.h -- training-path entry points (config 5: optimize_whitening), see include/enf.h.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "enf.h"
#include "enf_internal.h"

namespace enf {

enf_status set_error(enf_status st, const char* msg);
enf_status current_device_info(DeviceInfo* out);

enf_status negll_grad_workspace(bool f64, int64_t D, int64_t N, const enf_layer* layers, int32_t nlayers,
                                size_t* bytes);
enf_status negll_grad(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                      int32_t nlayers, void* out, void* workspace, size_t workspace_bytes, hipStream_t st);
enf_status negll_loss_workspace(bool f64, int64_t D, int64_t N, size_t* bytes);
// enf_loss.hip: the loss reduction of N columns (Y: D x N contiguous, L: N) into *total (double; first: set,
// else added), and *total added into out[0] (T)
enf_status negll_reduce(bool f64, int64_t D, int64_t N, const void* Y, const void* L, double* part, double* total,
                        bool first, hipStream_t st);
enf_status negll_add_total(bool f64, const double* total, void* out, hipStream_t st);
enf_status negll_loss(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                      int32_t nlayers, void* out, void* workspace, size_t workspace_bytes, hipStream_t st);
enf_status flow_vjp(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const void* dY, int64_t lddy,
                    const void* dladj, const enf_layer* layers, int32_t nlayers, void* dX, int64_t lddx, void* dparams,
                    void* workspace, size_t workspace_bytes, hipStream_t st);
enf_status adagrad_step(bool f64, int64_t count, void* params, void* acc, const void* grad, double grad_scale,
                        double eta, double epsilon, hipStream_t st);
enf_status householder_normalize(bool f64, int64_t D, int64_t k, void* V, int64_t ldv, hipStream_t st);

// Fused single-rank optimize_whitening step (enf_whitening_step): runs = [start, end) ranges of
// theta to update, hb = (offset, k, ldv) Householder column batches to re-normalise.
constexpr int kMaxStepRuns = 64;
constexpr int kMaxStepHB = 16;
enf_status whitening_step(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                          int32_t nlayers, void* theta, void* acc, const int64_t* runs, int32_t nruns,
                          const int64_t* hb, int32_t nhb, double eta, double epsilon, double* loss_out,
                          void* workspace, size_t workspace_bytes, hipStream_t st);

// In-place cross-rank sum of `count` values (f64: double, else float) on stream st (enf_whitening_step_dp: RCCL
// through the caller's communicator)
typedef enf_status (*AllreduceFn)(void* ctx, void* buf, int64_t count, bool f64, hipStream_t st);
// One rank's data-parallel optimize_whitening step (enf_whitening_step_dp): the gradient of its N columns, the
// cross-rank sum ar over nranks ranks of the slice totals -- or, on the fused (J o H)^n path, of the partial rows
// (double; none on one rank), then the tail normalised by the global batch B (loss, ADAGrad, re-normalisation) --
// whitening_step is the case B = N, ar = none, nranks = 1
enf_status whitening_step_dp(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                             int32_t nlayers, void* theta, void* acc, const int64_t* runs, int32_t nruns,
                             const int64_t* hb, int32_t nhb, double eta, double epsilon, int64_t B, double* loss_out,
                             AllreduceFn ar, void* ar_ctx, void* workspace, size_t workspace_bytes, hipStream_t st,
                             int nranks);
// The single-rank steps of one epoch over the minibatches [b0, b0 + bs) of N columns (enf_whitening_epoch)
enf_status whitening_epoch(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, int64_t bs,
                           const enf_layer* layers, int32_t nlayers, void* theta, void* acc, const int64_t* runs,
                           int32_t nruns, const int64_t* hb, int32_t nhb, double eta, double epsilon, double* loss_out,
                           void* workspace, size_t workspace_bytes, hipStream_t st);
// Update half of a data-parallel step after the all-reduce (enf_whitening_apply): g = 1 + nparams
// summed values of T, B = global batch size.
enf_status whitening_apply(bool f64, int64_t D, int64_t nparams, const void* g, int64_t B, void* theta, void* acc,
                           const int64_t* runs, int32_t nruns, const int64_t* hb, int32_t nhb, double eta,
                           double epsilon, double* loss_out, hipStream_t st);

// enf_copy.hip: the measurement copy (enf_stream_copy)
enf_status stream_copy(const void* src, void* dst, int64_t bytes, int32_t variant, hipStream_t st);

// Optimisers.jl 0.2 ADAGrad on one parameter (src/optimize_whitening.jl:40): the arithmetic shared
// by enf_adagrad_step and the fused step, so both round identically.
template <typename T>
__device__ __forceinline__ void adagrad_update(T& p, T& acc, T g, T scale, T eta, T eps) {
  const T dx = g * scale;
  const T a = acc + dx * dx;
  acc = a;
  p = p - dx * eta / (sqrt(a) + eps);
}

// Cross-lane moves without an LDS round trip (ds_bpermute, the __shfl_xor form, costs a round trip per stage on the
// chains of the one-block steps). dpp_mov<CTRL>: a DPP row move (quad_perm / row_ror) of every lane's value.
template <int CTRL, typename T>
__device__ __forceinline__ T dpp_mov(T x) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, true);
    return __builtin_bit_cast(T, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  }
}
// x + (the value of lane ^ M), M = 16 or 32, by gfx950's v_permlane16_swap / v_permlane32_swap (VALU): with both
// operands x the swap leaves x and its partner side by side, and their sum is x + __shfl_xor(x, M) bit for bit
// (the two addends are the same, and addition commutes)
template <int M, typename T>
__device__ __forceinline__ T add_xor_swap(T x) {
  static_assert(M == 16 || M == 32, "the permlane swaps pair lanes 16 or 32 apart");
#if defined(__gfx950__)
  // The instruction itself, not the builtin: hipcc 7.2 reads the builtin's second result from the first result's
  // register for a 32-bit value in this use (the swapped half added to itself: the round-5 run-27 failure, DESIGN
  // §4). Hazard (gfx950): a v_permlane16/32_swap that reads a VGPR written by a VALU instruction needs two wait
  // states after that write -- the compiler's own hazard recognizer pads its builtin with the same `s_nop 1`, but
  // it cannot see into this asm, so the pad is written here. tests/test_gpu_round6.py::test_cross_lane_primitives
  // checks every group size against the __shfl_xor butterfly bit for bit on the GPU (tests/xlane/).
  struct Pair {
    uint32_t a, b;
  };
  auto sw = [](uint32_t u) {
    Pair p{u, u};
    if constexpr (M == 32) asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(p.a), "+v"(p.b));
    else asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(p.a), "+v"(p.b));
    return p;
  };
  if constexpr (sizeof(T) == 4) {
    const Pair r = sw(__builtin_bit_cast(uint32_t, x));
    return __builtin_bit_cast(T, r.a) + __builtin_bit_cast(T, r.b);
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    const Pair lo = sw((uint32_t)u), hi = sw((uint32_t)(u >> 32));
    return __builtin_bit_cast(T, ((uint64_t)hi.a << 32) | lo.a) + __builtin_bit_cast(T, ((uint64_t)hi.b << 32) | lo.b);
  }
#else
  // (other targets -- and the host pass -- have no permlane swaps: the shuffle, bit-identical)
  return x + __shfl_xor(x, M);
#endif
}
// The xor butterfly over the lanes of a group of P (power of two, <= 64) consecutive lanes, strides P/2 .. 1 in that
// order: exactly `for (m = P / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m)`. Strides 32 and 16 are permlane swaps,
// 8 is row_ror:8 (lane (l + 8) mod 16 of the row is l ^ 8), 4 is row_ror:4 once stride 8 has made every value equal
// to its lane ^ 8 partner's (then (l + 4) mod 16 holds l ^ 4's value), 2 and 1 quad_perm; a stride-4 first stage
// (P = 8) keeps the shuffle.
template <typename T>
__device__ __forceinline__ T xor_tree(T v, int P) {
  if (P >= 64) v = add_xor_swap<32>(v);
  if (P >= 32) v = add_xor_swap<16>(v);
  if (P >= 16) v += dpp_mov<0x128>(v);  // row_ror:8
  if (P >= 16) v += dpp_mov<0x124>(v);  // row_ror:4
  else if (P >= 8) v += __shfl_xor(v, 4);
  if (P >= 4) v += dpp_mov<0x4E>(v);    // quad_perm(2,3,0,1): lane ^ 2
  if (P >= 2) v += dpp_mov<0xB1>(v);    // quad_perm(1,0,3,2): lane ^ 1
  return v;
}

// The sum over a wave's lanes of values held as d = lane, lane + 64, ... < D (lanes >= D hold zeros): the xor
// tree from half the smallest power of two >= min(D, 64) down; the strides it leaves out would only add zeros, so
// the value is that of the full 64-lane tree (round 5: 1 stage instead of 6 at D = 2). Every lane < D gets it.
__device__ __forceinline__ double lane_sum(double v, int64_t D) {
  int p = 64;
  if (D < 64) {
    p = 1;
    while (p < D) p <<= 1;
  }
  return xor_tree(v, p);
}

// LinearAlgebra.normalize! of one column by one wave (src/householder_trafo.jl:135-139), the sum
// of squares in double.
template <typename T>
__device__ __forceinline__ void normalize_column(T* __restrict__ v, int64_t D, int lane) {
  double ss = 0.0;
  for (int64_t d = lane; d < D; d += 64) ss += (double)v[d] * (double)v[d];
  ss = lane_sum(ss, D);
  const T inv = (T)(1.0 / sqrt(ss));
  for (int64_t d = lane; d < D; d += 64) v[d] *= inv;
}

}  // namespace enf
