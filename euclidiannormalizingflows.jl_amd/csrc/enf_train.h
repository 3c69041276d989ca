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
// cross-rank sum ar of the slice totals (double; none on one rank), then the tail normalised by the global batch
// B (loss, ADAGrad, re-normalisation) -- whitening_step is the case B = N, ar = none
enf_status whitening_step_dp(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                             int32_t nlayers, void* theta, void* acc, const int64_t* runs, int32_t nruns,
                             const int64_t* hb, int32_t nhb, double eta, double epsilon, int64_t B, double* loss_out,
                             AllreduceFn ar, void* ar_ctx, void* workspace, size_t workspace_bytes, hipStream_t st);
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

// The sum over a wave's lanes of values held as d = lane, lane + 64, ... < D (lanes >= D hold zeros): the xor
// tree from half the smallest power of two >= min(D, 64) down; the strides it leaves out would only add zeros, so
// the value is that of the full 64-lane tree (round 5: 1 stage instead of 6 at D = 2). Every lane < D gets it.
__device__ __forceinline__ double lane_sum(double v, int64_t D) {
  int m = 32;
  if (D < 64) {
    m = 1;
    while (m < D) m <<= 1;
    m >>= 1;
  }
  for (; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
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
