// enf_grad_tail.h -- the reduction side of the whitening-loss gradient (config 5), shared by the generic
// gradient kernel (enf_grad.hip) and the fused (J o H)^n kernels (enf_grad_hj.hip).
//
// Every gradient block writes one partial vector [loss, gradient...] (double). They are summed in
// kSumSlices slices of consecutive blocks, each slice in block order (grad_sum_kernel's fixed tree), the
// slices in order, then the Householder direction projection (householder_trafo.jl:22-40) and, for the
// fused single-rank optimize_whitening step, the loss / ADAGrad / re-normalisation
// (optimize_whitening.jl:36-42).
//
// Round 3 measured running the finalisation / whitening tail inside the slice-sum launch (a ticket taken
// after a device-scope fence, the last block runs the rest): 50.7 vs 44.7 us per config-5 step, and in the
// gradient kernel 98.7 vs 44.5 us -- on gfx950 each device-scope fence writes back and invalidates the XCD's
// L2 (profiles/r03_train_sum_tail_ab.txt, r03_train_fused_tail_in_gradient_ab.txt). Rejected; round 4
// removed that code path, so the product always launches the slice sums and the tail separately.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "enf_internal.h"
#include "enf_train.h"

namespace enf {

constexpr int kMaxGradSteps = 32;
constexpr int kSumSlices = 8;

// Sum the block partials (double, block order), project Householder direction gradients, add to out.
struct ReduceArgs {
  const double* partial;
  int32_t nblocks;
  int32_t nparams;
  int32_t D;
  int32_t nh;  // Householder columns
  int32_t skip_loss;  // enf_flow_vjp: out has no loss slot (out[i - 1] += tot[i])
  void* out;
  double* tot;  // kSumSlices x (1 + nparams) slice totals (workspace tail); slice 0 = the total
  // per Householder column: offset of its gradient vector and its device column pointer
  int32_t hoff[kMaxGradSteps];
  const void* hcol[kMaxGradSteps];
};

// The rest of a single-rank optimize_whitening step (enf_whitening_step) / the update half of a
// data-parallel one (enf_whitening_apply).
struct StepArgs {
  void* theta;
  void* acc;
  double* loss_out;
  double scale, eta, eps;
  int64_t D, nsamp;
  int32_t nruns, nhb;
  int64_t runs[kMaxStepRuns][2];
  int64_t hb[kMaxStepHB][3];  // offset, k, ldv
};

// Slices -> total, then the Householder direction projection on tot (whole block of 4 waves; ends
// with a barrier, tot[0 .. nparams] final).
template <typename T>
__device__ __forceinline__ void finalize_totals(const ReduceArgs& r) {
  double* tot = r.tot;
  const int64_t n = 1 + (int64_t)r.nparams;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // Householder columns h = w, w + 4, ... of this wave: their first 64 entries (one per lane; D > 64
  // adds entries lane + 64, lane + 128, ... below) loaded while the slices are summed (they do not
  // depend on the totals)
  constexpr int kPerWave = (kMaxGradSteps + 3) / 4;
  double vh[kPerWave], nrm[kPerWave];
#pragma unroll
  for (int j = 0; j < kPerWave; ++j) {
    const int h = w + 4 * j;
    vh[j] = (h < r.nh && lane < r.D) ? (double)((const T*)r.hcol[h])[lane] : 0.0;
  }
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {  // the slices in order, into slice 0
    double t = tot[i];
    for (int s = 1; s < kSumSlices; ++s) t += tot[s * n + i];
    tot[i] = t;
  }
#pragma unroll
  for (int j = 0; j < kPerWave; ++j) {
    const int h = w + 4 * j;
    double vv = vh[j] * vh[j];
    if (h < r.nh)
      for (int d = lane + 64; d < r.D; d += 64) {
        const double v = (double)((const T*)r.hcol[h])[d];
        vv += v * v;
      }
    for (int m = 32; m >= 1; m >>= 1) vv += __shfl_xor(vv, m);
    nrm[j] = sqrt(vv);
  }
  __syncthreads();
  // Householder: dS/dw = -sqrt2 * G;  dS/dv = (dS/dw - w (dS/dw . w)) / |v|  (householder_trafo.jl:32)
#pragma unroll
  for (int j = 0; j < kPerWave; ++j) {
    const int h = w + 4 * j;
    if (h >= r.nh) break;  // wave-uniform
    double* gw = tot + 1 + r.hoff[h];
    const T* vc = (const T*)r.hcol[h];
    const double g = lane < r.D ? gw[lane] : 0.0;
    const double wv = vh[j] / nrm[j];
    double wd = -1.4142135623730951 * g * wv;
    for (int d = lane + 64; d < r.D; d += 64) wd += -1.4142135623730951 * gw[d] * ((double)vc[d] / nrm[j]);
    for (int m = 32; m >= 1; m >>= 1) wd += __shfl_xor(wd, m);
    if (lane < r.D) gw[lane] = (-1.4142135623730951 * g - wv * wd) / nrm[j];
    for (int d = lane + 64; d < r.D; d += 64)
      gw[d] = (-1.4142135623730951 * gw[d] - ((double)vc[d] / nrm[j]) * wd) / nrm[j];
  }
  __syncthreads();
}

// grad_finalize_kernel's work: totals, projection, added into out
template <typename T>
__device__ __forceinline__ void finalize_into_out(const ReduceArgs& r) {
  finalize_totals<T>(r);
  T* out = (T*)r.out;
  if (r.skip_loss) {
    for (int i = threadIdx.x; i < r.nparams; i += blockDim.x) out[i] += (T)r.tot[1 + i];
  } else {
    for (int i = threadIdx.x; i < 1 + r.nparams; i += blockDim.x) out[i] += (T)r.tot[i];
  }
}

// whitening_tail_kernel's work (S: StepArgs): loss/B (as the host computes out[0] / B in T),
// ADAGrad over the trainable runs with g = (T)total (what enf_adagrad_step reads from a zeroed out), then
// the Householder re-normalisation of every batch -- the operations and roundings of the unfused sequence.
template <typename T, typename S>
__device__ __forceinline__ void whitening_tail_body(const ReduceArgs& r, const S& a) {
  finalize_totals<T>(r);
  const double* tot = r.tot;
  T* th = (T*)a.theta;
  T* ac = (T*)a.acc;
  if (threadIdx.x == 0) *a.loss_out = (double)((T)tot[0] / (T)a.nsamp);
  for (int q = 0; q < a.nruns; ++q)
    for (int64_t i = a.runs[q][0] + threadIdx.x; i < a.runs[q][1]; i += blockDim.x)
      adagrad_update<T>(th[i], ac[i], (T)tot[1 + i], (T)a.scale, (T)a.eta, (T)a.eps);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int q = 0; q < a.nhb; ++q)
    for (int64_t c = w; c < a.hb[q][1]; c += 4) normalize_column<T>(th + a.hb[q][0] + c * a.hb[q][2], a.D, lane);
}

}  // namespace enf
