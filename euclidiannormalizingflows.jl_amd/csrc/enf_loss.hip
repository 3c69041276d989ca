// enf_loss.hip -- mvnormal_negll_trafo (src/optimize_whitening.jl:7-15) on the device, loss only
// (enf_flow_negll): the flow's (Y, ladj) from enf_flow_apply into the workspace, then a deterministic
// reduction  sum_j [ sum_d (Y_dj^2 + log 2pi)/2 - ladj_j ]  added to out[0]. Any flow enf_flow_apply
// takes (no dimension or step bound, unlike the gradient kernels), so the Julia and Python hosts never
// copy Y to the host to form the loss.
//
// Per element: std_normal_logpdf(y) = -(y^2 + log 2pi)/2 (:4); the reference sums it in T (Julia's
// pairwise sum) and the ladj row in T (:12); here every term is accumulated in double in a fixed order
// (per thread a grid-strided sum, per block a tree, the blocks in index order, the chunks in order), so the
// result is deterministic and within rounding of the reference's.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "enf.h"
#include "enf_internal.h"
#include "enf_train.h"

namespace enf {

constexpr int kLossBlocks = 1024;  // partial sums (blocks of 256 threads)
constexpr double kLog2Pi = 1.8378770664093454836;

__device__ __forceinline__ double block_sum256(double v, double* red) {
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

template <typename T>
__global__ __launch_bounds__(256) void negll_partial_kernel(const T* __restrict__ Y, const T* __restrict__ ladj,
                                                            int64_t DN, int64_t N, double* __restrict__ part) {
  __shared__ double red[4];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double s = 0.0;
  for (int64_t i = i0; i < DN; i += stride) {
    const double y = (double)Y[i];
    s += 0.5 * (y * y + kLog2Pi);
  }
  for (int64_t j = i0; j < N; j += stride) s -= (double)ladj[j];
  const double t = block_sum256(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// the block partials in order, added to the running double total of the call (first chunk: set)
__global__ __launch_bounds__(256) void negll_chunk_kernel(const double* __restrict__ part, int nblocks,
                                                          double* __restrict__ total, int first) {
  __shared__ double red[4];
  double s = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += blockDim.x) s += part[b];
  const double t = block_sum256(s, red);
  if (threadIdx.x == 0) *total = first ? t : *total + t;
}

template <typename T>
__global__ void negll_out_kernel(const double* __restrict__ total, T* __restrict__ out) {
  if (threadIdx.x == 0) out[0] += (T)*total;
}

static size_t al256(size_t b) { return (b + 255) / 256 * 256; }

// Columns per chunk of enf_flow_negll (the workspace held a whole D x N copy of Y): the flow's
// output of at most this many columns is reduced at a time, so the workspace is O(D * chunk).
constexpr int64_t kLossChunkCols = (int64_t)1 << 20;
static int64_t loss_chunk(int64_t N) { return N < kLossChunkCols ? (N > 0 ? N : 1) : kLossChunkCols; }

enf_status negll_loss_workspace(bool f64, int64_t D, int64_t N, size_t* bytes) {
  const size_t e = f64 ? 8 : 4;
  const int64_t C = loss_chunk(N);
  *bytes = al256((size_t)(D > 0 ? D : 1) * (size_t)C * e) + al256((size_t)C * e) +
           al256((size_t)kLossBlocks * sizeof(double)) + 256;
  return ENF_OK;
}

// sum_j [sum_d (Y_dj^2 + log 2pi)/2 - L_j] of N columns (Y: D x N contiguous) into *total (first: set, else
// added), in double, in a fixed order
enf_status negll_reduce(bool f64, int64_t D, int64_t N, const void* Y, const void* L, double* part, double* total,
                        bool first, hipStream_t st) {
  const int64_t DN = D * N;
  int64_t nb = (DN + 255) / 256;
  if (nb > kLossBlocks) nb = kLossBlocks;
  if (nb < 1) nb = 1;
  if (f64)
    hipLaunchKernelGGL((negll_partial_kernel<double>), dim3((unsigned)nb), dim3(256), 0, st, (const double*)Y,
                       (const double*)L, DN, N, part);
  else
    hipLaunchKernelGGL((negll_partial_kernel<float>), dim3((unsigned)nb), dim3(256), 0, st, (const float*)Y,
                       (const float*)L, DN, N, part);
  hipLaunchKernelGGL(negll_chunk_kernel, dim3(1), dim3(256), 0, st, (const double*)part, (int)nb, total, first ? 1 : 0);
  const hipError_t h = hipGetLastError();
  return h == hipSuccess ? ENF_OK : set_error(ENF_ERR_HIP, hipGetErrorString(h));
}

enf_status negll_add_total(bool f64, const double* total, void* out, hipStream_t st) {
  if (f64) hipLaunchKernelGGL((negll_out_kernel<double>), dim3(1), dim3(64), 0, st, total, (double*)out);
  else hipLaunchKernelGGL((negll_out_kernel<float>), dim3(1), dim3(64), 0, st, total, (float*)out);
  const hipError_t h = hipGetLastError();
  return h == hipSuccess ? ENF_OK : set_error(ENF_ERR_HIP, hipGetErrorString(h));
}

enf_status negll_loss(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                      int32_t nlayers, void* out, void* workspace, size_t workspace_bytes, hipStream_t st) {
  size_t need = 0;
  negll_loss_workspace(f64, D, N, &need);
  if (!workspace || workspace_bytes < need) return set_error(ENF_ERR_INVALID, "enf_flow_negll: workspace too small");
  const size_t e = f64 ? 8 : 4;
  const int64_t C = loss_chunk(N), Dr = D > 0 ? D : 1;
  char* Y = (char*)workspace;
  char* L = Y + al256((size_t)Dr * (size_t)C * e);
  double* part = (double*)(L + al256((size_t)C * e));
  double* total = part + al256((size_t)kLossBlocks * sizeof(double)) / sizeof(double);
  for (int64_t c0 = 0; c0 < N; c0 += C) {
    const int64_t n = N - c0 < C ? N - c0 : C;
    const char* Xc = (const char*)X + (size_t)c0 * (size_t)ldx * e;
    enf_status s = enf_flow_apply(f64 ? ENF_F64 : ENF_F32, D, n, Xc, ldx, Y, Dr, L, 0, layers, nlayers, st);
    if (s != ENF_OK) return s;
    s = negll_reduce(f64, D, n, Y, L, part, total, c0 == 0, st);
    if (s != ENF_OK) return s;
  }
  return negll_add_total(f64, total, out, st);
}

}  // namespace enf
