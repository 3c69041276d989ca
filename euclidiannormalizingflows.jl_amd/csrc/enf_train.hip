// enf_train.hip -- training path of optimize_whitening (src/optimize_whitening.jl:25-45):
// the optimiser step and the HouseholderTrafo functor re-normalisation on the device.
// The fused forward+backward gradient kernel lives in enf_grad.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <type_traits>

#include "enf_train.h"

namespace enf {

// Optimisers.jl 0.2 ADAGrad apply!: acc .+= dx.^2; dx' = dx * eta / (sqrt(acc) + epsilon);
// Optimisers.update: x .-= dx'. g = grad * grad_scale (1/global batch size).
template <typename T>
__global__ void adagrad_kernel(int64_t n, T* __restrict__ p, T* __restrict__ acc, const T* __restrict__ g,
                               T scale, T eta, T eps) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    adagrad_update<T>(p[i], acc[i], g[i], scale, eta, eps);
}

enf_status adagrad_step(bool f64, int64_t count, void* params, void* acc, const void* grad, double grad_scale,
                        double eta, double epsilon, hipStream_t st) {
  int64_t blocks = (count + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (f64)
    hipLaunchKernelGGL(adagrad_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, st, count, (double*)params,
                       (double*)acc, (const double*)grad, grad_scale, eta, epsilon);
  else
    hipLaunchKernelGGL(adagrad_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, st, count, (float*)params,
                       (float*)acc, (const float*)grad, (float)grad_scale, (float)eta, (float)epsilon);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ENF_OK : set_error(ENF_ERR_HIP, hipGetErrorString(e));
}

// LinearAlgebra.normalize! of every column (src/householder_trafo.jl:135-139): v .*= inv(norm(v)).
// One wave per column; the sum of squares in double.
template <typename T>
__global__ void normalize_kernel(int64_t D, int64_t k, T* __restrict__ V, int64_t ldv) {
  const int lane = threadIdx.x & 63;
  const int64_t col = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (col >= k) return;  // whole wave exits together
  normalize_column<T>(V + col * ldv, D, lane);
}

enf_status householder_normalize(bool f64, int64_t D, int64_t k, void* V, int64_t ldv, hipStream_t st) {
  const unsigned blocks = (unsigned)((k + 3) / 4);
  if (f64) hipLaunchKernelGGL(normalize_kernel<double>, dim3(blocks), dim3(256), 0, st, D, k, (double*)V, ldv);
  else hipLaunchKernelGGL(normalize_kernel<float>, dim3(blocks), dim3(256), 0, st, D, k, (float*)V, ldv);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ENF_OK : set_error(ENF_ERR_HIP, hipGetErrorString(e));
}

}  // namespace enf
