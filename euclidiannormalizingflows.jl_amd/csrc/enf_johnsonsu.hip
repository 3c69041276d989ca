// enf_johnsonsu.hip -- the JohnsonSU distribution on the device:
// elementwise pdf / logpdf / cdf / logcdf / ccdf / logccdf / quantile (src/johnson_trafo.jl:120-129)
// and inverse-CDF sampling, which is what rand(JohnsonSU(...), n) does in the reference
// (Distributions' fallback rand -> quantile(d, rand()), exercised by test/test_johnson_trafo.jl:12-14).
//
// Formulas follow the reference line by line, in the precision T of the data:
//   y = johnsontrafo(x) = gamma + delta asinh((x - xi)/lambda)                    (johnson_trafo.jl:29-32)
//   deriv = (delta/lambda) / sqrt(1 + ((x - xi)/lambda)^2)                         (:39-42)
//   pdf = deriv * normpdf(y), logpdf = log(deriv * normpdf(y))                     (:120,123)
//   cdf = normcdf(y), logcdf = normlogcdf(y)                                       (:121,124)
//   ccdf = 1 - cdf, logccdf = log(1 - cdf)                                         (:125-126)
//   quantile(p) = johnsontrafo_inv(norminvcdf(p)) = lambda sinh((z - gamma)/delta) + xi  (:129, :34-37)
// with the StatsFuns definitions normpdf(y) = exp(-y^2/2)/sqrt(2 pi), normcdf(y) = erfc(-y/sqrt2)/2,
// normlogcdf(y) = log(erfcx(-y/sqrt2)/2) - y^2/2 for y < -1 else log1p(-erfc(y/sqrt2)/2),
// norminvcdf(p) = -sqrt2 erfcinv(2p) (= +sqrt2 erfcinv(2(1-p)) above 1/2). The reference's own tail behaviour is kept (logpdf of a
// product underflows to -Inf where the reference's does; ccdf = 1 - cdf loses the upper tail).
//
// Sampling: u_i uniform on (0, 1) from Philox4x32-10 (counter = offset + i / per-call samples,
// key = seed; 4 fp32 or 2 fp64 samples per call), x_i = quantile(u_i). Deterministic for a given
// (seed, offset), so sharded draws (offset = first sample index / samples per call) equal one draw.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "enf.h"
#include "enf_internal.h"

namespace enf {

namespace {

template <typename T>
struct JSU {
  T g, d, xi, l;
};

__device__ __forceinline__ float d_asinh(float x) { return asinhf(x); }
__device__ __forceinline__ double d_asinh(double x) { return asinh(x); }
__device__ __forceinline__ float d_sinh(float x) { return sinhf(x); }
__device__ __forceinline__ double d_sinh(double x) { return sinh(x); }
__device__ __forceinline__ float d_sqrt(float x) { return sqrtf(x); }
__device__ __forceinline__ double d_sqrt(double x) { return sqrt(x); }
__device__ __forceinline__ float d_exp(float x) { return expf(x); }
__device__ __forceinline__ double d_exp(double x) { return exp(x); }
__device__ __forceinline__ float d_log(float x) { return logf(x); }
__device__ __forceinline__ double d_log(double x) { return log(x); }
__device__ __forceinline__ float d_log1p(float x) { return log1pf(x); }
__device__ __forceinline__ double d_log1p(double x) { return log1p(x); }
__device__ __forceinline__ float d_erfc(float x) { return erfcf(x); }
__device__ __forceinline__ double d_erfc(double x) { return erfc(x); }
__device__ __forceinline__ float d_erfcx(float x) { return erfcxf(x); }
__device__ __forceinline__ double d_erfcx(double x) { return erfcx(x); }
__device__ __forceinline__ float d_erfcinv(float x) { return erfcinvf(x); }
__device__ __forceinline__ double d_erfcinv(double x) { return erfcinv(x); }

template <typename T>
__device__ __forceinline__ T jsu_eval(int fn, T x, const JSU<T>& p) {
  constexpr T kInvSqrt2 = (T)0.70710678118654752440;
  constexpr T kSqrt2 = (T)1.41421356237309504880;
  constexpr T kInvSqrt2Pi = (T)0.39894228040143267794;
  if (fn == ENF_JSU_QUANTILE) {
    // norminvcdf(p) = -sqrt2 erfcinv(2p), evaluated on the lower tail for both halves (1 - p is
    // exact for p >= 1/2): erfcinv near 2 loses the upper tail in fp32 (measured 3e-4 relative at
    // p = 1 - 2^-24), erfcinv near 0 does not
    const bool upper = x > (T)0.5;
    const T zl = -kSqrt2 * d_erfcinv((T)2 * (upper ? (T)1 - x : x));
    const T z = upper ? -zl : zl;
    return p.l * d_sinh((z - p.g) / p.d) + p.xi;
  }
  const T u = (x - p.xi) / p.l;
  const T y = p.g + p.d * d_asinh(u);
  switch (fn) {
    case ENF_JSU_PDF:
    case ENF_JSU_LOGPDF: {
      const T deriv = (p.d / p.l) * ((T)1 / d_sqrt((T)1 + u * u));
      const T pdf = deriv * (d_exp(-(y * y) / (T)2) * kInvSqrt2Pi);
      return fn == ENF_JSU_PDF ? pdf : d_log(pdf);
    }
    case ENF_JSU_CDF: return d_erfc(-y * kInvSqrt2) / (T)2;
    case ENF_JSU_LOGCDF:
      return y < (T)-1 ? d_log(d_erfcx(-y * kInvSqrt2) / (T)2) - y * y / (T)2
                       : d_log1p(-d_erfc(y * kInvSqrt2) / (T)2);
    case ENF_JSU_CCDF: return (T)1 - d_erfc(-y * kInvSqrt2) / (T)2;
    default: return d_log((T)1 - d_erfc(-y * kInvSqrt2) / (T)2);  // ENF_JSU_LOGCCDF
  }
}

template <typename T>
__global__ __launch_bounds__(256) void jsu_eval_kernel(int fn, int64_t n, const T* __restrict__ x, T* __restrict__ out,
                                                       JSU<T> p) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = jsu_eval<T>(fn, x[i], p);
}

// Philox4x32-10 (Salmon et al., SC'11): 10 rounds of the 4x32 S-box with the published constants
struct U4 {
  uint32_t v[4];
};
__device__ __forceinline__ U4 philox4x32_10(uint64_t ctr, uint64_t seed) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0u, c3 = 0u;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return {{c0, c1, c2, c3}};
}

// u in (0, 1): midpoints of the 2^-23 (fp32) / 2^-52 (fp64) grids, so u is never 0 or 1 after
// rounding (the largest value, 1 - 2^-24 resp. 1 - 2^-53, is representable)
__device__ __forceinline__ float uniform_f32(uint32_t w) { return ((float)(w >> 9) + 0.5f) * 0x1p-23f; }
__device__ __forceinline__ double uniform_f64(uint32_t hi, uint32_t lo) {
  const uint64_t m = (((uint64_t)hi << 32) | lo) >> 12;
  return ((double)m + 0.5) * 0x1p-52;
}

template <typename T>
__global__ __launch_bounds__(256) void jsu_sample_kernel(int64_t n, T* __restrict__ out, JSU<T> p, uint64_t seed,
                                                         uint64_t offset) {
  constexpr int PER = sizeof(T) == 4 ? 4 : 2;  // samples per Philox call
  const int64_t calls = (n + PER - 1) / PER;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < calls; c += (int64_t)gridDim.x * blockDim.x) {
    const U4 r = philox4x32_10(offset + (uint64_t)c, seed);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int64_t i = c * PER + k;
      if (i >= n) break;
      T u;
      if constexpr (sizeof(T) == 4) u = uniform_f32(r.v[k]);
      else u = uniform_f64(r.v[2 * k], r.v[2 * k + 1]);
      out[i] = jsu_eval<T>(ENF_JSU_QUANTILE, u, p);
    }
  }
}

int64_t grid_for(int64_t work, const DeviceInfo& dev) {
  int64_t b = (work + 255) / 256;
  const int64_t cap = (int64_t)dev.num_cu * 16;
  return b < 1 ? 1 : (b > cap ? cap : b);
}

}  // namespace

hipError_t launch_jsu_eval(bool f64, int fn, int64_t n, const void* x, void* out, const double (&prm)[4], hipStream_t st,
                           const DeviceInfo& dev) {
  const unsigned blocks = (unsigned)grid_for(n, dev);
  if (f64) {
    const JSU<double> p{prm[0], prm[1], prm[2], prm[3]};
    hipLaunchKernelGGL(jsu_eval_kernel<double>, dim3(blocks), dim3(256), 0, st, fn, n, (const double*)x, (double*)out, p);
  } else {
    const JSU<float> p{(float)prm[0], (float)prm[1], (float)prm[2], (float)prm[3]};
    hipLaunchKernelGGL(jsu_eval_kernel<float>, dim3(blocks), dim3(256), 0, st, fn, n, (const float*)x, (float*)out, p);
  }
  return hipGetLastError();
}

hipError_t launch_jsu_sample(bool f64, int64_t n, void* out, const double (&prm)[4], uint64_t seed, uint64_t offset,
                             hipStream_t st, const DeviceInfo& dev) {
  const int64_t calls = (n + (f64 ? 1 : 3)) / (f64 ? 2 : 4);
  const unsigned blocks = (unsigned)grid_for(calls, dev);
  if (f64) {
    const JSU<double> p{prm[0], prm[1], prm[2], prm[3]};
    hipLaunchKernelGGL(jsu_sample_kernel<double>, dim3(blocks), dim3(256), 0, st, n, (double*)out, p, seed, offset);
  } else {
    const JSU<float> p{(float)prm[0], (float)prm[1], (float)prm[2], (float)prm[3]};
    hipLaunchKernelGGL(jsu_sample_kernel<float>, dim3(blocks), dim3(256), 0, st, n, (float*)out, p, seed, offset);
  }
  return hipGetLastError();
}

}  // namespace enf
