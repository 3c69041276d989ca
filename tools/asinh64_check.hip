// Accuracy and throughput probe for the fp64 asinh / log / sinh / log1p of enf_math64.h against ocml's (design
// probe, not product). Accuracy: ulp error of both against x86 long-double asinhl / logl over a
// wide sweep (1e-320 .. 1e308, both signs, special values). Throughput: 1e8 evaluations each.
// Build: hipcc --offload-arch=gfx950 -O3 -I euclidiannormalizingflows.jl_amd/csrc \
//          -o tools/asinh64_check tools/asinh64_check.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "enf_math64.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

template <int F>
__global__ __launch_bounds__(256) void eval(const double* x, double* y, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  if (F == 0) y[i] = asinh(v);
  if (F == 1) y[i] = enf::asinh64(v);
  if (F == 2) y[i] = log(v);
  if (F == 3) y[i] = enf::log64_ge1(v);
  if (F == 4) y[i] = sinh(v);
  if (F == 5) y[i] = enf::sinh64(v);
  if (F == 6) y[i] = log1p(v);
  if (F == 7) y[i] = enf::log1p64_ge0(v);
}

// throughput: 8 independent elements per lane, each through `rep` dependent evaluations
template <int F>
__global__ __launch_bounds__(256) void thr(double* out, int rep, double seed) {
  double a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = seed * (threadIdx.x + 1) + k;
  for (int r = 0; r < rep; ++r)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (F == 0) a[k] = asinh(a[k]) * 3.0 + 1.0;
      if (F == 1) a[k] = enf::asinh64(a[k]) * 3.0 + 1.0;
      if (F == 2) a[k] = sinh(a[k]) * 0.3 + 0.5;
      if (F == 3) a[k] = enf::sinh64(a[k]) * 0.3 + 0.5;
    }
  double s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k];
  out[(long)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static double ulps(double got, long double ref) {
  if (std::isnan((double)ref)) return std::isnan(got) ? 0 : 1e30;
  if (std::isinf((double)ref)) return got == (double)ref ? 0 : 1e30;
  const double r = (double)ref;
  if (r == 0) return got == 0 && std::signbit(got) == std::signbit(r) ? 0 : 1e30;
  int e;
  std::frexp(r, &e);
  const long double u = std::ldexp(1.0L, std::max(e - 53, -1074));
  return (double)(std::fabs((long double)got - ref) / u);
}

int main() {
  std::mt19937_64 g(7);
  std::vector<double> xs;
  for (int i = 0; i <= 200000; ++i) xs.push_back(std::pow(10.0, -320.0 + 628.0 * i / 200000.0));
  std::uniform_real_distribution<double> U(0, 1);
  for (int i = 0; i < 400000; ++i) xs.push_back(4.0 * U(g));           // around the a = 2 switch
  for (int i = 0; i < 200000; ++i) xs.push_back(std::ldexp(1.0 + U(g), 28 - (int)(4 * U(g))));
  std::normal_distribution<double> N(0, 1);
  for (int i = 0; i < 200000; ++i) xs.push_back(N(g) * 3);
  for (int i = 0; i < 200000; ++i) xs.push_back(720.0 * U(g));         // the sinh range
  for (double v : {0.999999999, 1.0, 1.0000000001, 709.78, 710.0, 710.47, 710.48, 711.0}) xs.push_back(v);
  const double sp[] = {0.0, 5e-324, 1e-300, 1.0, 2.0, std::nextafter(2.0, 3.0), 268435456.0,
                       std::nextafter(268435456.0, 0.0), 1.7976931348623157e308, INFINITY, NAN};
  for (double v : sp) xs.push_back(v);
  const size_t n0 = xs.size();
  for (size_t i = 0; i < n0; ++i) xs.push_back(-xs[i]);
  const long n = xs.size();
  double *dx, *dy;
  CK(hipMalloc(&dx, n * 8));
  CK(hipMalloc(&dy, n * 8));
  CK(hipMemcpy(dx, xs.data(), n * 8, hipMemcpyHostToDevice));
  std::vector<double> y(n);
  const char* nm[8] = {"ocml asinh", "asinh64", "ocml log", "log64_ge1", "ocml sinh", "sinh64", "ocml log1p",
                       "log1p64_ge0"};
  for (int f = 0; f < 8; ++f) {
    const int blocks = (n + 255) / 256;
    if (f == 0) eval<0><<<blocks, 256>>>(dx, dy, n);
    if (f == 1) eval<1><<<blocks, 256>>>(dx, dy, n);
    if (f == 2) eval<2><<<blocks, 256>>>(dx, dy, n);
    if (f == 3) eval<3><<<blocks, 256>>>(dx, dy, n);
    if (f == 4) eval<4><<<blocks, 256>>>(dx, dy, n);
    if (f == 5) eval<5><<<blocks, 256>>>(dx, dy, n);
    if (f == 6) eval<6><<<blocks, 256>>>(dx, dy, n);
    if (f == 7) eval<7><<<blocks, 256>>>(dx, dy, n);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(y.data(), dy, n * 8, hipMemcpyDeviceToHost));
    double worst = 0, sum = 0;
    long cnt = 0, worst_i = 0;
    for (long i = 0; i < n; ++i) {
      long double ref;
      if (f < 2) {
        ref = asinhl((long double)xs[i]);
      } else if (f < 4) {
        if (!(xs[i] >= 1.0)) continue;  // log64_ge1 domain
        ref = logl((long double)xs[i]);
      } else if (f < 6) {
        if (!(std::fabs(xs[i]) <= 720.0) && !std::isnan(xs[i]) && !std::isinf(xs[i])) continue;
        ref = sinhl((long double)xs[i]);
      } else {
        if (!(xs[i] >= 0.0)) continue;  // log1p64_ge0 domain
        ref = log1pl((long double)xs[i]);
      }
      const double e = ulps(y[i], ref);
      sum += e < 1e29 ? e : 0;
      ++cnt;
      if (e > worst) { worst = e; worst_i = i; }
    }
    printf("%-12s n=%ld max ulp %.3f (x=%.17g got %.17g) mean ulp %.4f\n", nm[f], cnt, worst, xs[worst_i],
           y[worst_i], sum / cnt);
  }
  double* dout;
  const int blocks = 256 * 8 * 4;
  CK(hipMalloc(&dout, (long)blocks * 256 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* tn[4] = {"ocml asinh", "asinh64", "ocml sinh", "sinh64"};
  for (int f = 0; f < 4; ++f) {
    for (int w = 0; w < 2; ++w) {
      const int rep = 8;
      CK(hipEventRecord(e0));
      if (f == 0) thr<0><<<blocks, 256>>>(dout, rep, 1e-3);
      if (f == 1) thr<1><<<blocks, 256>>>(dout, rep, 1e-3);
      if (f == 2) thr<2><<<blocks, 256>>>(dout, rep, 1e-3);
      if (f == 3) thr<3><<<blocks, 256>>>(dout, rep, 1e-3);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double evals = (double)blocks * 256 * 8 * rep;
      if (w) printf("%-12s %.3f ms  %.3e evals/s\n", tn[f], ms, evals / (ms * 1e-3));
    }
  }
  return 0;
}
