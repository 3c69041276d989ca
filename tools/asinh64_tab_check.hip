// Accuracy probe of the fp64 table functions of enf_math64.h that the compiled fp64 program uses (design probe,
// not product; round 4): asinh64_tab_fin over |x| < 2^26 (the range flow_hj64_kernel's check admits) and,
// to show why the check is needed, over 2^26 .. 2^500 (1/u = (s1 - a) + corr loses to rounding past ~2^40),
// asinh64_tab over the whole double range, log64_tab over u >= 1 (the degree-6 log1p polynomial), each in ulps
// against x86 long-double asinhl / logl (also their FOLD variants); sinh64_in (the fp64 inverse program's sinh) and sinh64 over |w| < 709
// against sinhl.
// Build: hipcc --offload-arch=gfx950 -O3 -I euclidiannormalizingflows.jl_amd/csrc \
//          -o tools/asinh64_tab_check tools/asinh64_tab_check.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "enf_math64.h"
#include "enf_logtab_b78.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

template <int F>
__global__ __launch_bounds__(256) void eval(const double* x, double* y, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  if (F == 0) y[i] = enf::asinh64_tab_fin(v, enf::kLogTab);
  if (F == 1) y[i] = enf::asinh64_tab(v, enf::kLogTab);
  if (F == 2) y[i] = enf::log64_tab(v, 0, enf::kLogTab);
  if (F == 3) y[i] = enf::sinh64_in(v);
  if (F == 4) y[i] = enf::sinh64(v);
  if (F == 5) y[i] = enf::asinh64_tab_fin<enf::kLogTabBits, true>(v, enf::kLogTab);
  if (F == 6) y[i] = enf::log64_tab_b<enf::kLogTabBits, true>(v, 0, enf::kLogTab);
  if (F == 8) y[i] = enf::asinh64_tab_fin<6>(v, enf::kLogTabB6);
  if (F == 9) y[i] = enf::log64_tab_b<6>(v, 0, enf::kLogTabB6);
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
  std::mt19937_64 g(11);
  std::vector<double> xs;
  for (int i = 0; i <= 400000; ++i) xs.push_back(std::pow(10.0, -320.0 + 628.0 * i / 400000.0));
  std::uniform_real_distribution<double> U(0, 1);
  for (int i = 0; i < 400000; ++i) xs.push_back(4.0 * U(g));
  for (int i = 0; i < 400000; ++i) xs.push_back(std::ldexp(1.0 + U(g), (int)(40 * U(g)) - 20));
  for (int i = 0; i < 200000; ++i) xs.push_back(std::ldexp(1.0 + U(g), 20 + (int)(480 * U(g))));  // 2^20..2^500
  std::normal_distribution<double> N(0, 1);
  for (int i = 0; i < 400000; ++i) xs.push_back(N(g) * 3);
  for (int i = 0; i < 200000; ++i) xs.push_back(709.0 * U(g));
  const double sp[] = {0.0, 5e-324, 1e-300, 1.0, 2.0, 67108864.0, std::nextafter(67108864.0, 0.0),
                       0x1p499, 0x1p500, 1.7976931348623157e308, INFINITY, NAN};
  for (double v : sp) xs.push_back(v);
  const size_t n0 = xs.size();
  for (size_t i = 0; i < n0; ++i) xs.push_back(-xs[i]);
  const long n = xs.size();
  double *dx, *dy;
  CK(hipMalloc(&dx, n * 8));
  CK(hipMalloc(&dy, n * 8));
  CK(hipMemcpy(dx, xs.data(), n * 8, hipMemcpyHostToDevice));
  std::vector<double> y(n);
  const char* nm[10] = {"asinh64_tab_fin (|x| < 2^26)", "asinh64_tab", "log64_tab (u >= 1)",
                       "sinh64_in (|w| < 709)", "sinh64 (|w| < 709)", "asinh64_tab_fin FOLD", "log64_tab FOLD",
                       "asinh64_tab_fin 2^26..2^500", "asinh64_tab_fin B=6", "log64_tab B=6"};
  for (int f = 0; f < 10; ++f) {
    const int blocks = (n + 255) / 256;
    if (f == 0) eval<0><<<blocks, 256>>>(dx, dy, n);
    if (f == 1) eval<1><<<blocks, 256>>>(dx, dy, n);
    if (f == 2) eval<2><<<blocks, 256>>>(dx, dy, n);
    if (f == 3) eval<3><<<blocks, 256>>>(dx, dy, n);
    if (f == 4) eval<4><<<blocks, 256>>>(dx, dy, n);
    if (f == 5) eval<5><<<blocks, 256>>>(dx, dy, n);
    if (f == 6) eval<6><<<blocks, 256>>>(dx, dy, n);
    if (f == 7) eval<0><<<blocks, 256>>>(dx, dy, n);
    if (f == 8) eval<8><<<blocks, 256>>>(dx, dy, n);
    if (f == 9) eval<9><<<blocks, 256>>>(dx, dy, n);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(y.data(), dy, n * 8, hipMemcpyDeviceToHost));
    double worst = 0, sum = 0;
    long cnt = 0, worst_i = 0, over1 = 0;
    for (long i = 0; i < n; ++i) {
      const double v = xs[i];
      long double ref;
      if (f == 0 || f == 5 || f == 8) {
        if (!(std::fabs(v) < 0x1p26)) continue;
        ref = asinhl((long double)v);
      } else if (f == 7) {
        if (!(std::fabs(v) >= 0x1p26 && std::fabs(v) < 0x1p500)) continue;
        ref = asinhl((long double)v);
      } else if (f == 1) {
        ref = asinhl((long double)v);
      } else if (f == 2 || f == 6 || f == 9) {
        if (!(v >= 1.0) || std::isinf(v)) continue;
        ref = logl((long double)v);
      } else {
        if (!(std::fabs(v) < 709.0)) continue;
        ref = sinhl((long double)v);
      }
      const double e = ulps(y[i], ref);
      sum += e < 1e29 ? e : 0;
      over1 += e > 1.0;
      ++cnt;
      if (e > worst) { worst = e; worst_i = i; }
    }
    printf("%-30s n=%ld max ulp %.3f (x=%.17g got %.17g) mean ulp %.4f, %ld above 1 ulp\n", nm[f], cnt, worst,
           xs[worst_i], y[worst_i], sum / cnt, over1);
  }
  return 0;
}
