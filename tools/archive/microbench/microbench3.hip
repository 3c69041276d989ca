// Issue-rate probe (design probe, not product): plain f32 FMA and an FMA/log mix at 1, 2, 4, 8 waves
// per SIMD, to see whether co-resident waves raise a SIMD's VALU issue rate above one wave's.
// Reports cycles per wave-instruction per SIMD using s_memtime-free wall time and the clock from
// hipDeviceProp (nominal) -- compare ratios between wave counts, not absolute cycles.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench3 tools/microbench3.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

template <int NT, int NF>
__global__ __launch_bounds__(256) void mix(float* out, int iters, float seed) {
  float a[16], b[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) { a[k] = 1.5f + seed * (threadIdx.x + k); b[k] = a[k] * 0.5f; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        float v = __builtin_amdgcn_logf(a[k]);
        asm volatile("" : "+v"(v));
        a[k] = v;
      }
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        b[k] = __builtin_fmaf(b[k], 0.999f, 1e-3f);
        asm volatile("" : "+v"(b[k]));
      }
    }
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += a[k] + b[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float* o;
  CK(hipMalloc(&o, 256 * 64 * 256 * 4));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount, iters = 4096;
  auto run = [&](auto k, const char* name, int nt, int nf) {
    for (int w : {1, 2, 4, 8}) {
      const int grid = cus * w;  // w blocks of 4 waves per CU = w waves per SIMD
      k<<<grid, 256>>>(o, iters, 1e-6f);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int r = 0; r < 3; ++r) k<<<grid, 256>>>(o, iters, 1e-6f);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 3;
      const double instr = (double)iters * 16 * (nt + nf) * w;  // wave-instructions per SIMD
      printf("%-16s waves/SIMD %d  %8.3f ms  ns per wave-instr per SIMD %.4f\n", name, w, ms, ms * 1e6 / instr);
    }
  };
  run(mix<0, 8>, "fma x8", 0, 8);
  run(mix<1, 0>, "log x1", 1, 0);
  run(mix<1, 4>, "log x1 + fma x4", 1, 4);
  return 0;
}
