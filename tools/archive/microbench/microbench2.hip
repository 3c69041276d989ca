// Issue-cost probe for the fp32 flow kernel's instruction mix on gfx950 (design probe, not product).
// 16 independent chains per lane, 8 waves per SIMD; every kernel runs the same number of loop
// iterations, so time ratios against the FMA-only kernel give issue costs in FMA units
// (v_fma_f32 wave64 = 2 cycles on a SIMD32). Mixed kernels show whether transcendental ops
// (v_log/v_exp/v_sqrt/v_rcp) overlap with plain VALU work of other waves.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench2 tools/microbench2.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

// NT = transcendental ops, NF = fma ops per chain per iteration; TR selects the transcendental
template <int NT, int NF, int TR>
__global__ __launch_bounds__(256) void mix(float* out, int iters, float seed) {
  float a[16], b[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) { a[k] = 1.5f + seed * (threadIdx.x + k); b[k] = a[k] * 0.5f; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        float v;
        if (TR == 0) v = __builtin_amdgcn_logf(a[k]);
        if (TR == 1) v = __builtin_amdgcn_sqrtf(a[k]);
        if (TR == 2) v = __builtin_amdgcn_exp2f(a[k]);
        if (TR == 3) v = __builtin_amdgcn_rcpf(a[k]);
        if (TR == 4) v = __builtin_amdgcn_rsqf(a[k]);
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

__global__ __launch_bounds__(256) void dppk(float* out, int iters, float seed) {
  float a[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) a[k] = seed * (threadIdx.x + k);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      a[k] += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a[k]), 0x141, 0xF, 0xF, false));
      asm volatile("" : "+v"(a[k]));
    }
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float* o;
  CK(hipMalloc(&o, 256 * 64 * 256 * 4));
  const int grid = 256 * 8, blk = 256, iters = 2048;  // 8 blocks/CU = 8 waves/SIMD
  auto run = [&](auto k, const char* name, int nt, int nf) {
    k<<<grid, blk>>>(o, iters, 1e-6f);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 3; ++r) k<<<grid, blk>>>(o, iters, 1e-6f);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 3;
    const double per_simd_wave_instr = (double)iters * 16 * (nt + nf) * 8;  // per SIMD (8 waves)
    printf("%-22s %8.3f ms  ns per (wave-instr per SIMD) %.4f\n", name, ms, ms * 1e6 / per_simd_wave_instr);
    return ms;
  };
  const float f8 = run(mix<0, 8, 0>, "fma x8", 0, 8);
  const float l1 = run(mix<1, 0, 0>, "log x1", 1, 0);
  const float l1f2 = run(mix<1, 2, 0>, "log x1 + fma x2", 1, 2);
  const float l1f4 = run(mix<1, 4, 0>, "log x1 + fma x4", 1, 4);
  const float l1f8 = run(mix<1, 8, 0>, "log x1 + fma x8", 1, 8);
  run(mix<1, 0, 1>, "sqrt x1", 1, 0);
  run(mix<1, 0, 2>, "exp x1", 1, 0);
  run(mix<1, 0, 3>, "rcp x1", 1, 0);
  run(mix<1, 0, 4>, "rsq x1", 1, 0);
  run(mix<1, 4, 1>, "sqrt x1 + fma x4", 1, 4);
  run(dppk, "dpp add", 0, 1);
  const double fma_ns = f8 / 8.0, log_ns = l1;
  printf("cost ratio log/fma = %.2f ; log+2fma = %.2f fma ; log+4fma = %.2f fma ; log+8fma = %.2f fma\n",
         log_ns / fma_ns, l1f2 / fma_ns, l1f4 / fma_ns, l1f8 / fma_ns);
  printf("(sum model: log+Nfma = %.2f + N ; overlap model: max(%.2f, N))\n", log_ns / fma_ns, log_ns / fma_ns);
  return 0;
}
