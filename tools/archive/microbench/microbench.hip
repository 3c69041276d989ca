// Design-probe microbenchmarks for the flow kernels on gfx950 (not product code).
// Answers, on the real MI355X:
//   1. practical HBM ceiling (coalesced float4 copy),
//   2. column-per-lane access of a column-major D x N fp32 matrix (each lane owns one
//      128-B column at D=32) vs coalesced access of the same bytes,
//   3. VALU / transcendental / packed-fp32 issue throughput with many waves,
//   4. accuracy of the hardware v_log_f32 / v_sqrt_f32 / v_rcp_f32 / v_exp_f32.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void copy_f4(const float4* __restrict__ in, float4* __restrict__ out, size_t n4) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n4; i += stride) out[i] = in[i];
}

// each lane owns one column of D=32 floats (128 B): 8 float4 loads + 8 float4 stores.
__global__ void colcopy_lane(const float4* __restrict__ in, float4* __restrict__ out, size_t ncol) {
  size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; j < ncol; j += stride) {
    float4 r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = in[j * 8 + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) out[j * 8 + k] = r[k];
  }
}

// columns of 32 floats, staged through LDS: the block loads 256 columns (32 KB) coalesced,
// each lane then reads its own column from LDS (XOR-swizzled 16-B chunks), writes back via LDS.
__global__ __launch_bounds__(256) void colcopy_lds(const float4* __restrict__ in, float4* __restrict__ out, size_t ncol) {
  __shared__ float4 tile[256 * 8];
  const int t = threadIdx.x;
  for (size_t c0 = (size_t)blockIdx.x * 256; c0 < ncol; c0 += (size_t)gridDim.x * 256) {
    const float4* src = in + c0 * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      int idx = k * 256 + t;           // linear float4 index in the tile
      int col = idx >> 3, ch = idx & 7;
      tile[col * 8 + (ch ^ (col & 7))] = src[idx];
    }
    __syncthreads();
    float4 r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = tile[t * 8 + (k ^ (t & 7))];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) tile[t * 8 + (k ^ (t & 7))] = r[k];
    __syncthreads();
    float4* dst = out + c0 * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      int idx = k * 256 + t;
      int col = idx >> 3, ch = idx & 7;
      dst[idx] = tile[col * 8 + (ch ^ (col & 7))];
    }
    __syncthreads();
  }
}

template <int OP>
__global__ void valu_tp(float* out, int iters, float seed) {
  float a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = seed + threadIdx.x * 1e-3f + k;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (OP == 0) a[k] = __builtin_fmaf(a[k], 0.999f, 1e-3f);
      if (OP == 1) a[k] = __builtin_amdgcn_logf(a[k]) + 2.0f;      // v_log_f32 + add
      if (OP == 2) a[k] = __builtin_amdgcn_sqrtf(a[k]) + 1.0f;     // v_sqrt_f32 + add
      if (OP == 3) a[k] = __builtin_amdgcn_rcpf(a[k]) + 1.0f;      // v_rcp_f32 + add
      if (OP == 4) a[k] = __builtin_amdgcn_exp2f(a[k] * 1e-3f);     // v_exp_f32 + mul
    }
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void valu_pk(float* out, int iters, float seed) {
  f2 a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { a[k].x = seed + threadIdx.x * 1e-3f + k; a[k].y = a[k].x + 0.5f; }
  const f2 m = {0.999f, 0.998f}, c = {1e-3f, 2e-3f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = __builtin_elementwise_fma(a[k], m, c);
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k].x + a[k].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void accuracy(const float* x, float* lg, float* sq, float* rc, float* ex, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    lg[i] = __builtin_amdgcn_logf(x[i]);
    sq[i] = __builtin_amdgcn_sqrtf(x[i]);
    rc[i] = __builtin_amdgcn_rcpf(x[i]);
    ex[i] = __builtin_amdgcn_exp2f(x[i] - 1.5f);
  }
}

static double ulp_of(float f) { return std::nextafter(std::fabs(f), INFINITY) - std::fabs(f); }

int main() {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const size_t ncol = 10000000, nfl = ncol * 32;
  float *a, *b;
  CK(hipMalloc(&a, nfl * 4)); CK(hipMalloc(&b, nfl * 4));
  CK(hipMemset(a, 0, nfl * 4)); CK(hipMemset(b, 0, nfl * 4));
  auto timeit = [&](auto launch, const char* name, double bytes) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipEventRecord(e0));
    const int reps = 20;
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
    printf("%-28s %9.3f us  %8.1f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
  };
  for (int grid : {2048, 4096, 8192, 40000}) {
    char nm[64]; snprintf(nm, 64, "copy_f4 grid=%d", grid);
    timeit([&] { copy_f4<<<grid, 256>>>((float4*)a, (float4*)b, nfl / 4); }, nm, 2.0 * nfl * 4);
  }
  for (int grid : {2048, 4096, 8192, 39063}) {
    char nm[64]; snprintf(nm, 64, "colcopy_lane grid=%d", grid);
    timeit([&] { colcopy_lane<<<grid, 256>>>((float4*)a, (float4*)b, ncol); }, nm, 2.0 * nfl * 4);
  }
  for (int grid : {1024, 2048, 4096, 39063}) {
    char nm[64]; snprintf(nm, 64, "colcopy_lds grid=%d", grid);
    timeit([&] { colcopy_lds<<<grid, 256>>>((float4*)a, (float4*)b, ncol); }, nm, 2.0 * nfl * 4);
  }
  // VALU throughput: 256 CUs x 8 blocks x 256 threads
  float* o; CK(hipMalloc(&o, 1 << 26));
  const int iters = 4096, grid = 256 * 16, blk = 256;
  const double lanes = (double)grid * blk;
  const char* names[5] = {"v_fma_f32", "v_log_f32+add", "v_sqrt_f32+add", "v_rcp_f32+add", "v_exp_f32+mul"};
  auto vt = [&](auto launch, const char* name, double ops) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-20s %9.3f ms  %.3e lane-ops/s\n", name, ms, ops / (ms * 1e-3));
  };
  vt([&] { valu_tp<0><<<grid, blk>>>(o, iters, 1.f); }, names[0], lanes * iters * 8);
  vt([&] { valu_tp<1><<<grid, blk>>>(o, iters, 1.f); }, names[1], lanes * iters * 8);
  vt([&] { valu_tp<2><<<grid, blk>>>(o, iters, 1.f); }, names[2], lanes * iters * 8);
  vt([&] { valu_tp<3><<<grid, blk>>>(o, iters, 1.f); }, names[3], lanes * iters * 8);
  vt([&] { valu_tp<4><<<grid, blk>>>(o, iters, 1.f); }, names[4], lanes * iters * 8);
  vt([&] { valu_pk<<<grid, blk>>>(o, iters, 1.f); }, "v_pk_fma_f32 (x2)", lanes * iters * 8 * 2);

  // accuracy sweep
  const int n = 1 << 22;
  std::vector<float> hx(n);
  for (int i = 0; i < n; ++i) {
    if (i < n / 4) hx[i] = 1.0f + (float)i / (n / 4) * 1e-3f;                     // near 1
    else if (i < n / 2) hx[i] = 1.0f + (float)(i - n / 4) / (n / 4);               // [1,2)
    else hx[i] = std::exp2f(-20.f + 60.f * (float)(i - n / 2) / (n / 2));           // wide
  }
  float *dx, *dl, *ds, *dr, *de;
  CK(hipMalloc(&dx, n * 4)); CK(hipMalloc(&dl, n * 4)); CK(hipMalloc(&ds, n * 4));
  CK(hipMalloc(&dr, n * 4)); CK(hipMalloc(&de, n * 4));
  CK(hipMemcpy(dx, hx.data(), n * 4, hipMemcpyHostToDevice));
  accuracy<<<n / 256, 256>>>(dx, dl, ds, dr, de, n);
  std::vector<float> hl(n), hs(n), hr(n), he(n);
  CK(hipMemcpy(hl.data(), dl, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hs.data(), ds, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), dr, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(he.data(), de, n * 4, hipMemcpyDeviceToHost));
  double ml[3] = {0, 0, 0}, mla[3] = {0, 0, 0}, msq = 0, mrc = 0, mex = 0;
  for (int i = 0; i < n; ++i) {
    int reg = i < n / 4 ? 0 : (i < n / 2 ? 1 : 2);
    double x = hx[i];
    double tl = std::log2(x);
    if (tl != 0) ml[reg] = std::fmax(ml[reg], std::fabs(hl[i] - tl) / ulp_of((float)tl));
    mla[reg] = std::fmax(mla[reg], std::fabs(hl[i] - tl));
    msq = std::fmax(msq, std::fabs(hs[i] - std::sqrt(x)) / ulp_of((float)std::sqrt(x)));
    mrc = std::fmax(mrc, std::fabs(hr[i] - 1.0 / x) / ulp_of((float)(1.0 / x)));
    if (x < 40) mex = std::fmax(mex, std::fabs(he[i] - std::exp2(x - 1.5)) / ulp_of((float)std::exp2(x - 1.5)));
  }
  printf("v_log_f32 max ulp: near1 %.2f  [1,2) %.2f  wide %.2f ; max abs err near1 %.3e [1,2) %.3e\n",
         ml[0], ml[1], ml[2], mla[0], mla[1]);
  printf("v_sqrt_f32 max ulp %.2f  v_rcp_f32 max ulp %.2f  v_exp_f32 max ulp %.2f\n", msq, mrc, mex);
  return 0;
}
