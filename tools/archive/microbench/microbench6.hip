#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
// per-instruction issue cost probe 2 on gfx950 (design probe, not product): 16 independent instructions
// per block, one case per kernel, W waves per SIMD. ns per wave-instruction per SIMD.
#define CLOB "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "vcc"
__global__ __launch_bounds__(256) void k0(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_fma_f32 v[20], v41, v42, v43\nv_fma_f32 v[21], v41, v42, v43\nv_fma_f32 v[22], v41, v42, v43\nv_fma_f32 v[23], v41, v42, v43\nv_fma_f32 v[24], v41, v42, v43\nv_fma_f32 v[25], v41, v42, v43\nv_fma_f32 v[26], v41, v42, v43\nv_fma_f32 v[27], v41, v42, v43\nv_fma_f32 v[28], v41, v42, v43\nv_fma_f32 v[29], v41, v42, v43\nv_fma_f32 v[30], v41, v42, v43\nv_fma_f32 v[31], v41, v42, v43\nv_fma_f32 v[32], v41, v42, v43\nv_fma_f32 v[33], v41, v42, v43\nv_fma_f32 v[34], v41, v42, v43\nv_fma_f32 v[35], v41, v42, v43\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k1(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_fma_f32 v[20], -v41, v42, v43\nv_fma_f32 v[21], -v41, v42, v43\nv_fma_f32 v[22], -v41, v42, v43\nv_fma_f32 v[23], -v41, v42, v43\nv_fma_f32 v[24], -v41, v42, v43\nv_fma_f32 v[25], -v41, v42, v43\nv_fma_f32 v[26], -v41, v42, v43\nv_fma_f32 v[27], -v41, v42, v43\nv_fma_f32 v[28], -v41, v42, v43\nv_fma_f32 v[29], -v41, v42, v43\nv_fma_f32 v[30], -v41, v42, v43\nv_fma_f32 v[31], -v41, v42, v43\nv_fma_f32 v[32], -v41, v42, v43\nv_fma_f32 v[33], -v41, v42, v43\nv_fma_f32 v[34], -v41, v42, v43\nv_fma_f32 v[35], -v41, v42, v43\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k2(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_fma_f32 v[20], v41, v45, v42\nv_fma_f32 v[21], v41, v45, v42\nv_fma_f32 v[22], v41, v45, v42\nv_fma_f32 v[23], v41, v45, v42\nv_fma_f32 v[24], v41, v45, v42\nv_fma_f32 v[25], v41, v45, v42\nv_fma_f32 v[26], v41, v45, v42\nv_fma_f32 v[27], v41, v45, v42\nv_fma_f32 v[28], v41, v45, v42\nv_fma_f32 v[29], v41, v45, v42\nv_fma_f32 v[30], v41, v45, v42\nv_fma_f32 v[31], v41, v45, v42\nv_fma_f32 v[32], v41, v45, v42\nv_fma_f32 v[33], v41, v45, v42\nv_fma_f32 v[34], v41, v45, v42\nv_fma_f32 v[35], v41, v45, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k3(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_fma_f32 v[20], v41, v42, v45\nv_fma_f32 v[21], v41, v42, v45\nv_fma_f32 v[22], v41, v42, v45\nv_fma_f32 v[23], v41, v42, v45\nv_fma_f32 v[24], v41, v42, v45\nv_fma_f32 v[25], v41, v42, v45\nv_fma_f32 v[26], v41, v42, v45\nv_fma_f32 v[27], v41, v42, v45\nv_fma_f32 v[28], v41, v42, v45\nv_fma_f32 v[29], v41, v42, v45\nv_fma_f32 v[30], v41, v42, v45\nv_fma_f32 v[31], v41, v42, v45\nv_fma_f32 v[32], v41, v42, v45\nv_fma_f32 v[33], v41, v42, v45\nv_fma_f32 v[34], v41, v42, v45\nv_fma_f32 v[35], v41, v42, v45\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k4(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_fma_f32 v[20], v42, v41, v45\nv_fma_f32 v[21], v42, v41, v45\nv_fma_f32 v[22], v42, v41, v45\nv_fma_f32 v[23], v42, v41, v45\nv_fma_f32 v[24], v42, v41, v45\nv_fma_f32 v[25], v42, v41, v45\nv_fma_f32 v[26], v42, v41, v45\nv_fma_f32 v[27], v42, v41, v45\nv_fma_f32 v[28], v42, v41, v45\nv_fma_f32 v[29], v42, v41, v45\nv_fma_f32 v[30], v42, v41, v45\nv_fma_f32 v[31], v42, v41, v45\nv_fma_f32 v[32], v42, v41, v45\nv_fma_f32 v[33], v42, v41, v45\nv_fma_f32 v[34], v42, v41, v45\nv_fma_f32 v[35], v42, v41, v45\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k5(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_fma_f32 v[20], v40, v44, v48\nv_fma_f32 v[21], v40, v44, v48\nv_fma_f32 v[22], v40, v44, v48\nv_fma_f32 v[23], v40, v44, v48\nv_fma_f32 v[24], v40, v44, v48\nv_fma_f32 v[25], v40, v44, v48\nv_fma_f32 v[26], v40, v44, v48\nv_fma_f32 v[27], v40, v44, v48\nv_fma_f32 v[28], v40, v44, v48\nv_fma_f32 v[29], v40, v44, v48\nv_fma_f32 v[30], v40, v44, v48\nv_fma_f32 v[31], v40, v44, v48\nv_fma_f32 v[32], v40, v44, v48\nv_fma_f32 v[33], v40, v44, v48\nv_fma_f32 v[34], v40, v44, v48\nv_fma_f32 v[35], v40, v44, v48\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k6(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_fmac_f32 v[21], v41, v45\nv_fmac_f32 v[25], v41, v45\nv_fmac_f32 v[29], v41, v45\nv_fmac_f32 v[33], v41, v45\nv_fmac_f32 v[21], v41, v45\nv_fmac_f32 v[25], v41, v45\nv_fmac_f32 v[29], v41, v45\nv_fmac_f32 v[33], v41, v45\nv_fmac_f32 v[21], v41, v45\nv_fmac_f32 v[25], v41, v45\nv_fmac_f32 v[29], v41, v45\nv_fmac_f32 v[33], v41, v45\nv_fmac_f32 v[21], v41, v45\nv_fmac_f32 v[25], v41, v45\nv_fmac_f32 v[29], v41, v45\nv_fmac_f32 v[33], v41, v45\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k7(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_max_f32 v[20], v41, v42\nv_max_f32 v[21], v41, v42\nv_max_f32 v[22], v41, v42\nv_max_f32 v[23], v41, v42\nv_max_f32 v[24], v41, v42\nv_max_f32 v[25], v41, v42\nv_max_f32 v[26], v41, v42\nv_max_f32 v[27], v41, v42\nv_max_f32 v[28], v41, v42\nv_max_f32 v[29], v41, v42\nv_max_f32 v[30], v41, v42\nv_max_f32 v[31], v41, v42\nv_max_f32 v[32], v41, v42\nv_max_f32 v[33], v41, v42\nv_max_f32 v[34], v41, v42\nv_max_f32 v[35], v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k8(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_min_f32 v[20], v41, v42\nv_min_f32 v[21], v41, v42\nv_min_f32 v[22], v41, v42\nv_min_f32 v[23], v41, v42\nv_min_f32 v[24], v41, v42\nv_min_f32 v[25], v41, v42\nv_min_f32 v[26], v41, v42\nv_min_f32 v[27], v41, v42\nv_min_f32 v[28], v41, v42\nv_min_f32 v[29], v41, v42\nv_min_f32 v[30], v41, v42\nv_min_f32 v[31], v41, v42\nv_min_f32 v[32], v41, v42\nv_min_f32 v[33], v41, v42\nv_min_f32 v[34], v41, v42\nv_min_f32 v[35], v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k9(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_max_f32_e64 v[20], -v41, v42\nv_max_f32_e64 v[21], -v41, v42\nv_max_f32_e64 v[22], -v41, v42\nv_max_f32_e64 v[23], -v41, v42\nv_max_f32_e64 v[24], -v41, v42\nv_max_f32_e64 v[25], -v41, v42\nv_max_f32_e64 v[26], -v41, v42\nv_max_f32_e64 v[27], -v41, v42\nv_max_f32_e64 v[28], -v41, v42\nv_max_f32_e64 v[29], -v41, v42\nv_max_f32_e64 v[30], -v41, v42\nv_max_f32_e64 v[31], -v41, v42\nv_max_f32_e64 v[32], -v41, v42\nv_max_f32_e64 v[33], -v41, v42\nv_max_f32_e64 v[34], -v41, v42\nv_max_f32_e64 v[35], -v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k10(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_sub_f32 v[20], v41, v42\nv_sub_f32 v[21], v41, v42\nv_sub_f32 v[22], v41, v42\nv_sub_f32 v[23], v41, v42\nv_sub_f32 v[24], v41, v42\nv_sub_f32 v[25], v41, v42\nv_sub_f32 v[26], v41, v42\nv_sub_f32 v[27], v41, v42\nv_sub_f32 v[28], v41, v42\nv_sub_f32 v[29], v41, v42\nv_sub_f32 v[30], v41, v42\nv_sub_f32 v[31], v41, v42\nv_sub_f32 v[32], v41, v42\nv_sub_f32 v[33], v41, v42\nv_sub_f32 v[34], v41, v42\nv_sub_f32 v[35], v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k11(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_med3_f32 v[20], v41, v42, v43\nv_med3_f32 v[21], v41, v42, v43\nv_med3_f32 v[22], v41, v42, v43\nv_med3_f32 v[23], v41, v42, v43\nv_med3_f32 v[24], v41, v42, v43\nv_med3_f32 v[25], v41, v42, v43\nv_med3_f32 v[26], v41, v42, v43\nv_med3_f32 v[27], v41, v42, v43\nv_med3_f32 v[28], v41, v42, v43\nv_med3_f32 v[29], v41, v42, v43\nv_med3_f32 v[30], v41, v42, v43\nv_med3_f32 v[31], v41, v42, v43\nv_med3_f32 v[32], v41, v42, v43\nv_med3_f32 v[33], v41, v42, v43\nv_med3_f32 v[34], v41, v42, v43\nv_med3_f32 v[35], v41, v42, v43\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k12(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_mul_f32_e64 v[20], v41, v42 mul:2\nv_mul_f32_e64 v[21], v41, v42 mul:2\nv_mul_f32_e64 v[22], v41, v42 mul:2\nv_mul_f32_e64 v[23], v41, v42 mul:2\nv_mul_f32_e64 v[24], v41, v42 mul:2\nv_mul_f32_e64 v[25], v41, v42 mul:2\nv_mul_f32_e64 v[26], v41, v42 mul:2\nv_mul_f32_e64 v[27], v41, v42 mul:2\nv_mul_f32_e64 v[28], v41, v42 mul:2\nv_mul_f32_e64 v[29], v41, v42 mul:2\nv_mul_f32_e64 v[30], v41, v42 mul:2\nv_mul_f32_e64 v[31], v41, v42 mul:2\nv_mul_f32_e64 v[32], v41, v42 mul:2\nv_mul_f32_e64 v[33], v41, v42 mul:2\nv_mul_f32_e64 v[34], v41, v42 mul:2\nv_mul_f32_e64 v[35], v41, v42 mul:2\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k13(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_xor_b32 v[20], v41, v42\nv_xor_b32 v[21], v41, v42\nv_xor_b32 v[22], v41, v42\nv_xor_b32 v[23], v41, v42\nv_xor_b32 v[24], v41, v42\nv_xor_b32 v[25], v41, v42\nv_xor_b32 v[26], v41, v42\nv_xor_b32 v[27], v41, v42\nv_xor_b32 v[28], v41, v42\nv_xor_b32 v[29], v41, v42\nv_xor_b32 v[30], v41, v42\nv_xor_b32 v[31], v41, v42\nv_xor_b32 v[32], v41, v42\nv_xor_b32 v[33], v41, v42\nv_xor_b32 v[34], v41, v42\nv_xor_b32 v[35], v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k14(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_and_b32 v[20], v41, v42\nv_and_b32 v[21], v41, v42\nv_and_b32 v[22], v41, v42\nv_and_b32 v[23], v41, v42\nv_and_b32 v[24], v41, v42\nv_and_b32 v[25], v41, v42\nv_and_b32 v[26], v41, v42\nv_and_b32 v[27], v41, v42\nv_and_b32 v[28], v41, v42\nv_and_b32 v[29], v41, v42\nv_and_b32 v[30], v41, v42\nv_and_b32 v[31], v41, v42\nv_and_b32 v[32], v41, v42\nv_and_b32 v[33], v41, v42\nv_and_b32 v[34], v41, v42\nv_and_b32 v[35], v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k15(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_mov_b32 v[20], v41\nv_mov_b32 v[21], v41\nv_mov_b32 v[22], v41\nv_mov_b32 v[23], v41\nv_mov_b32 v[24], v41\nv_mov_b32 v[25], v41\nv_mov_b32 v[26], v41\nv_mov_b32 v[27], v41\nv_mov_b32 v[28], v41\nv_mov_b32 v[29], v41\nv_mov_b32 v[30], v41\nv_mov_b32 v[31], v41\nv_mov_b32 v[32], v41\nv_mov_b32 v[33], v41\nv_mov_b32 v[34], v41\nv_mov_b32 v[35], v41\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k16(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_ldexp_f32 v[20], v41, v42\nv_ldexp_f32 v[21], v41, v42\nv_ldexp_f32 v[22], v41, v42\nv_ldexp_f32 v[23], v41, v42\nv_ldexp_f32 v[24], v41, v42\nv_ldexp_f32 v[25], v41, v42\nv_ldexp_f32 v[26], v41, v42\nv_ldexp_f32 v[27], v41, v42\nv_ldexp_f32 v[28], v41, v42\nv_ldexp_f32 v[29], v41, v42\nv_ldexp_f32 v[30], v41, v42\nv_ldexp_f32 v[31], v41, v42\nv_ldexp_f32 v[32], v41, v42\nv_ldexp_f32 v[33], v41, v42\nv_ldexp_f32 v[34], v41, v42\nv_ldexp_f32 v[35], v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k17(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_cvt_f32_i32 v[20], v41\nv_cvt_f32_i32 v[21], v41\nv_cvt_f32_i32 v[22], v41\nv_cvt_f32_i32 v[23], v41\nv_cvt_f32_i32 v[24], v41\nv_cvt_f32_i32 v[25], v41\nv_cvt_f32_i32 v[26], v41\nv_cvt_f32_i32 v[27], v41\nv_cvt_f32_i32 v[28], v41\nv_cvt_f32_i32 v[29], v41\nv_cvt_f32_i32 v[30], v41\nv_cvt_f32_i32 v[31], v41\nv_cvt_f32_i32 v[32], v41\nv_cvt_f32_i32 v[33], v41\nv_cvt_f32_i32 v[34], v41\nv_cvt_f32_i32 v[35], v41\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k18(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_add_u32 v[20], v41, v42\nv_add_u32 v[21], v41, v42\nv_add_u32 v[22], v41, v42\nv_add_u32 v[23], v41, v42\nv_add_u32 v[24], v41, v42\nv_add_u32 v[25], v41, v42\nv_add_u32 v[26], v41, v42\nv_add_u32 v[27], v41, v42\nv_add_u32 v[28], v41, v42\nv_add_u32 v[29], v41, v42\nv_add_u32 v[30], v41, v42\nv_add_u32 v[31], v41, v42\nv_add_u32 v[32], v41, v42\nv_add_u32 v[33], v41, v42\nv_add_u32 v[34], v41, v42\nv_add_u32 v[35], v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k19(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_log_f32_e64 v[20], v41 div:2\nv_log_f32_e64 v[21], v41 div:2\nv_log_f32_e64 v[22], v41 div:2\nv_log_f32_e64 v[23], v41 div:2\nv_log_f32_e64 v[24], v41 div:2\nv_log_f32_e64 v[25], v41 div:2\nv_log_f32_e64 v[26], v41 div:2\nv_log_f32_e64 v[27], v41 div:2\nv_log_f32_e64 v[28], v41 div:2\nv_log_f32_e64 v[29], v41 div:2\nv_log_f32_e64 v[30], v41 div:2\nv_log_f32_e64 v[31], v41 div:2\nv_log_f32_e64 v[32], v41 div:2\nv_log_f32_e64 v[33], v41 div:2\nv_log_f32_e64 v[34], v41 div:2\nv_log_f32_e64 v[35], v41 div:2\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k20(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_rsq_f32 v[20], v41\nv_rsq_f32 v[21], v41\nv_rsq_f32 v[22], v41\nv_rsq_f32 v[23], v41\nv_rsq_f32 v[24], v41\nv_rsq_f32 v[25], v41\nv_rsq_f32 v[26], v41\nv_rsq_f32 v[27], v41\nv_rsq_f32 v[28], v41\nv_rsq_f32 v[29], v41\nv_rsq_f32 v[30], v41\nv_rsq_f32 v[31], v41\nv_rsq_f32 v[32], v41\nv_rsq_f32 v[33], v41\nv_rsq_f32 v[34], v41\nv_rsq_f32 v[35], v41\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k21(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_exp_f32 v[20], v41\nv_exp_f32 v[21], v41\nv_exp_f32 v[22], v41\nv_exp_f32 v[23], v41\nv_exp_f32 v[24], v41\nv_exp_f32 v[25], v41\nv_exp_f32 v[26], v41\nv_exp_f32 v[27], v41\nv_exp_f32 v[28], v41\nv_exp_f32 v[29], v41\nv_exp_f32 v[30], v41\nv_exp_f32 v[31], v41\nv_exp_f32 v[32], v41\nv_exp_f32 v[33], v41\nv_exp_f32 v[34], v41\nv_exp_f32 v[35], v41\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k22(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_rcp_f32 v[20], v41\nv_rcp_f32 v[21], v41\nv_rcp_f32 v[22], v41\nv_rcp_f32 v[23], v41\nv_rcp_f32 v[24], v41\nv_rcp_f32 v[25], v41\nv_rcp_f32 v[26], v41\nv_rcp_f32 v[27], v41\nv_rcp_f32 v[28], v41\nv_rcp_f32 v[29], v41\nv_rcp_f32 v[30], v41\nv_rcp_f32 v[31], v41\nv_rcp_f32 v[32], v41\nv_rcp_f32 v[33], v41\nv_rcp_f32 v[34], v41\nv_rcp_f32 v[35], v41\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k23(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_bfi_b32 v[20], v46, v41, v42\nv_bfi_b32 v[21], v46, v41, v42\nv_bfi_b32 v[22], v46, v41, v42\nv_bfi_b32 v[23], v46, v41, v42\nv_bfi_b32 v[24], v46, v41, v42\nv_bfi_b32 v[25], v46, v41, v42\nv_bfi_b32 v[26], v46, v41, v42\nv_bfi_b32 v[27], v46, v41, v42\nv_bfi_b32 v[28], v46, v41, v42\nv_bfi_b32 v[29], v46, v41, v42\nv_bfi_b32 v[30], v46, v41, v42\nv_bfi_b32 v[31], v46, v41, v42\nv_bfi_b32 v[32], v46, v41, v42\nv_bfi_b32 v[33], v46, v41, v42\nv_bfi_b32 v[34], v46, v41, v42\nv_bfi_b32 v[35], v46, v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k24(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_cndmask_b32 v[20], v41, v42, vcc\nv_cndmask_b32 v[21], v41, v42, vcc\nv_cndmask_b32 v[22], v41, v42, vcc\nv_cndmask_b32 v[23], v41, v42, vcc\nv_cndmask_b32 v[24], v41, v42, vcc\nv_cndmask_b32 v[25], v41, v42, vcc\nv_cndmask_b32 v[26], v41, v42, vcc\nv_cndmask_b32 v[27], v41, v42, vcc\nv_cndmask_b32 v[28], v41, v42, vcc\nv_cndmask_b32 v[29], v41, v42, vcc\nv_cndmask_b32 v[30], v41, v42, vcc\nv_cndmask_b32 v[31], v41, v42, vcc\nv_cndmask_b32 v[32], v41, v42, vcc\nv_cndmask_b32 v[33], v41, v42, vcc\nv_cndmask_b32 v[34], v41, v42, vcc\nv_cndmask_b32 v[35], v41, v42, vcc\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k25(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_pk_fma_f32 v[20:21], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[22:23], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[24:25], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[26:27], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[28:29], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[30:31], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[32:33], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[34:35], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[20:21], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[22:23], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[24:25], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[26:27], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[28:29], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[30:31], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[32:33], v[42:43], v[44:45], v[46:47]\nv_pk_fma_f32 v[34:35], v[42:43], v[44:45], v[46:47]\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k26(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_pk_mul_f32 v[20:21], v[42:43], v[44:45]\nv_pk_mul_f32 v[22:23], v[42:43], v[44:45]\nv_pk_mul_f32 v[24:25], v[42:43], v[44:45]\nv_pk_mul_f32 v[26:27], v[42:43], v[44:45]\nv_pk_mul_f32 v[28:29], v[42:43], v[44:45]\nv_pk_mul_f32 v[30:31], v[42:43], v[44:45]\nv_pk_mul_f32 v[32:33], v[42:43], v[44:45]\nv_pk_mul_f32 v[34:35], v[42:43], v[44:45]\nv_pk_mul_f32 v[20:21], v[42:43], v[44:45]\nv_pk_mul_f32 v[22:23], v[42:43], v[44:45]\nv_pk_mul_f32 v[24:25], v[42:43], v[44:45]\nv_pk_mul_f32 v[26:27], v[42:43], v[44:45]\nv_pk_mul_f32 v[28:29], v[42:43], v[44:45]\nv_pk_mul_f32 v[30:31], v[42:43], v[44:45]\nv_pk_mul_f32 v[32:33], v[42:43], v[44:45]\nv_pk_mul_f32 v[34:35], v[42:43], v[44:45]\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k27(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n v_mov_b32 v46, 0x7fffffff\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_pk_add_f32 v[20:21], v[42:43], v[44:45]\nv_pk_add_f32 v[22:23], v[42:43], v[44:45]\nv_pk_add_f32 v[24:25], v[42:43], v[44:45]\nv_pk_add_f32 v[26:27], v[42:43], v[44:45]\nv_pk_add_f32 v[28:29], v[42:43], v[44:45]\nv_pk_add_f32 v[30:31], v[42:43], v[44:45]\nv_pk_add_f32 v[32:33], v[42:43], v[44:45]\nv_pk_add_f32 v[34:35], v[42:43], v[44:45]\nv_pk_add_f32 v[20:21], v[42:43], v[44:45]\nv_pk_add_f32 v[22:23], v[42:43], v[44:45]\nv_pk_add_f32 v[24:25], v[42:43], v[44:45]\nv_pk_add_f32 v[26:27], v[42:43], v[44:45]\nv_pk_add_f32 v[28:29], v[42:43], v[44:45]\nv_pk_add_f32 v[30:31], v[42:43], v[44:45]\nv_pk_add_f32 v[32:33], v[42:43], v[44:45]\nv_pk_add_f32 v[34:35], v[42:43], v[44:45]\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
int main(int argc, char** argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 4; const int iters = 4096, grid = 256 * W;
  float* o; (void)hipMalloc(&o, (size_t)grid * 256 * 4); hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); float ms;
  k0<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k0<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "fma v,v,v banks 1,2,3", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k1<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k1<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "fma -v,v,v banks 1,2,3", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k2<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k2<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "fma banks 1,1,2", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k3<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k3<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "fma banks 1,2,1 (src2)", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k4<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k4<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "fma banks 2,1,1", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k5<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k5<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "fma banks 0,0,0", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k6<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k6<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "fmac dst same bank as srcs", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k7<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k7<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "max v,v", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k8<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k8<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "min v,v", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k9<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k9<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "max -v,v", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k10<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k10<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "sub v,v", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k11<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k11<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "med3", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k12<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k12<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "mul omod*2", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k13<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k13<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "xor_b32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k14<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k14<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "and_b32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k15<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k15<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "mov_b32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k16<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k16<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "ldexp", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k17<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k17<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "cvt_f32_i32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k18<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k18<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "mul_legacy?add_u32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k19<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k19<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "log omod div:2", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k20<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k20<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "rsq", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k21<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k21<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "exp", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k22<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k22<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "rcp", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k23<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k23<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "copysign via bfi vgpr mask", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k24<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k24<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "cndmask_e32 vcc (vcc const)", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k25<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k25<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "pk_fma", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k26<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k26<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "pk_mul", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k27<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k27<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-30s ns per wave-instr per SIMD %.4f\n", W, "pk_add", ms / 3 * 1e6 / ((double)iters * 64 * W));
  return 0;
}
