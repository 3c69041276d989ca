#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
// transcendental / FMA mixing probe on gfx950 (design probe, not product): 32-instruction blocks,
// one pattern per kernel, W waves per SIMD. ns per wave-instruction per SIMD and per block.
#define CLOB "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"
__global__ __launch_bounds__(256) void k0(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_log_f32 v20, v61\nv_log_f32 v21, v61\nv_log_f32 v22, v61\nv_log_f32 v23, v61\nv_log_f32 v24, v61\nv_log_f32 v25, v61\nv_log_f32 v26, v61\nv_log_f32 v27, v61\nv_log_f32 v28, v61\nv_log_f32 v29, v61\nv_log_f32 v30, v61\nv_log_f32 v31, v61\nv_log_f32 v32, v61\nv_log_f32 v33, v61\nv_log_f32 v34, v61\nv_log_f32 v35, v61\nv_log_f32 v36, v61\nv_log_f32 v37, v61\nv_log_f32 v38, v61\nv_log_f32 v39, v61\nv_log_f32 v40, v61\nv_log_f32 v41, v61\nv_log_f32 v42, v61\nv_log_f32 v43, v61\nv_log_f32 v44, v61\nv_log_f32 v45, v61\nv_log_f32 v46, v61\nv_log_f32 v47, v61\nv_log_f32 v48, v61\nv_log_f32 v49, v61\nv_log_f32 v50, v61\nv_log_f32 v51, v61\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k1(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_fma_f32 v20, v61, v62, v63\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_fma_f32 v24, v61, v62, v63\nv_fma_f32 v25, v61, v62, v63\nv_fma_f32 v26, v61, v62, v63\nv_fma_f32 v27, v61, v62, v63\nv_fma_f32 v28, v61, v62, v63\nv_fma_f32 v29, v61, v62, v63\nv_fma_f32 v30, v61, v62, v63\nv_fma_f32 v31, v61, v62, v63\nv_fma_f32 v32, v61, v62, v63\nv_fma_f32 v33, v61, v62, v63\nv_fma_f32 v34, v61, v62, v63\nv_fma_f32 v35, v61, v62, v63\nv_fma_f32 v36, v61, v62, v63\nv_fma_f32 v37, v61, v62, v63\nv_fma_f32 v38, v61, v62, v63\nv_fma_f32 v39, v61, v62, v63\nv_fma_f32 v40, v61, v62, v63\nv_fma_f32 v41, v61, v62, v63\nv_fma_f32 v42, v61, v62, v63\nv_fma_f32 v43, v61, v62, v63\nv_fma_f32 v44, v61, v62, v63\nv_fma_f32 v45, v61, v62, v63\nv_fma_f32 v46, v61, v62, v63\nv_fma_f32 v47, v61, v62, v63\nv_fma_f32 v48, v61, v62, v63\nv_fma_f32 v49, v61, v62, v63\nv_fma_f32 v50, v61, v62, v63\nv_fma_f32 v51, v61, v62, v63\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k2(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_fma_f32 v24, v61, v62, v63\nv_fma_f32 v25, v61, v62, v63\nv_fma_f32 v26, v61, v62, v63\nv_fma_f32 v27, v61, v62, v63\nv_log_f32 v28, v61\nv_fma_f32 v29, v61, v62, v63\nv_fma_f32 v30, v61, v62, v63\nv_fma_f32 v31, v61, v62, v63\nv_fma_f32 v32, v61, v62, v63\nv_fma_f32 v33, v61, v62, v63\nv_fma_f32 v34, v61, v62, v63\nv_fma_f32 v35, v61, v62, v63\nv_log_f32 v36, v61\nv_fma_f32 v37, v61, v62, v63\nv_fma_f32 v38, v61, v62, v63\nv_fma_f32 v39, v61, v62, v63\nv_fma_f32 v40, v61, v62, v63\nv_fma_f32 v41, v61, v62, v63\nv_fma_f32 v42, v61, v62, v63\nv_fma_f32 v43, v61, v62, v63\nv_log_f32 v44, v61\nv_fma_f32 v45, v61, v62, v63\nv_fma_f32 v46, v61, v62, v63\nv_fma_f32 v47, v61, v62, v63\nv_fma_f32 v48, v61, v62, v63\nv_fma_f32 v49, v61, v62, v63\nv_fma_f32 v50, v61, v62, v63\nv_fma_f32 v51, v61, v62, v63\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k3(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_log_f32 v20, v61\nv_log_f32 v21, v61\nv_log_f32 v22, v61\nv_log_f32 v23, v61\nv_fma_f32 v24, v61, v62, v63\nv_fma_f32 v25, v61, v62, v63\nv_fma_f32 v26, v61, v62, v63\nv_fma_f32 v27, v61, v62, v63\nv_fma_f32 v28, v61, v62, v63\nv_fma_f32 v29, v61, v62, v63\nv_fma_f32 v30, v61, v62, v63\nv_fma_f32 v31, v61, v62, v63\nv_fma_f32 v32, v61, v62, v63\nv_fma_f32 v33, v61, v62, v63\nv_fma_f32 v34, v61, v62, v63\nv_fma_f32 v35, v61, v62, v63\nv_fma_f32 v36, v61, v62, v63\nv_fma_f32 v37, v61, v62, v63\nv_fma_f32 v38, v61, v62, v63\nv_fma_f32 v39, v61, v62, v63\nv_fma_f32 v40, v61, v62, v63\nv_fma_f32 v41, v61, v62, v63\nv_fma_f32 v42, v61, v62, v63\nv_fma_f32 v43, v61, v62, v63\nv_fma_f32 v44, v61, v62, v63\nv_fma_f32 v45, v61, v62, v63\nv_fma_f32 v46, v61, v62, v63\nv_fma_f32 v47, v61, v62, v63\nv_fma_f32 v48, v61, v62, v63\nv_fma_f32 v49, v61, v62, v63\nv_fma_f32 v50, v61, v62, v63\nv_fma_f32 v51, v61, v62, v63\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k4(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v24, v61\nv_fma_f32 v25, v61, v62, v63\nv_fma_f32 v26, v61, v62, v63\nv_fma_f32 v27, v61, v62, v63\nv_log_f32 v28, v61\nv_fma_f32 v29, v61, v62, v63\nv_fma_f32 v30, v61, v62, v63\nv_fma_f32 v31, v61, v62, v63\nv_log_f32 v32, v61\nv_fma_f32 v33, v61, v62, v63\nv_fma_f32 v34, v61, v62, v63\nv_fma_f32 v35, v61, v62, v63\nv_log_f32 v36, v61\nv_fma_f32 v37, v61, v62, v63\nv_fma_f32 v38, v61, v62, v63\nv_fma_f32 v39, v61, v62, v63\nv_log_f32 v40, v61\nv_fma_f32 v41, v61, v62, v63\nv_fma_f32 v42, v61, v62, v63\nv_fma_f32 v43, v61, v62, v63\nv_log_f32 v44, v61\nv_fma_f32 v45, v61, v62, v63\nv_fma_f32 v46, v61, v62, v63\nv_fma_f32 v47, v61, v62, v63\nv_log_f32 v48, v61\nv_fma_f32 v49, v61, v62, v63\nv_fma_f32 v50, v61, v62, v63\nv_fma_f32 v51, v61, v62, v63\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k5(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_log_f32 v20, v61\nv_log_f32 v21, v61\nv_log_f32 v22, v61\nv_log_f32 v23, v61\nv_log_f32 v24, v61\nv_log_f32 v25, v61\nv_log_f32 v26, v61\nv_log_f32 v27, v61\nv_fma_f32 v28, v61, v62, v63\nv_fma_f32 v29, v61, v62, v63\nv_fma_f32 v30, v61, v62, v63\nv_fma_f32 v31, v61, v62, v63\nv_fma_f32 v32, v61, v62, v63\nv_fma_f32 v33, v61, v62, v63\nv_fma_f32 v34, v61, v62, v63\nv_fma_f32 v35, v61, v62, v63\nv_fma_f32 v36, v61, v62, v63\nv_fma_f32 v37, v61, v62, v63\nv_fma_f32 v38, v61, v62, v63\nv_fma_f32 v39, v61, v62, v63\nv_fma_f32 v40, v61, v62, v63\nv_fma_f32 v41, v61, v62, v63\nv_fma_f32 v42, v61, v62, v63\nv_fma_f32 v43, v61, v62, v63\nv_fma_f32 v44, v61, v62, v63\nv_fma_f32 v45, v61, v62, v63\nv_fma_f32 v46, v61, v62, v63\nv_fma_f32 v47, v61, v62, v63\nv_fma_f32 v48, v61, v62, v63\nv_fma_f32 v49, v61, v62, v63\nv_fma_f32 v50, v61, v62, v63\nv_fma_f32 v51, v61, v62, v63\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k6(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_log_f32 v22, v61\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v24, v61\nv_fma_f32 v25, v61, v62, v63\nv_log_f32 v26, v61\nv_fma_f32 v27, v61, v62, v63\nv_log_f32 v28, v61\nv_fma_f32 v29, v61, v62, v63\nv_log_f32 v30, v61\nv_fma_f32 v31, v61, v62, v63\nv_log_f32 v32, v61\nv_fma_f32 v33, v61, v62, v63\nv_log_f32 v34, v61\nv_fma_f32 v35, v61, v62, v63\nv_log_f32 v36, v61\nv_fma_f32 v37, v61, v62, v63\nv_log_f32 v38, v61\nv_fma_f32 v39, v61, v62, v63\nv_log_f32 v40, v61\nv_fma_f32 v41, v61, v62, v63\nv_log_f32 v42, v61\nv_fma_f32 v43, v61, v62, v63\nv_log_f32 v44, v61\nv_fma_f32 v45, v61, v62, v63\nv_log_f32 v46, v61\nv_fma_f32 v47, v61, v62, v63\nv_log_f32 v48, v61\nv_fma_f32 v49, v61, v62, v63\nv_log_f32 v50, v61\nv_fma_f32 v51, v61, v62, v63\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k7(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_log_f32 v20, v61\nv_log_f32 v21, v61\nv_log_f32 v22, v61\nv_log_f32 v23, v61\nv_log_f32 v24, v61\nv_log_f32 v25, v61\nv_log_f32 v26, v61\nv_log_f32 v27, v61\nv_log_f32 v28, v61\nv_log_f32 v29, v61\nv_log_f32 v30, v61\nv_log_f32 v31, v61\nv_log_f32 v32, v61\nv_log_f32 v33, v61\nv_log_f32 v34, v61\nv_log_f32 v35, v61\nv_fma_f32 v36, v61, v62, v63\nv_fma_f32 v37, v61, v62, v63\nv_fma_f32 v38, v61, v62, v63\nv_fma_f32 v39, v61, v62, v63\nv_fma_f32 v40, v61, v62, v63\nv_fma_f32 v41, v61, v62, v63\nv_fma_f32 v42, v61, v62, v63\nv_fma_f32 v43, v61, v62, v63\nv_fma_f32 v44, v61, v62, v63\nv_fma_f32 v45, v61, v62, v63\nv_fma_f32 v46, v61, v62, v63\nv_fma_f32 v47, v61, v62, v63\nv_fma_f32 v48, v61, v62, v63\nv_fma_f32 v49, v61, v62, v63\nv_fma_f32 v50, v61, v62, v63\nv_fma_f32 v51, v61, v62, v63\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k8(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_log_f32 v20, v61\nv_fma_f32 v21, v20, v62, v63\nv_fma_f32 v22, v20, v62, v63\nv_fma_f32 v23, v20, v62, v63\nv_log_f32 v24, v61\nv_fma_f32 v25, v24, v62, v63\nv_fma_f32 v26, v24, v62, v63\nv_fma_f32 v27, v24, v62, v63\nv_log_f32 v28, v61\nv_fma_f32 v29, v28, v62, v63\nv_fma_f32 v30, v28, v62, v63\nv_fma_f32 v31, v28, v62, v63\nv_log_f32 v32, v61\nv_fma_f32 v33, v32, v62, v63\nv_fma_f32 v34, v32, v62, v63\nv_fma_f32 v35, v32, v62, v63\nv_log_f32 v36, v61\nv_fma_f32 v37, v36, v62, v63\nv_fma_f32 v38, v36, v62, v63\nv_fma_f32 v39, v36, v62, v63\nv_log_f32 v40, v61\nv_fma_f32 v41, v40, v62, v63\nv_fma_f32 v42, v40, v62, v63\nv_fma_f32 v43, v40, v62, v63\nv_log_f32 v44, v61\nv_fma_f32 v45, v44, v62, v63\nv_fma_f32 v46, v44, v62, v63\nv_fma_f32 v47, v44, v62, v63\nv_log_f32 v48, v61\nv_fma_f32 v49, v48, v62, v63\nv_fma_f32 v50, v48, v62, v63\nv_fma_f32 v51, v48, v62, v63\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k9(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v24, v61\nv_fma_f32 v25, v61, v62, v63\nv_fma_f32 v26, v61, v62, v63\nv_fma_f32 v27, v61, v62, v63\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v24, v61\nv_fma_f32 v25, v61, v62, v63\nv_fma_f32 v26, v61, v62, v63\nv_fma_f32 v27, v61, v62, v63\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v24, v61\nv_fma_f32 v25, v61, v62, v63\nv_fma_f32 v26, v61, v62, v63\nv_fma_f32 v27, v61, v62, v63\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v24, v61\nv_fma_f32 v25, v61, v62, v63\nv_fma_f32 v26, v61, v62, v63\nv_fma_f32 v27, v61, v62, v63\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k10(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_log_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k11(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_fma_f32 v20, v61, v62, v63\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_fma_f32 v20, v61, v62, v63\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_fma_f32 v20, v61, v62, v63\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_fma_f32 v20, v61, v62, v63\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_fma_f32 v20, v61, v62, v63\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_fma_f32 v20, v61, v62, v63\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_fma_f32 v20, v61, v62, v63\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_fma_f32 v20, v61, v62, v63\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k12(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_log_f32 v20, v61\nv_log_f32 v21, v61\nv_log_f32 v22, v61\nv_log_f32 v23, v61\nv_log_f32 v20, v61\nv_log_f32 v21, v61\nv_log_f32 v22, v61\nv_log_f32 v23, v61\nv_log_f32 v20, v61\nv_log_f32 v21, v61\nv_log_f32 v22, v61\nv_log_f32 v23, v61\nv_log_f32 v20, v61\nv_log_f32 v21, v61\nv_log_f32 v22, v61\nv_log_f32 v23, v61\nv_log_f32 v20, v61\nv_log_f32 v21, v61\nv_log_f32 v22, v61\nv_log_f32 v23, v61\nv_log_f32 v20, v61\nv_log_f32 v21, v61\nv_log_f32 v22, v61\nv_log_f32 v23, v61\nv_log_f32 v20, v61\nv_log_f32 v21, v61\nv_log_f32 v22, v61\nv_log_f32 v23, v61\nv_log_f32 v20, v61\nv_log_f32 v21, v61\nv_log_f32 v22, v61\nv_log_f32 v23, v61\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k13(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 2\nv_sqrt_f32 v20, v61\nv_fma_f32 v21, v61, v62, v63\nv_fma_f32 v22, v61, v62, v63\nv_fma_f32 v23, v61, v62, v63\nv_sqrt_f32 v24, v61\nv_fma_f32 v25, v61, v62, v63\nv_fma_f32 v26, v61, v62, v63\nv_fma_f32 v27, v61, v62, v63\nv_sqrt_f32 v28, v61\nv_fma_f32 v29, v61, v62, v63\nv_fma_f32 v30, v61, v62, v63\nv_fma_f32 v31, v61, v62, v63\nv_sqrt_f32 v32, v61\nv_fma_f32 v33, v61, v62, v63\nv_fma_f32 v34, v61, v62, v63\nv_fma_f32 v35, v61, v62, v63\nv_sqrt_f32 v36, v61\nv_fma_f32 v37, v61, v62, v63\nv_fma_f32 v38, v61, v62, v63\nv_fma_f32 v39, v61, v62, v63\nv_sqrt_f32 v40, v61\nv_fma_f32 v41, v61, v62, v63\nv_fma_f32 v42, v61, v62, v63\nv_fma_f32 v43, v61, v62, v63\nv_sqrt_f32 v44, v61\nv_fma_f32 v45, v61, v62, v63\nv_fma_f32 v46, v61, v62, v63\nv_fma_f32 v47, v61, v62, v63\nv_sqrt_f32 v48, v61\nv_fma_f32 v49, v61, v62, v63\nv_fma_f32 v50, v61, v62, v63\nv_fma_f32 v51, v61, v62, v63\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
int main(int argc, char** argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 4; const int iters = 4096, grid = 256 * W;
  float* o; (void)hipMalloc(&o, (size_t)grid * 256 * 4); hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); float ms;
  k0<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k0<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "32 log", ns, ns * 32); }
  k1<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k1<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "32 fma", ns, ns * 32); }
  k2<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k2<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "4 log spread + 28 fma", ns, ns * 32); }
  k3<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k3<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "4 log grouped + 28 fma", ns, ns * 32); }
  k4<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k4<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "8 log spread (1:3)", ns, ns * 32); }
  k5<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k5<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "8 log grouped + 24 fma", ns, ns * 32); }
  k6<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k6<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "16 log alternating", ns, ns * 32); }
  k7<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k7<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "16 log grouped + 16 fma", ns, ns * 32); }
  k8<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k8<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "8 log spread RAW next", ns, ns * 32); }
  k9<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k9<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "8 log spread WAW dist 8", ns, ns * 32); }
  k10<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k10<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "8 log spread WAW dist 4", ns, ns * 32); }
  k11<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k11<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "32 fma WAW dist 4", ns, ns * 32); }
  k12<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k12<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "32 log WAW dist 4", ns, ns * 32); }
  k13<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k13<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  { double ns = ms / 3 * 1e6 / ((double)iters * 64 * W); printf("W=%d %-28s ns/instr %.4f  ns per 32-block %.2f\n", W, "8 sqrt spread (1:3)", ns, ns * 32); }
  return 0;
}
