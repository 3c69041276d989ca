#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
// per-instruction issue cost probe 3 on gfx950 (design probe, not product): 16 independent instructions
// per block, one case per kernel, W waves per SIMD. ns per wave-instruction per SIMD.
#define CLOB "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "vcc", "s10", "s11"
__global__ __launch_bounds__(256) void k0(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_max_u32 v[20], v41, v42\nv_max_u32 v[21], v41, v42\nv_max_u32 v[22], v41, v42\nv_max_u32 v[23], v41, v42\nv_max_u32 v[24], v41, v42\nv_max_u32 v[25], v41, v42\nv_max_u32 v[26], v41, v42\nv_max_u32 v[27], v41, v42\nv_max_u32 v[28], v41, v42\nv_max_u32 v[29], v41, v42\nv_max_u32 v[30], v41, v42\nv_max_u32 v[31], v41, v42\nv_max_u32 v[32], v41, v42\nv_max_u32 v[33], v41, v42\nv_max_u32 v[34], v41, v42\nv_max_u32 v[35], v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k1(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_min_u32 v[20], v41, v42\nv_min_u32 v[21], v41, v42\nv_min_u32 v[22], v41, v42\nv_min_u32 v[23], v41, v42\nv_min_u32 v[24], v41, v42\nv_min_u32 v[25], v41, v42\nv_min_u32 v[26], v41, v42\nv_min_u32 v[27], v41, v42\nv_min_u32 v[28], v41, v42\nv_min_u32 v[29], v41, v42\nv_min_u32 v[30], v41, v42\nv_min_u32 v[31], v41, v42\nv_min_u32 v[32], v41, v42\nv_min_u32 v[33], v41, v42\nv_min_u32 v[34], v41, v42\nv_min_u32 v[35], v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k2(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_max_i32 v[20], v41, v42\nv_max_i32 v[21], v41, v42\nv_max_i32 v[22], v41, v42\nv_max_i32 v[23], v41, v42\nv_max_i32 v[24], v41, v42\nv_max_i32 v[25], v41, v42\nv_max_i32 v[26], v41, v42\nv_max_i32 v[27], v41, v42\nv_max_i32 v[28], v41, v42\nv_max_i32 v[29], v41, v42\nv_max_i32 v[30], v41, v42\nv_max_i32 v[31], v41, v42\nv_max_i32 v[32], v41, v42\nv_max_i32 v[33], v41, v42\nv_max_i32 v[34], v41, v42\nv_max_i32 v[35], v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k3(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_or_b32 v[20], v41, v42\nv_or_b32 v[21], v41, v42\nv_or_b32 v[22], v41, v42\nv_or_b32 v[23], v41, v42\nv_or_b32 v[24], v41, v42\nv_or_b32 v[25], v41, v42\nv_or_b32 v[26], v41, v42\nv_or_b32 v[27], v41, v42\nv_or_b32 v[28], v41, v42\nv_or_b32 v[29], v41, v42\nv_or_b32 v[30], v41, v42\nv_or_b32 v[31], v41, v42\nv_or_b32 v[32], v41, v42\nv_or_b32 v[33], v41, v42\nv_or_b32 v[34], v41, v42\nv_or_b32 v[35], v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k4(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_and_b32 v[20], 0x80000000, v41\nv_and_b32 v[21], 0x80000000, v41\nv_and_b32 v[22], 0x80000000, v41\nv_and_b32 v[23], 0x80000000, v41\nv_and_b32 v[24], 0x80000000, v41\nv_and_b32 v[25], 0x80000000, v41\nv_and_b32 v[26], 0x80000000, v41\nv_and_b32 v[27], 0x80000000, v41\nv_and_b32 v[28], 0x80000000, v41\nv_and_b32 v[29], 0x80000000, v41\nv_and_b32 v[30], 0x80000000, v41\nv_and_b32 v[31], 0x80000000, v41\nv_and_b32 v[32], 0x80000000, v41\nv_and_b32 v[33], 0x80000000, v41\nv_and_b32 v[34], 0x80000000, v41\nv_and_b32 v[35], 0x80000000, v41\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k5(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_or3_b32 v[20], v41, v42, v43\nv_or3_b32 v[21], v41, v42, v43\nv_or3_b32 v[22], v41, v42, v43\nv_or3_b32 v[23], v41, v42, v43\nv_or3_b32 v[24], v41, v42, v43\nv_or3_b32 v[25], v41, v42, v43\nv_or3_b32 v[26], v41, v42, v43\nv_or3_b32 v[27], v41, v42, v43\nv_or3_b32 v[28], v41, v42, v43\nv_or3_b32 v[29], v41, v42, v43\nv_or3_b32 v[30], v41, v42, v43\nv_or3_b32 v[31], v41, v42, v43\nv_or3_b32 v[32], v41, v42, v43\nv_or3_b32 v[33], v41, v42, v43\nv_or3_b32 v[34], v41, v42, v43\nv_or3_b32 v[35], v41, v42, v43\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k6(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_and_or_b32 v[20], v41, v42, v43\nv_and_or_b32 v[21], v41, v42, v43\nv_and_or_b32 v[22], v41, v42, v43\nv_and_or_b32 v[23], v41, v42, v43\nv_and_or_b32 v[24], v41, v42, v43\nv_and_or_b32 v[25], v41, v42, v43\nv_and_or_b32 v[26], v41, v42, v43\nv_and_or_b32 v[27], v41, v42, v43\nv_and_or_b32 v[28], v41, v42, v43\nv_and_or_b32 v[29], v41, v42, v43\nv_and_or_b32 v[30], v41, v42, v43\nv_and_or_b32 v[31], v41, v42, v43\nv_and_or_b32 v[32], v41, v42, v43\nv_and_or_b32 v[33], v41, v42, v43\nv_and_or_b32 v[34], v41, v42, v43\nv_and_or_b32 v[35], v41, v42, v43\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k7(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_ashrrev_i32 v[20], 31, v41\nv_ashrrev_i32 v[21], 31, v41\nv_ashrrev_i32 v[22], 31, v41\nv_ashrrev_i32 v[23], 31, v41\nv_ashrrev_i32 v[24], 31, v41\nv_ashrrev_i32 v[25], 31, v41\nv_ashrrev_i32 v[26], 31, v41\nv_ashrrev_i32 v[27], 31, v41\nv_ashrrev_i32 v[28], 31, v41\nv_ashrrev_i32 v[29], 31, v41\nv_ashrrev_i32 v[30], 31, v41\nv_ashrrev_i32 v[31], 31, v41\nv_ashrrev_i32 v[32], 31, v41\nv_ashrrev_i32 v[33], 31, v41\nv_ashrrev_i32 v[34], 31, v41\nv_ashrrev_i32 v[35], 31, v41\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k8(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_lshlrev_b32 v[20], 1, v41\nv_lshlrev_b32 v[21], 1, v41\nv_lshlrev_b32 v[22], 1, v41\nv_lshlrev_b32 v[23], 1, v41\nv_lshlrev_b32 v[24], 1, v41\nv_lshlrev_b32 v[25], 1, v41\nv_lshlrev_b32 v[26], 1, v41\nv_lshlrev_b32 v[27], 1, v41\nv_lshlrev_b32 v[28], 1, v41\nv_lshlrev_b32 v[29], 1, v41\nv_lshlrev_b32 v[30], 1, v41\nv_lshlrev_b32 v[31], 1, v41\nv_lshlrev_b32 v[32], 1, v41\nv_lshlrev_b32 v[33], 1, v41\nv_lshlrev_b32 v[34], 1, v41\nv_lshlrev_b32 v[35], 1, v41\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k9(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_sub_u32 v[20], v41, v42\nv_sub_u32 v[21], v41, v42\nv_sub_u32 v[22], v41, v42\nv_sub_u32 v[23], v41, v42\nv_sub_u32 v[24], v41, v42\nv_sub_u32 v[25], v41, v42\nv_sub_u32 v[26], v41, v42\nv_sub_u32 v[27], v41, v42\nv_sub_u32 v[28], v41, v42\nv_sub_u32 v[29], v41, v42\nv_sub_u32 v[30], v41, v42\nv_sub_u32 v[31], v41, v42\nv_sub_u32 v[32], v41, v42\nv_sub_u32 v[33], v41, v42\nv_sub_u32 v[34], v41, v42\nv_sub_u32 v[35], v41, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k10(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_sub_f32_e64 v[20], 2.0, v41 clamp\nv_sub_f32_e64 v[21], 2.0, v41 clamp\nv_sub_f32_e64 v[22], 2.0, v41 clamp\nv_sub_f32_e64 v[23], 2.0, v41 clamp\nv_sub_f32_e64 v[24], 2.0, v41 clamp\nv_sub_f32_e64 v[25], 2.0, v41 clamp\nv_sub_f32_e64 v[26], 2.0, v41 clamp\nv_sub_f32_e64 v[27], 2.0, v41 clamp\nv_sub_f32_e64 v[28], 2.0, v41 clamp\nv_sub_f32_e64 v[29], 2.0, v41 clamp\nv_sub_f32_e64 v[30], 2.0, v41 clamp\nv_sub_f32_e64 v[31], 2.0, v41 clamp\nv_sub_f32_e64 v[32], 2.0, v41 clamp\nv_sub_f32_e64 v[33], 2.0, v41 clamp\nv_sub_f32_e64 v[34], 2.0, v41 clamp\nv_sub_f32_e64 v[35], 2.0, v41 clamp\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k11(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_fma_f32 v[20], |v41|, v42, 1.0\nv_fma_f32 v[21], |v41|, v42, 1.0\nv_fma_f32 v[22], |v41|, v42, 1.0\nv_fma_f32 v[23], |v41|, v42, 1.0\nv_fma_f32 v[24], |v41|, v42, 1.0\nv_fma_f32 v[25], |v41|, v42, 1.0\nv_fma_f32 v[26], |v41|, v42, 1.0\nv_fma_f32 v[27], |v41|, v42, 1.0\nv_fma_f32 v[28], |v41|, v42, 1.0\nv_fma_f32 v[29], |v41|, v42, 1.0\nv_fma_f32 v[30], |v41|, v42, 1.0\nv_fma_f32 v[31], |v41|, v42, 1.0\nv_fma_f32 v[32], |v41|, v42, 1.0\nv_fma_f32 v[33], |v41|, v42, 1.0\nv_fma_f32 v[34], |v41|, v42, 1.0\nv_fma_f32 v[35], |v41|, v42, 1.0\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k12(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_mul_f32_e64 v[20], |v41|, v42\nv_mul_f32_e64 v[21], |v41|, v42\nv_mul_f32_e64 v[22], |v41|, v42\nv_mul_f32_e64 v[23], |v41|, v42\nv_mul_f32_e64 v[24], |v41|, v42\nv_mul_f32_e64 v[25], |v41|, v42\nv_mul_f32_e64 v[26], |v41|, v42\nv_mul_f32_e64 v[27], |v41|, v42\nv_mul_f32_e64 v[28], |v41|, v42\nv_mul_f32_e64 v[29], |v41|, v42\nv_mul_f32_e64 v[30], |v41|, v42\nv_mul_f32_e64 v[31], |v41|, v42\nv_mul_f32_e64 v[32], |v41|, v42\nv_mul_f32_e64 v[33], |v41|, v42\nv_mul_f32_e64 v[34], |v41|, v42\nv_mul_f32_e64 v[35], |v41|, v42\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k13(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_xad_u32 v[20], v41, v42, v43\nv_xad_u32 v[21], v41, v42, v43\nv_xad_u32 v[22], v41, v42, v43\nv_xad_u32 v[23], v41, v42, v43\nv_xad_u32 v[24], v41, v42, v43\nv_xad_u32 v[25], v41, v42, v43\nv_xad_u32 v[26], v41, v42, v43\nv_xad_u32 v[27], v41, v42, v43\nv_xad_u32 v[28], v41, v42, v43\nv_xad_u32 v[29], v41, v42, v43\nv_xad_u32 v[30], v41, v42, v43\nv_xad_u32 v[31], v41, v42, v43\nv_xad_u32 v[32], v41, v42, v43\nv_xad_u32 v[33], v41, v42, v43\nv_xad_u32 v[34], v41, v42, v43\nv_xad_u32 v[35], v41, v42, v43\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k14(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_cndmask_b32_e64 v[20], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[21], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[22], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[23], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[24], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[25], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[26], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[27], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[28], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[29], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[30], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[31], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[32], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[33], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[34], 0, 1.0, s[10:11]\nv_cndmask_b32_e64 v[35], 0, 1.0, s[10:11]\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k15(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_fma_f32 v[20], -v40, v44, v48\nv_fma_f32 v[21], -v40, v44, v48\nv_fma_f32 v[22], -v40, v44, v48\nv_fma_f32 v[23], -v40, v44, v48\nv_fma_f32 v[24], -v40, v44, v48\nv_fma_f32 v[25], -v40, v44, v48\nv_fma_f32 v[26], -v40, v44, v48\nv_fma_f32 v[27], -v40, v44, v48\nv_fma_f32 v[28], -v40, v44, v48\nv_fma_f32 v[29], -v40, v44, v48\nv_fma_f32 v[30], -v40, v44, v48\nv_fma_f32 v[31], -v40, v44, v48\nv_fma_f32 v[32], -v40, v44, v48\nv_fma_f32 v[33], -v40, v44, v48\nv_fma_f32 v[34], -v40, v44, v48\nv_fma_f32 v[35], -v40, v44, v48\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k16(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_fmac_f32 v[20], v41, v45\nv_fmac_f32 v[21], v41, v45\nv_fmac_f32 v[22], v41, v45\nv_fmac_f32 v[23], v41, v45\nv_fmac_f32 v[24], v41, v45\nv_fmac_f32 v[25], v41, v45\nv_fmac_f32 v[26], v41, v45\nv_fmac_f32 v[27], v41, v45\nv_fmac_f32 v[28], v41, v45\nv_fmac_f32 v[29], v41, v45\nv_fmac_f32 v[30], v41, v45\nv_fmac_f32 v[31], v41, v45\nv_fmac_f32 v[32], v41, v45\nv_fmac_f32 v[33], v41, v45\nv_fmac_f32 v[34], v41, v45\nv_fmac_f32 v[35], v41, v45\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k17(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_add_f32 v[20], v41, v45\nv_add_f32 v[21], v41, v45\nv_add_f32 v[22], v41, v45\nv_add_f32 v[23], v41, v45\nv_add_f32 v[24], v41, v45\nv_add_f32 v[25], v41, v45\nv_add_f32 v[26], v41, v45\nv_add_f32 v[27], v41, v45\nv_add_f32 v[28], v41, v45\nv_add_f32 v[29], v41, v45\nv_add_f32 v[30], v41, v45\nv_add_f32 v[31], v41, v45\nv_add_f32 v[32], v41, v45\nv_add_f32 v[33], v41, v45\nv_add_f32 v[34], v41, v45\nv_add_f32 v[35], v41, v45\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k18(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_mul_f32 v[20], v41, v45\nv_mul_f32 v[21], v41, v45\nv_mul_f32 v[22], v41, v45\nv_mul_f32 v[23], v41, v45\nv_mul_f32 v[24], v41, v45\nv_mul_f32 v[25], v41, v45\nv_mul_f32 v[26], v41, v45\nv_mul_f32 v[27], v41, v45\nv_mul_f32 v[28], v41, v45\nv_mul_f32 v[29], v41, v45\nv_mul_f32 v[30], v41, v45\nv_mul_f32 v[31], v41, v45\nv_mul_f32 v[32], v41, v45\nv_mul_f32 v[33], v41, v45\nv_mul_f32 v[34], v41, v45\nv_mul_f32 v[35], v41, v45\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k19(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_fma_f32 v[20], v41, v42, v43\nv_mul_f32 v[21], v41, v42\nv_add_f32_e64 v[22], |v41|, v42\nv_fma_f32 v[23], v41, v41, 1.0\nv_fmac_f32 v[24], v42, v43\nv_log_f32 v[25], v41\nv_fma_f32 v[26], v41, v42, v43\nv_mul_f32 v[27], v41, v42\nv_add_f32_e64 v[28], |v41|, v42\nv_fma_f32 v[29], v41, v41, 1.0\nv_fmac_f32 v[30], v42, v43\nv_log_f32 v[31], v41\nv_add_f32_e64 v[32], |v41|, v42\nv_fma_f32 v[33], v41, v41, 1.0\nv_fmac_f32 v[34], v42, v43\nv_fma_f32 v[35], v41, v42, v43\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
int main(int argc, char** argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 4; const int iters = 4096, grid = 256 * W;
  float* o; (void)hipMalloc(&o, (size_t)grid * 256 * 4); hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); float ms;
  k0<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k0<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "max_u32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k1<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k1<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "min_u32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k2<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k2<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "max_i32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k3<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k3<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "or_b32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k4<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k4<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "and_b32 literal", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k5<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k5<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "or3_b32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k6<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k6<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "and_or_b32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k7<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k7<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "ashrrev_i32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k8<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k8<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "lshlrev_b32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k9<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k9<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "sub_u32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k10<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k10<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "sub_f32 clamp", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k11<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k11<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "fma 1 vgpr abs", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k12<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k12<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "mul |v|,v", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k13<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k13<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "xad_u32", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k14<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k14<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "cndmask_e64 inline consts", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k15<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k15<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "fma banks 0,0,0 with one src neg", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k16<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k16<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "fmac 2 same + dst other", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k17<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k17<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "add_f32 v,v same bank", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k18<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k18<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "mul v,v same bank", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k19<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k19<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-34s ns per wave-instr per SIMD %.4f\n", W, "mixed: mul,fma,log x (5:1)", ms / 3 * 1e6 / ((double)iters * 64 * W));
  return 0;
}
