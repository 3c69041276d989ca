#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
// v_cndmask / VCC probe on gfx950 (design probe, not product). ns per wave-instruction per SIMD.
#define CLOB "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "vcc", "s10", "s11", "s12", "s13", "s14", "s15", "s16", "s17"
__global__ __launch_bounds__(256) void k0(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_cmp_lt_f32 vcc, v41, v42\nv_cndmask_b32 v20, v43, v44, vcc\nv_cmp_lt_f32 vcc, v41, v43\nv_cndmask_b32 v21, v43, v44, vcc\nv_cmp_lt_f32 vcc, v41, v42\nv_cndmask_b32 v22, v43, v44, vcc\nv_cmp_lt_f32 vcc, v41, v43\nv_cndmask_b32 v23, v43, v44, vcc\nv_cmp_lt_f32 vcc, v41, v42\nv_cndmask_b32 v24, v43, v44, vcc\nv_cmp_lt_f32 vcc, v41, v43\nv_cndmask_b32 v25, v43, v44, vcc\nv_cmp_lt_f32 vcc, v41, v42\nv_cndmask_b32 v26, v43, v44, vcc\nv_cmp_lt_f32 vcc, v41, v43\nv_cndmask_b32 v27, v43, v44, vcc\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k1(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_cmp_lt_f32_e64 s[10:11], v41, v42\nv_cndmask_b32_e64 v20, v43, v44, s[10:11]\nv_cmp_lt_f32_e64 s[12:13], v41, v43\nv_cndmask_b32_e64 v21, v43, v44, s[12:13]\nv_cmp_lt_f32_e64 s[14:15], v41, v42\nv_cndmask_b32_e64 v22, v43, v44, s[14:15]\nv_cmp_lt_f32_e64 s[16:17], v41, v43\nv_cndmask_b32_e64 v23, v43, v44, s[16:17]\nv_cmp_lt_f32_e64 s[10:11], v41, v42\nv_cndmask_b32_e64 v24, v43, v44, s[10:11]\nv_cmp_lt_f32_e64 s[12:13], v41, v43\nv_cndmask_b32_e64 v25, v43, v44, s[12:13]\nv_cmp_lt_f32_e64 s[14:15], v41, v42\nv_cndmask_b32_e64 v26, v43, v44, s[14:15]\nv_cmp_lt_f32_e64 s[16:17], v41, v43\nv_cndmask_b32_e64 v27, v43, v44, s[16:17]\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k2(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_cndmask_b32_e64 v20, v43, v44, vcc\nv_cndmask_b32_e64 v21, v43, v44, vcc\nv_cndmask_b32_e64 v22, v43, v44, vcc\nv_cndmask_b32_e64 v23, v43, v44, vcc\nv_cndmask_b32_e64 v24, v43, v44, vcc\nv_cndmask_b32_e64 v25, v43, v44, vcc\nv_cndmask_b32_e64 v26, v43, v44, vcc\nv_cndmask_b32_e64 v27, v43, v44, vcc\nv_cndmask_b32_e64 v28, v43, v44, vcc\nv_cndmask_b32_e64 v29, v43, v44, vcc\nv_cndmask_b32_e64 v30, v43, v44, vcc\nv_cndmask_b32_e64 v31, v43, v44, vcc\nv_cndmask_b32_e64 v32, v43, v44, vcc\nv_cndmask_b32_e64 v33, v43, v44, vcc\nv_cndmask_b32_e64 v34, v43, v44, vcc\nv_cndmask_b32_e64 v35, v43, v44, vcc\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k3(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_cndmask_b32 v20, v43, v44, vcc\nv_cndmask_b32 v21, v43, v44, vcc\nv_cndmask_b32 v22, v43, v44, vcc\nv_cndmask_b32 v23, v43, v44, vcc\nv_cndmask_b32 v24, v43, v44, vcc\nv_cndmask_b32 v25, v43, v44, vcc\nv_cndmask_b32 v26, v43, v44, vcc\nv_cndmask_b32 v27, v43, v44, vcc\nv_cndmask_b32 v28, v43, v44, vcc\nv_cndmask_b32 v29, v43, v44, vcc\nv_cndmask_b32 v30, v43, v44, vcc\nv_cndmask_b32 v31, v43, v44, vcc\nv_cndmask_b32 v32, v43, v44, vcc\nv_cndmask_b32 v33, v43, v44, vcc\nv_cndmask_b32 v34, v43, v44, vcc\nv_cndmask_b32 v35, v43, v44, vcc\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k4(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n s_mov_b64 vcc, -1\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_cndmask_b32_e64 v20, v43, v44, s[10:11]\nv_cndmask_b32_e64 v21, v43, v44, s[10:11]\nv_cndmask_b32_e64 v22, v43, v44, s[10:11]\nv_cndmask_b32_e64 v23, v43, v44, s[10:11]\nv_cndmask_b32_e64 v24, v43, v44, s[10:11]\nv_cndmask_b32_e64 v25, v43, v44, s[10:11]\nv_cndmask_b32_e64 v26, v43, v44, s[10:11]\nv_cndmask_b32_e64 v27, v43, v44, s[10:11]\nv_cndmask_b32_e64 v28, v43, v44, s[10:11]\nv_cndmask_b32_e64 v29, v43, v44, s[10:11]\nv_cndmask_b32_e64 v30, v43, v44, s[10:11]\nv_cndmask_b32_e64 v31, v43, v44, s[10:11]\nv_cndmask_b32_e64 v32, v43, v44, s[10:11]\nv_cndmask_b32_e64 v33, v43, v44, s[10:11]\nv_cndmask_b32_e64 v34, v43, v44, s[10:11]\nv_cndmask_b32_e64 v35, v43, v44, s[10:11]\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
__global__ __launch_bounds__(256) void k5(float* out, int iters) {
  asm volatile(".set .Li, 20\n.rept 44\n v_mov_b32 v[.Li], 1.5\n .set .Li, .Li+1\n.endr\n s_mov_b64 s[10:11], -1\n s_mov_b64 vcc, 0\n" ::: CLOB);
  for (int it = 0; it < iters; ++it)
    asm volatile(".rept 4\nv_cndmask_b32 v20, v43, v44, vcc\nv_cndmask_b32 v21, v43, v44, vcc\nv_cndmask_b32 v22, v43, v44, vcc\nv_cndmask_b32 v23, v43, v44, vcc\nv_cndmask_b32 v24, v43, v44, vcc\nv_cndmask_b32 v25, v43, v44, vcc\nv_cndmask_b32 v26, v43, v44, vcc\nv_cndmask_b32 v27, v43, v44, vcc\nv_cndmask_b32 v28, v43, v44, vcc\nv_cndmask_b32 v29, v43, v44, vcc\nv_cndmask_b32 v30, v43, v44, vcc\nv_cndmask_b32 v31, v43, v44, vcc\nv_cndmask_b32 v32, v43, v44, vcc\nv_cndmask_b32 v33, v43, v44, vcc\nv_cndmask_b32 v34, v43, v44, vcc\nv_cndmask_b32 v35, v43, v44, vcc\n.endr\n" ::: CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}
int main(int argc, char** argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 4; const int iters = 4096, grid = 256 * W;
  float* o; (void)hipMalloc(&o, (size_t)grid * 256 * 4); hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); float ms;
  k0<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k0<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-36s ns/instr %.4f\n", W, "cmp_e32 vcc + cndmask_e32 pairs", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k1<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k1<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-36s ns/instr %.4f\n", W, "cmp_e64 sgpr + cndmask_e64 pairs", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k2<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k2<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-36s ns/instr %.4f\n", W, "cndmask_e64 mask=vcc (set once)", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k3<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k3<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-36s ns/instr %.4f\n", W, "cndmask_e32 vcc (set once)", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k4<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k4<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-36s ns/instr %.4f\n", W, "cndmask_e64 s[10:11] (set once)", ms / 3 * 1e6 / ((double)iters * 64 * W));
  k5<<<grid, 256>>>(o, iters); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0); for (int r = 0; r < 3; ++r) k5<<<grid, 256>>>(o, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d %-36s ns/instr %.4f\n", W, "cndmask_e32 vcc, vcc=0", ms / 3 * 1e6 / ((double)iters * 64 * W));
  return 0;
}
