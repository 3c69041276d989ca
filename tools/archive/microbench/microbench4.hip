// Issue cost of v_fma_f32 by operand kind on gfx950 (design probe, not product): is a 3-VGPR-operand
// FMA (the flow kernel's z = L*P + Q - dot*R) as cheap as the 1-VGPR FMA of microbench2, and do VGPR
// banks (index mod 4) matter? 16 independent chains per lane, W waves per SIMD (grid = 256 CUs x W
// blocks of 256 threads). Prints ns per wave-instruction per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench4 tools/microbench4.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

// MODE 0: fma(a, 0.999, 1e-3) (1 VGPR); 1: fma(a, b, c) (3 VGPRs, compiler-assigned registers);
// 2: fma(a, s, c) (2 VGPRs + 1 SGPR); 3: add(a, b); 4: fma(a,b,c) asm, a/b/c in the same bank
// (v[4k], v[4k+64], v[4k+128]); 5: fma asm, a/b/c in three different banks;
// 6: mode 1 with a log every 4 fmas (trans + 3-operand mix); 7: mode 0 with a log every 4 fmas
template <int MODE>
__global__ __launch_bounds__(256) void k_fma(float* out, int iters, float seed, float s) {
  float a[16], b[16], c[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    a[k] = 1.5f + seed * (threadIdx.x + k);
    b[k] = 0.999f + seed * k;
    c[k] = 1e-3f * (1 + k);
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if constexpr (MODE == 0) {
          a[k] = __builtin_fmaf(a[k], 0.999f, 1e-3f);
          asm volatile("" : "+v"(a[k]));
        } else if constexpr (MODE == 1 || MODE == 6) {
          asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(a[k]) : "v"(a[k]), "v"(b[k]), "v"(c[k]));
        } else if constexpr (MODE == 2) {
          asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(a[k]) : "v"(a[k]), "s"(s), "v"(c[k]));
        } else if constexpr (MODE == 3) {
          asm volatile("v_add_f32 %0, %1, %2" : "=v"(a[k]) : "v"(a[k]), "v"(b[k]));
        } else if constexpr (MODE == 7) {
          asm volatile("v_fma_f32 %0, %1, 0.5, 1.0" : "=v"(a[k]) : "v"(a[k]));
        }
        if constexpr (MODE == 6 || MODE == 7) {
          if ((k & 3) == 3) {
            float t = __builtin_amdgcn_logf(a[k - 3]);
            asm volatile("" : "+v"(t));
            a[k - 3] = t;
          }
        }
      }
    }
  }
  float acc = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc += a[k] + b[k] + c[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

#define CLOB "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123"
// explicit register banks: 8 chains (twice per block), a in v[20+4k+oa], b in v[56+4k+ob], c in v[92+4k+oc]
// (<= 123 VGPRs: 4 waves per SIMD)
template <int OA, int OB, int OC>
__global__ __launch_bounds__(256) void k_bank(float* out, int iters) {
  // every register the chains touch is clobbered so the kernel allocates (and initialises) them
  asm volatile(".set .Li, 20\n.rept 104\n v_mov_b32 v[.Li], 1.0\n .set .Li, .Li+1\n.endr\n" ::: CLOB);
  for (int it = 0; it < iters; ++it) {
#define F(K) "v_fma_f32 v[" #K "*4+20+%0], v[" #K "*4+20+%0], v[" #K "*4+56+%1], v[" #K "*4+92+%2]\n"
    asm volatile(".rept 4\n" F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7) F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7)
                 ".endr\n" ::"i"(OA), "i"(OB), "i"(OC)
                 : CLOB);
#undef F
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}

int main(int argc, char** argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 4;  // waves per SIMD
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float* o;
  CK(hipMalloc(&o, (size_t)256 * 8 * 256 * 4));
  const int grid = 256 * W, blk = 256, iters = 4096;
  auto run = [&](auto launch, const char* name, double instr_per_iter) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 3; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 3;
    const double per_simd = (double)iters * instr_per_iter * W;  // wave-instructions per SIMD
    printf("W=%d %-40s %8.3f ms  ns per wave-instr per SIMD %.4f\n", W, name, ms, ms * 1e6 / per_simd);
  };
  run([&] { k_fma<0><<<grid, blk>>>(o, iters, 1e-7f, 0.999f); }, "fma 1 VGPR (inline consts)", 64);
  run([&] { k_fma<1><<<grid, blk>>>(o, iters, 1e-7f, 0.999f); }, "fma 3 VGPR (compiler regs)", 64);
  run([&] { k_fma<2><<<grid, blk>>>(o, iters, 1e-7f, 0.999f); }, "fma 2 VGPR + SGPR", 64);
  run([&] { k_fma<3><<<grid, blk>>>(o, iters, 1e-7f, 0.999f); }, "add 2 VGPR", 64);
  run([&] { k_fma<6><<<grid, blk>>>(o, iters, 1e-7f, 0.999f); }, "fma 3 VGPR + log/4 (instr count)", 80);
  run([&] { k_fma<7><<<grid, blk>>>(o, iters, 1e-7f, 0.999f); }, "fma 1 VGPR + log/4 (instr count)", 80);
  run([&] { k_bank<0, 0, 0><<<grid, blk>>>(o, iters); }, "fma 3 VGPR same bank (0,0,0)", 64);
  run([&] { k_bank<0, 1, 2><<<grid, blk>>>(o, iters); }, "fma 3 VGPR banks (0,1,2)", 64);
  run([&] { k_bank<0, 0, 1><<<grid, blk>>>(o, iters); }, "fma 3 VGPR banks (0,0,1)", 64);
  run([&] { k_bank<1, 2, 3><<<grid, blk>>>(o, iters); }, "fma 3 VGPR banks (1,2,3)", 64);
  return 0;
}
