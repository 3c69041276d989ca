// enf_grad_hj.h -- fused negll forward + backward for (J o H)^n fp32 flows (enf_grad_hj.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "enf.h"
#include "enf_internal.h"

namespace enf {

constexpr int kHJGradMaxPairs = 8;

struct HJGradArgs {
  const float* X;
  int64_t N;
  int32_t n;  // pairs
  int32_t D;
  double* partial;  // [gridDim.x][1 + nparams]
  int32_t nparams;
  int32_t pad_;
  const float* v[kHJGradMaxPairs];
  const float* g[kHJGradMaxPairs];
  const float* d[kHJGradMaxPairs];
  const float* xi[kHJGradMaxPairs];
  const float* lam[kHJGradMaxPairs];
  int32_t goffH[kHJGradMaxPairs];  // gradient offset of pair p's reflection vector
  int32_t goffJ[kHJGradMaxPairs];  // gradient offset of pair p's gamma (delta, xi, lambda follow)
};

// fp32, D in {32, 64}, contiguous 16-byte aligned columns, layers H, J, H, J, ... (k = 1), <= 8 pairs
bool hj_grad_eligible(int64_t D, int64_t ldx, const void* X, const enf_layer* layers, int32_t nlayers);
hipError_t launch_hj_grad(int64_t D, int64_t N, const void* X, const enf_layer* layers, int32_t nlayers,
                          int32_t nparams, double* partial, int blocks, hipStream_t st);

}  // namespace enf
