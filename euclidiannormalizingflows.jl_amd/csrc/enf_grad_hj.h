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
  double* partial;  // [nblocks][1 + nparams]: block 1 + b writes row b (block 0 computes the constant below)
  double* ctot_out;  // the flow's constant ladj sum_p sum_d log|delta/lambda| (double), written by block 0
  int32_t nparams;
  int32_t pad_;
  const float* v[kHJGradMaxPairs];
  const float* g[kHJGradMaxPairs];
  const float* d[kHJGradMaxPairs];
  const float* xi[kHJGradMaxPairs];
  const float* lam[kHJGradMaxPairs];
  int32_t goffH[kHJGradMaxPairs];  // gradient offset of pair p's reflection vector
  int32_t goffJ[kHJGradMaxPairs];  // gradient offset of pair p's gamma (delta, xi, lambda follow)
  // nullable (the data-parallel rows path): block 0 also writes the row {-N ctot, 0, ..., 0} here, so that the
  // partial rows alone sum to the loss and gradient (no reduction launch before the cross-rank sum of the rows)
  double* ctot_row;
};

// fp32, D in {32, 64}, contiguous 16-byte aligned columns, layers H, J, H, J, ... (k = 1), <= 8 pairs
bool hj_grad_eligible(int64_t D, int64_t ldx, const void* X, const enf_layer* layers, int32_t nlayers);
// the flow's shape alone (no pointer / stride test): what the workspace query can know
bool hj_grad_shape_ok(int64_t D, const enf_layer* layers, int32_t nlayers);
// partial rows the fused kernel writes for N columns (the workspace holds at least this many)
int hj_grad_blocks(int64_t D, int64_t N, int32_t npairs);
// the exact number of partial rows a launch planned for Nplan columns writes (without a ctot row)
int hj_grad_launch_rows(int64_t D, int64_t Nplan, int32_t npairs);
// Launches the fused kernel (grid: 1 + *nblocks blocks); the loss partials EXCLUDE the constant ladj, which
// block 0 writes to *ctot_out (the reduction subtracts N * ctot from the loss once). Nplan > 0: the kernel shape
// and grid of a batch of Nplan columns (every rank of a data-parallel step launches the same grid, so their rows
// add element by element); ctot_row: block 0 also writes the row {-N ctot, 0...} after the blocks' rows and
// *nblocks counts it.
hipError_t launch_hj_grad(int64_t D, int64_t N, const void* X, const enf_layer* layers, int32_t nlayers,
                          int32_t nparams, double* partial, double* ctot_out, int* nblocks, hipStream_t st,
                          int64_t Nplan = 0, bool ctot_row = false);

}  // namespace enf
