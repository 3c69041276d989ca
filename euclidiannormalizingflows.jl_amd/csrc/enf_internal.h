// enf_internal.h -- structures shared by the C ABI (enf_capi.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace enf {

enum : int32_t {
  OP_SCALESHIFT = 0,
  OP_CENTER_STRETCH = 1,
  OP_CENTER_CONTRACT = 2,
  OP_JOHNSON = 3,
  OP_JOHNSON_INV = 4,
  OP_HOUSEHOLDER = 5,
};

constexpr int kMaxLayers = 16;  // layers per launch (kernarg table)
constexpr int kMaxSteps = 64;   // steps per launch (one per transform / per reflection)
// LDS header: per-step double scratch + the double ladj constant, padded to 16 B
constexpr size_t kLdsHeader = ((kMaxSteps + 1) * sizeof(double) + 15) / 16 * 16;
constexpr size_t kLdsParamBudget = 32 * 1024;  // parameter records per launch

struct LayerDesc {
  int32_t op;
  int32_t k;
  const void* p[4];
};

struct Step {
  int32_t op;
  int32_t layer;  // index into FlowArgs::layers
  int32_t col;    // Householder: column of V
  int32_t off;    // offset of the step's parameter records in LDS, in elements of T
};

struct FlowArgs {
  const void* X;
  void* Y;
  void* ladj;  // nullptr: no ladj
  int64_t N;
  int64_t ldx;
  int64_t ldy;
  int32_t D;
  int32_t nsteps;
  int32_t nlayers;
  int32_t accumulate;
  LayerDesc layers[kMaxLayers];
  Step steps[kMaxSteps];
};

struct DeviceInfo {
  int num_cu = 0;
};

// parameter record width (values of T per row) of a step; see enf_flow.hip
__host__ __device__ constexpr int record_width(int op) {
  return op == OP_HOUSEHOLDER ? 1 : op == OP_SCALESHIFT ? 2 : (op == OP_JOHNSON || op == OP_JOHNSON_INV) ? 4 : 8;
}
inline int record_width_host(int op) { return record_width(op); }

size_t program_lds_bytes(const FlowArgs& a, size_t elem);
bool frag_supported(const FlowArgs& a, size_t elem);
hipError_t launch_flow(const FlowArgs& a, bool f64, hipStream_t st, const DeviceInfo& dev);

}  // namespace enf
