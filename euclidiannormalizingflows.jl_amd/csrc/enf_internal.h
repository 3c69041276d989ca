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
  OP_DENSE = 6,  // internal: a whole chained HouseholderTrafo as one orthogonal D x D product (MFMA)
};

constexpr int kMaxLayers = 16;  // layers per launch (kernarg table)
constexpr int kMaxSteps = 64;   // steps per launch (one per transform / per reflection)
// LDS header: per-step double scratch + the double ladj constant (padded to 16 B), then the
// per-wave ladj staging slots of the fragment kernel (4 waves x kStagePerWave values of T <= 8 B)
constexpr size_t kLdsScalars = ((kMaxSteps + 1) * sizeof(double) + 15) / 16 * 16;
constexpr int kStagePerWave = 256;
constexpr size_t kLdsHeader = kLdsScalars + 4 * kStagePerWave * sizeof(double);
constexpr size_t kLdsParamBudget = 32 * 1024;  // parameter records per launch

// ENF_NEGLL_ZYGOTE of the running training call (include/enf.h): set by the C API entry for the duration of the
// call, read when the gradient launch is planned (GradArgs::zq) -- 1: the reported loss omits ScaleShiftTrafo's ladj
extern thread_local int tl_negll_zygote;

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
  uint32_t csum;  // bounds-check build only: checksum of the tables below (flow_args_csum), else 0
  int32_t pad0_;
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
  int32_t frag;  // 1: fragment kernel (records laid out with RV = 16/elem), 0: generic kernel
  int32_t wy;  // 1: run on the dense-Householder MFMA kernel (the step table has OP_DENSE steps)
  int32_t img_off;  // dense kernel: LDS byte offset of the per-wave transpose images (set at launch)
  int32_t dk;       // padded fragment path: the power of two the kernel lays the D rows out as (0: D)
  LayerDesc layers[kMaxLayers];
  Step steps[kMaxSteps];
  int32_t desc[kMaxSteps + 1];  // per step: op | (record offset << 4); desc[nsteps] = sentinel 0
};

// Checksum of a FlowArgs from X through desc[] (FNV-1a over 32-bit words). The bounds-check build
// (ENF_BOUNDS) sets it on the host right before each launch and every block of the interpreter kernels
// recomputes it from its kernel-argument copy: a mismatch means the kernel read kernel arguments other
// than the ones launched (printed as ENF_KARG_STALE).
__host__ __device__ inline uint32_t flow_args_csum(const FlowArgs& a) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&a);
  const size_t n = (offsetof(FlowArgs, desc) + sizeof(a.desc)) / 4;
  uint32_t h = 2166136261u;
  for (size_t i = offsetof(FlowArgs, X) / 4; i < n; ++i) h = (h ^ w[i]) * 16777619u;
  return h;
}

struct DeviceInfo {
  int num_cu = 0;
};

// parameter record width (values of T per row) of a step; see enf_flow.hip
__host__ __device__ constexpr int record_width(int op) {
  return op == OP_HOUSEHOLDER ? 1 : op == OP_SCALESHIFT ? 2 : (op == OP_JOHNSON || op == OP_JOHNSON_INV) ? 4 : 8;
}
inline int record_width_host(int op) { return record_width(op); }

// The fragment (fast) kernel handles power-of-two D up to 256 (fp32) / 128 (fp64: at most 64 lanes
// per column), contiguous columns (ld == D) and 16-byte aligned X / Y; everything else runs on the
// generic kernel.
inline bool frag_path(int64_t D, int64_t ldx, int64_t ldy, const void* X, const void* Y, size_t elem) {
  const int64_t dmax = elem == 4 ? 256 : 128;
  const bool pow2 = D >= 1 && D <= dmax && (D & (D - 1)) == 0;
  return pow2 && ldx == D && ldy == D && ((((uintptr_t)X) | ((uintptr_t)Y)) & 15) == 0;
}

// Padded fragment path: D not a power of two but whole 16-byte fragments per column (D a multiple of
// 16/elem), contiguous 16-byte aligned columns, at most 256 (fp32) / 128 (fp64) rows once rounded up to
// a power of two. The kernel lays the column out as Dp = that power of two; lanes whose rows lie past
// D neither load nor store and carry neutral parameters (enf_steps.h build_program). Returns Dp, or 0.
inline int64_t frag_pad_dim(int64_t D, int64_t ldx, int64_t ldy, const void* X, const void* Y, size_t elem) {
  const int64_t dmax = elem == 4 ? 256 : 128, v = (int64_t)(16 / elem);
  if (D < v || D > dmax || (D & (D - 1)) == 0 || D % v != 0 || ldx != D || ldy != D) return 0;
  if (((((uintptr_t)X) | ((uintptr_t)Y)) & 15) != 0) return 0;
  int64_t p = 1;
  while (p < D) p <<= 1;
  return p;
}

// Values of T in one step's LDS record: W * max(D, RV) (RV = 16/elem on the fragment path, else 1),
// rounded up to 16 bytes.
inline size_t record_elems(int op, int64_t D, size_t elem, bool frag) {
  if (op == OP_DENSE) return (size_t)(D * D);  // the product's MFMA A-operand image
  const int64_t rv = frag ? (int64_t)(16 / elem) : 1;
  size_t n = (size_t)record_width(op) * (size_t)(D > rv ? D : rv);
  const size_t q = 16 / elem;
  return (n + q - 1) / q * q;
}

// Bounds-check build (`make bcheck`, a diagnostics aid, never shipped): the global tile accesses of the
// fused flow kernels check their index against the tensor's extent; a violation is printed and the
// access skipped.
#ifndef ENF_BOUNDS
#define ENF_BOUNDS 0
#endif
#if ENF_BOUNDS
#define ENF_INB(ok, what, idx, lim)                                                                   \
  ((ok) ? true                                                                                        \
        : (printf("ENF_OOB %s idx=%lld lim=%lld blk=%d thr=%d\n", what, (long long)(idx), (long long)(lim), \
                  (int)blockIdx.x, (int)threadIdx.x),                                                 \
           false))
#define ENF_KARG_CHECK(a)                                                                             \
  do {                                                                                                \
    if (threadIdx.x == 0) {                                                                           \
      const uint32_t h_ = flow_args_csum(a);                                                          \
      if (h_ != (a).csum)                                                                             \
        printf("ENF_KARG_STALE blk=%d got=%08x want=%08x N=%lld D=%d nsteps=%d\n", (int)blockIdx.x, h_, \
               (a).csum, (long long)(a).N, (a).D, (a).nsteps);                                         \
    }                                                                                                 \
  } while (0)
#else
#define ENF_INB(ok, what, idx, lim) true
#define ENF_KARG_CHECK(a) do { } while (0)
#endif

// Tuning and diagnostic knobs. The shipping library (libenf.so) is built with ENF_DIAG=0: every
// knob is its compile-time default, nothing is read from the environment and the diagnostic kernel
// variants (ENF_DEBUG_MODE: synthesized tiles / no stores) are not compiled in. The diagnostics
// build (make diag -> libenf_diag.so, tools/ only) reads them from the environment.
#ifndef ENF_DIAG
#define ENF_DIAG 0
#endif
#if ENF_DIAG
int env_int(const char* name, int dflt);
#define ENF_KNOB(name, dflt) env_int(name, dflt)
#else
#define ENF_KNOB(name, dflt) (dflt)
#endif

size_t program_lds_bytes(const FlowArgs& a, size_t elem);
bool frag_supported(const FlowArgs& a, size_t elem);
hipError_t launch_flow(const FlowArgs& a, bool f64, hipStream_t st, const DeviceInfo& dev);

// Dense-Householder MFMA kernel (enf_flow_wy.hip): a chained HouseholderTrafo with k >= wy_min_k()
// reflections runs as one D x D orthogonal product on the matrix cores, the other steps of the flow
// elementwise in the same launch. Fragment path, D in {32, 64}, fp32 or fp64.
bool wy_supported(int64_t D, bool frag);
int wy_min_k();
constexpr size_t kLdsParamBudgetWY = 64 * 1024;
hipError_t launch_wy(const FlowArgs& a, bool f64, hipStream_t st, const DeviceInfo& dev);

// JohnsonSU distribution (enf_johnsonsu.hip); prm = {gamma, delta, xi, lambda}
hipError_t launch_jsu_eval(bool f64, int fn, int64_t n, const void* x, void* out, const double (&prm)[4], hipStream_t st,
                           const DeviceInfo& dev);
hipError_t launch_jsu_sample(bool f64, int64_t n, void* out, const double (&prm)[4], uint64_t seed, uint64_t offset,
                             hipStream_t st, const DeviceInfo& dev);

// Compiled (J o H)^n program (enf_flow_hj.hip): n if the fp32 step table is H, J, H, J, ... (one
// reflection per H, Johnson forward) on the fragment path with D in {32, 64}, else 0.
int hj_program_pairs(const FlowArgs& a);  // (J o H)^n at layout D 32 / 64 / 128, padded or not
// lm: 0 no ladj, 1 write, 2 accumulate; dbg: ENF_DEBUG_MODE. hipErrorNotSupported: not a program.
hipError_t launch_hj_program(const FlowArgs& a, int lm, int dbg, hipStream_t st, const DeviceInfo& dev);
int hji_program_pairs(const FlowArgs& a);  // (J^-1, H)^n -- the inverse of (J o H)^n -- at layout D 32 / 64 / 128
hipError_t launch_hji_program(const FlowArgs& a, int lm, hipStream_t st, const DeviceInfo& dev);
// the same program in fp64 (enf_flow_hj64.hip); hipErrorNotSupported: not a program
hipError_t launch_hj64_program(const FlowArgs& a, int lm, hipStream_t st, const DeviceInfo& dev);
hipError_t launch_hji64_program(const FlowArgs& a, int lm, hipStream_t st, const DeviceInfo& dev);  // fp64 (J^-1, H)^n
// config 2 (J o H, D = 2, fp64): enf_flow_d2.hip
bool d2_program(const FlowArgs& a);
hipError_t launch_d2_program(const FlowArgs& a, int lm, hipStream_t st, const DeviceInfo& dev);

}  // namespace enf
