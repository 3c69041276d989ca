// Test-only library (tests/test_gpu_round6.py::test_cross_lane_primitives; never part of libenf.so): the cross-lane
// sums of enf_train.h -- xor_tree over groups of P lanes, add_xor_swap<16> / <32> on gfx950's v_permlane16/32_swap
// written as inline asm with a hand-placed hazard pad -- beside the __shfl_xor butterfly they replace, for float and
// double, so the test can require them to agree bit for bit at every group size (the round-5 run-27 miscompile of
// the swap builtin gave wrong sums). Built by csrc/Makefile `xlane` (__graft_entry__.build()).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "enf_train.h"

namespace {

// out[0..63]: xor_tree(in, P); [64..127]: the __shfl_xor butterfly over P; [128..191]: add_xor_swap<16>(in);
// [192..255]: in + __shfl_xor(in, 16); [256..319]: add_xor_swap<32>(in); [320..383]: in + __shfl_xor(in, 32);
// [384..447]: lane_sum(in, D = P) (double only; float: copy of [0..63])
template <typename T>
__global__ __launch_bounds__(64) void xlane_kernel(const T* __restrict__ in, T* __restrict__ out, int P) {
  const int l = threadIdx.x;
  const T v = in[l];
  T w = v;
  for (int m = P / 2; m >= 1; m >>= 1) w += __shfl_xor(w, m);
  out[l] = enf::xor_tree(v, P);
  out[64 + l] = w;
  out[128 + l] = enf::add_xor_swap<16>(v);
  out[192 + l] = v + __shfl_xor(v, 16);
  out[256 + l] = enf::add_xor_swap<32>(v);
  out[320 + l] = v + __shfl_xor(v, 32);
  if constexpr (sizeof(T) == 8) {
    out[384 + l] = enf::lane_sum(l < P ? v : 0.0, P);
  } else {
    out[384 + l] = out[l];
  }
}

}  // namespace

// dtype 0: float, 1: double; in: 64 values, out: 448 values (device pointers); P: group size, a power of two <= 64.
// Returns 0, or the hipError_t of the launch.
extern "C" int enf_xlane_check(int dtype, int P, const void* in, void* out, void* stream) {
  if (P < 1 || P > 64 || (P & (P - 1))) return -1;
  if (dtype == 0)
    hipLaunchKernelGGL(xlane_kernel<float>, dim3(1), dim3(64), 0, (hipStream_t)stream, (const float*)in, (float*)out, P);
  else
    hipLaunchKernelGGL(xlane_kernel<double>, dim3(1), dim3(64), 0, (hipStream_t)stream, (const double*)in, (double*)out,
                       P);
  return (int)hipGetLastError();
}
