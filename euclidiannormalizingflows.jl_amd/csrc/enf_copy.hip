// enf_copy.hip -- a hand-written streaming device copy: the practical HBM ceiling the flow kernels are measured
// against ("also measure a device copy kernel"; VERDICT r04 item 2: torch's copy_ reached
// 4.6 TB/s on the box where the MI355X guide's float4 copy reaches 6.29 TB/s, so a ratio to torch's copy
// overstated the kernels). Not a reference operation: bench.py times it under the same settle protocol as the
// headline and reports the best variant as roofline.copy_ceiling_GBps.
//
// Each lane moves UNR 16-byte fragments per iteration (global_load_dwordx4, all loads issued before the
// stores), the waves striding over the buffer in whole 1-KiB wave-instructions; NT: nontemporal loads and
// stores (the streaming hint the flow kernels use for X and Y).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "enf_frag.h"
#include "enf_train.h"

namespace enf {

namespace {

template <int UNR, bool NT>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n16) {
  const int64_t lanes = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t i = tid;
  for (; i + (UNR - 1) * lanes < n16; i += UNR * lanes) {
    u32x4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * lanes) : src[i + u * lanes];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], dst + i + u * lanes);
      else dst[i + u * lanes] = v[u];
    }
  }
  for (; i < n16; i += lanes) dst[i] = NT ? __builtin_nontemporal_load(src + i) : src[i];
}

__global__ void copy_tail_kernel(const unsigned char* __restrict__ src, unsigned char* __restrict__ dst, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

}  // namespace

// variant: 0 = 4 fragments per lane per iteration, nontemporal; 1 = the same with plain loads / stores;
// 2 = 8 fragments, nontemporal; 3 = one fragment, nontemporal, one pass (a lane per fragment)
enf_status stream_copy(const void* src, void* dst, int64_t bytes, int32_t variant, hipStream_t st) {
  if (bytes <= 0) return ENF_OK;
  if ((((uintptr_t)src) & 15) != 0 || (((uintptr_t)dst) & 15) != 0)
    return set_error(ENF_ERR_INVALID, "enf_stream_copy: src and dst must be 16-byte aligned");
  DeviceInfo dev;
  if (current_device_info(&dev) != ENF_OK) return ENF_ERR_HIP;
  const int64_t n16 = bytes / 16;
  const u32x4* s = (const u32x4*)src;
  u32x4* d = (u32x4*)dst;
  const unsigned persistent = (unsigned)dev.num_cu * 8;  // 8 blocks of 4 waves per CU: every wave slot
  if (n16 > 0) {
    switch (variant) {
      case 0: hipLaunchKernelGGL((copy_kernel<4, true>), dim3(persistent), dim3(256), 0, st, s, d, n16); break;
      case 1: hipLaunchKernelGGL((copy_kernel<4, false>), dim3(persistent), dim3(256), 0, st, s, d, n16); break;
      case 2: hipLaunchKernelGGL((copy_kernel<8, true>), dim3(persistent), dim3(256), 0, st, s, d, n16); break;
      case 3: {
        const int64_t blocks = (n16 + 255) / 256;
        if (blocks > 0x7fffffff) return set_error(ENF_ERR_UNSUPPORTED, "enf_stream_copy: buffer too large for variant 3");
        hipLaunchKernelGGL((copy_kernel<1, true>), dim3((unsigned)blocks), dim3(256), 0, st, s, d, n16);
        break;
      }
      default: return set_error(ENF_ERR_INVALID, "enf_stream_copy: variant must be 0..3");
    }
  }
  const int64_t rest = bytes - n16 * 16;
  if (rest > 0)
    hipLaunchKernelGGL(copy_tail_kernel, dim3(1), dim3(16), 0, st, (const unsigned char*)src + n16 * 16,
                       (unsigned char*)dst + n16 * 16, rest);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? ENF_OK : set_error(ENF_ERR_HIP, hipGetErrorString(e));
}

}  // namespace enf
