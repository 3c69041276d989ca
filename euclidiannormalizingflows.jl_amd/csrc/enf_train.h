// enf_train.h -- training-path entry points (config 5: optimize_whitening), see include/enf.h.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "enf.h"
#include "enf_internal.h"

namespace enf {

enf_status set_error(enf_status st, const char* msg);
enf_status current_device_info(DeviceInfo* out);

enf_status negll_grad_workspace(bool f64, int64_t D, int64_t N, const enf_layer* layers, int32_t nlayers,
                                size_t* bytes);
enf_status negll_grad(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                      int32_t nlayers, void* out, void* workspace, size_t workspace_bytes, hipStream_t st);
enf_status adagrad_step(bool f64, int64_t count, void* params, void* acc, const void* grad, double grad_scale,
                        double eta, double epsilon, hipStream_t st);
enf_status householder_normalize(bool f64, int64_t D, int64_t k, void* V, int64_t ldv, hipStream_t st);

}  // namespace enf
