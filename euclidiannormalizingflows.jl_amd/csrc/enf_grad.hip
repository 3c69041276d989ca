// enf_grad.hip -- fused forward + backward of the whitening loss (config 5), see include/enf.h
// enf_flow_negll_grad. (Implementation follows.)
#include <hip/hip_runtime.h>

#include "enf_train.h"

namespace enf {

enf_status negll_grad_workspace(bool f64, int64_t D, int64_t N, const enf_layer* layers, int32_t nlayers,
                                size_t* bytes) {
  (void)f64; (void)D; (void)N; (void)layers; (void)nlayers;
  *bytes = 0;
  return ENF_OK;
}

enf_status negll_grad(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                      int32_t nlayers, void* out, void* workspace, size_t workspace_bytes, hipStream_t st) {
  (void)f64; (void)D; (void)N; (void)X; (void)ldx; (void)layers; (void)nlayers; (void)out;
  (void)workspace; (void)workspace_bytes; (void)st;
  return set_error(ENF_ERR_UNSUPPORTED, "enf_flow_negll_grad: not implemented yet");
}

}  // namespace enf
