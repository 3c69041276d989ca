/* enf.h -- C ABI of libenf.so, the MI355X-native (gfx950) bijector hot path of
 * bat/EuclidianNormalizingFlows.jl.
 *
 * Every entry point is `extern "C"`, takes plain pointers and sizes, never throws, and returns
 * an enf_status; the message of the last failure on the calling thread is enf_last_error().
 * Compute calls are asynchronous on the given HIP stream (NULL = the default stream) and
 * never keep a pointer past the completion of the work they enqueue. The caller owns every
 * buffer. Data layout is Julia's: a batch is a column-major D x N matrix, sample j being the
 * contiguous column X[j*ldx .. j*ldx+D-1]; ladj is a length-N vector (Julia's 1 x N row).
 *
 * Reference interface replaced (bat/EuclidianNormalizingFlows.jl v0.1.0):
 *   ChangesOfVariables.with_logabsdet_jacobian(f, X) for
 *     ScaleShiftTrafo   src/scale_shift_trafo.jl:15-24
 *     CenterStretch     src/center_stretch.jl:37-43
 *     CenterContract    src/center_stretch.jl:61-67
 *     JohnsonTrafo      src/johnson_trafo.jl:74-80
 *     JohnsonTrafoInv   src/johnson_trafo.jl:99-105
 *     HouseholderTrafo  src/householder_trafo.jl:156-160 (vector and matrix V)
 *   and their Base.ComposedFunction (ChangesOfVariables 0.1: inner first, ladj_inner+ladj_outer)
 *   -> enf_flow_apply (one fused launch for the whole composition).
 *   (f)(X)  (the same call sites without ladj)                    -> enf_flow_apply, ladj = NULL.
 *   the same calls on host Arrays (config 1, no GPU)               -> enf_flow_apply_cpu
 *   InverseFunctions.inverse(f)  is host-side parameter algebra (src/scale_shift_trafo.jl:26-30,
 *   src/center_stretch.jl:45,69, src/johnson_trafo.jl:82,107, src/householder_trafo.jl:153-154)
 *   and stays in the host mirror; inverse flows run through enf_flow_apply with swapped ops.
 *   mvnormal_negll_trafo / mvnormal_negll_trafograd (src/optimize_whitening.jl:7-22)
 *                                                                -> enf_flow_negll_grad
 *   Zygote.pullback of with_logabsdet_jacobian(f, X), incl. the Householder rrules
 *     (src/householder_trafo.jl:43-54,105-124)                   -> enf_flow_vjp
 *   Optimisers.update(ADAGrad) + HouseholderTrafo functor re-normalisation
 *     (src/optimize_whitening.jl:40, src/householder_trafo.jl:134-146) -> enf_adagrad_step
 */
#ifndef ENF_H
#define ENF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ENF_VERSION_MAJOR 0
#define ENF_VERSION_MINOR 1
#define ENF_VERSION_PATCH 0

typedef enum {
  ENF_OK = 0,
  ENF_ERR_INVALID = 1,     /* bad argument (shape, null pointer, unknown op ...) */
  ENF_ERR_HIP = 2,         /* a HIP runtime call failed */
  ENF_ERR_UNSUPPORTED = 3, /* valid request the library does not implement */
  ENF_ERR_RCCL = 4         /* an RCCL call failed */
} enf_status;

typedef enum { ENF_F32 = 0, ENF_F64 = 1 } enf_dtype;
/* Flag OR'd into the dtype of the training entry points (enf_flow_negll_grad, enf_whitening_step,
 * enf_whitening_epoch, enf_whitening_step_dp): the loss they report is the one the reference RECORDS,
 * mvnormal_negll_trafo under Zygote.pullback (src/optimize_whitening.jl:18-22, 36-41), where
 * rrule(similar_fill) returns zeros as the primal (src/abstract_trafo.jl:30-33), so every ScaleShiftTrafo's
 * ladj sum(log|a|) (src/scale_shift_trafo.jl:22-23) is missing from it: the reported loss is the true negll +
 * sum log|a| at the step's parameters (the unnormalised out[0] of enf_flow_negll_grad: + N sum log|a|). The
 * gradient is unchanged (the rrule's pullback passes sum(dOmega) to the ladj value). Without the flag the
 * true negll is reported. */
#define ENF_NEGLL_ZYGOTE 0x100

/* Transform kinds; params p[0..3] are DEVICE pointers to length-D vectors of the flow's dtype
 * (a Julia scalar parameter is broadcast to length D by the host). */
typedef enum {
  ENF_OP_SCALESHIFT = 0,      /* p = {a, b}:                 y = muladd(x, a, b)            */
  ENF_OP_CENTER_STRETCH = 1,  /* p = {a, b, c}                                              */
  ENF_OP_CENTER_CONTRACT = 2, /* p = {a, b, c}                                              */
  ENF_OP_JOHNSON = 3,         /* p = {gamma, delta, xi, lambda}: y = g + d*asinh((x-xi)/l)  */
  ENF_OP_JOHNSON_INV = 4,     /* p = {gamma, delta, xi, lambda}: y = l*sinh((x-g)/d) + xi   */
  ENF_OP_HOUSEHOLDER = 5      /* p = {V}, V column-major D x k, reflections V[:,0]..V[:,k-1]
                                 applied in column order (chained_householder_trafo!)        */
} enf_op;

typedef struct {
  int32_t op;        /* enf_op */
  int32_t k;         /* HOUSEHOLDER: number of reflection columns (>= 1).
                      * SCALESHIFT: 0 = `a` is a length-D vector; 1 = `a` is a LENGTH-1 vector that the
                      * caller broadcast to the D rows p[0] points at: the ladj constant is log|a[1]|
                      * once (sum(log.(abs.(f.a))) over the length-1 vector, src/scale_shift_trafo.jl:22)
                      * and so is its gradient (1/a on row 0 only). Otherwise ignored (0). */
  const void* p[4];  /* device pointers */
} enf_layer;

/* ---------------------------------------------------------------- version / errors ---- */
/* "MAJOR.MINOR.PATCH gfx950" */
const char* enf_version(void);
/* Message of the last failing call on this thread ("" if none). */
const char* enf_last_error(void);

/* ---------------------------------------------------------------- device helpers ------ */
enf_status enf_device_count(int32_t* count);
enf_status enf_set_device(int32_t device);
enf_status enf_get_device(int32_t* device);
enf_status enf_malloc(void** ptr, size_t bytes);
enf_status enf_free(void* ptr);
/* kind: 0 host->device, 1 device->host, 2 device->device, 3 default (inferred). Async on stream. */
enf_status enf_memcpy(void* dst, const void* src, size_t bytes, int32_t kind, void* hip_stream);
enf_status enf_stream_synchronize(void* hip_stream);

/* ---------------------------------------------------------------- forward / inverse ---- */
/* Apply the composed flow layers[0], then layers[1], ... (layers[0] innermost, i.e. the
 * Julia value layers[n-1] o ... o layers[0]) to X (D x N, leading dim ldx >= D) and write
 * Y (leading dim ldy >= D). Y may alias X exactly (ldx == ldy) for an in-place transform.
 * ladj (length N) may be NULL (plain call f(X)); otherwise it receives sum over layers of the
 * per-sample log|det J|, or has it ADDED when accumulate_ladj != 0.
 * N == 0 is a no-op. Asynchronous on hip_stream. */
enf_status enf_flow_apply(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx,
                          void* Y, int64_t ldy, void* ladj, int32_t accumulate_ladj,
                          const enf_layer* layers, int32_t nlayers, void* hip_stream);

/* Host-resident batch (optimize_whitening's VectorOfSimilarVectors /
 * flatview batches, src/optimize_whitening.jl:26,38, and N beyond device memory): the same
 * computation as enf_flow_apply with X, Y and ladj in HOST memory. Column chunks of chunk_cols
 * samples (0 or more than fit: as many as fill a 32 MB slot) stream through a 3-slot device ring: host->device copy of chunk
 * i+1, the fused flow on chunk i (on hip_stream) and device->host copy of chunk i-1 overlap.
 * The caller's arrays are never page-locked: chunks pass through the ring's own pinned staging
 * slots (threaded host copies overlap the device work). Layer parameters are device
 * pointers as in enf_flow_apply. Synchronous: returns when Y and ladj are in host memory.
 * Y may alias X exactly (ldx == ldy). */
enf_status enf_flow_apply_host(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx,
                               void* Y, int64_t ldy, void* ladj, int32_t accumulate_ladj,
                               const enf_layer* layers, int32_t nlayers, int64_t chunk_cols,
                               void* hip_stream);

/* Host (CPU) execution, SURVEY.md §8 config 1 ("on CPU, no GPU"): the same flow with X, Y, ladj AND
 * the layer parameter pointers in HOST memory, computed on the host cores with the reference's
 * formulas in the data type (host libm asinh / log / exp / sinh; muladd as fma, nothing else fused),
 * per-layer ladj summed per column and combined as ChangesOfVariables combines a left-associated
 * f_n o ... o f_1: l_1 + (l_2 + (... + l_n)). nthreads <= 0: all hardware threads. Synchronous;
 * needs no GPU. Y may alias X exactly (ldx == ldy). */
enf_status enf_flow_apply_cpu(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx,
                              void* Y, int64_t ldy, void* ladj, int32_t accumulate_ladj,
                              const enf_layer* layers, int32_t nlayers, int32_t nthreads);

/* ---------------------------------------------------------------- training (config 5) -- */
/* Number of gradient entries of the flow: sum over layers of D*nparams (Householder D*k).
 * The gradient buffer layout is layer by layer, parameter by parameter, each a length-D vector
 * (Householder: the D x k matrix, column-major), in the order of enf_layer.p. */
enf_status enf_flow_param_count(int64_t D, const enf_layer* layers, int32_t nlayers,
                                int64_t* count);
/* Per-GPU UNNORMALISED sums for mvnormal_negll_trafo (src/optimize_whitening.jl:7-15) over the
 * N local samples: out[0] += sum_j [ sum_d (y_dj^2 + log 2pi)/2 - ladj_j ]  (= N * negll),
 * out[1 + i] += d(out[0]) / d(theta_i) for every flow parameter theta_i (layout above).
 * out has 1 + param_count entries and is ACCUMULATED into (zero it first). Divide by the
 * global batch size after the cross-GPU sum to obtain negll and its gradient.
 * workspace: device scratch of enf_flow_negll_grad_workspace() bytes.
 * Limits: D <= 1024. A flow beyond one gradient launch's bounds (more than 16 layers or 32 steps, or
 * parameter accumulators that do not fit the LDS, as at large D) runs as consecutive chunks of layers with
 * a checkpoint (D x N) of each chunk's input in the workspace (round 4; ENF_ERR_UNSUPPORTED only when a
 * single transform exceeds the kernel's bounds). */
enf_status enf_flow_negll_grad_workspace(enf_dtype dtype, int64_t D, int64_t N,
                                         const enf_layer* layers, int32_t nlayers,
                                         size_t* bytes);
enf_status enf_flow_negll_grad(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx,
                               const enf_layer* layers, int32_t nlayers, void* out,
                               void* workspace, size_t workspace_bytes, void* hip_stream);
/* mvnormal_negll_trafo (src/optimize_whitening.jl:7-15) without the gradient, for any flow
 * enf_flow_apply takes (no dimension / step limits): out[0] (device, dtype) += the unnormalised
 *   sum_j [ sum_d (y_dj^2 + log 2pi)/2 - ladj_j ]        (negll = out[0] / N)
 * with (Y, ladj) = with_logabsdet_jacobian(flow, X), reduced on the device in double in a fixed order
 * (deterministic). workspace: device scratch of enf_flow_negll_workspace() bytes (holds Y, ladj and
 * the partial sums). Asynchronous on hip_stream. */
enf_status enf_flow_negll_workspace(enf_dtype dtype, int64_t D, int64_t N, size_t* bytes);
enf_status enf_flow_negll(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx,
                          const enf_layer* layers, int32_t nlayers, void* out, void* workspace,
                          size_t workspace_bytes, void* hip_stream);
/* Vector-Jacobian product of (Y, ladj) = with_logabsdet_jacobian(flow, X) (the Zygote pullback the
 * reference's rrules build: householder_trafo_pullback_x / chained_householder_trafo_pullback_x,
 * src/householder_trafo.jl:43-54,105-124, and broadcast AD of the elementwise maps). Given the
 * cotangents dY (D x N, leading dim lddy) and dladj (length N; NULL = zero), writes
 *   dX[:, j] = J_j' dY[:, j] + dladj[j] * grad_x ladj_j          (D x N, leading dim lddx)
 * for every sample j (J_j = dY[:, j]/dX[:, j]). dX may alias dY exactly (lddx == lddy), not X.
 * When dparams != NULL it also ACCUMULATES the parameter VJP summed over the samples into dparams
 * (enf_flow_param_count entries, the layout of enf_flow_negll_grad's out[1:]); workspace is then
 * required (enf_flow_negll_grad_workspace bytes), otherwise it may be NULL -- except for a chunked flow
 * (enf_flow_negll_grad), which always needs it (its checkpoints). The accurate library arithmetic of
 * enf_flow_negll_grad's generic kernel; limits as enf_flow_negll_grad. */
enf_status enf_flow_vjp(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx, const void* dY,
                        int64_t lddy, const void* dladj, const enf_layer* layers, int32_t nlayers, void* dX,
                        int64_t lddx, void* dparams, void* workspace, size_t workspace_bytes,
                        void* hip_stream);
/* In-place ADAGrad step of Optimisers.jl 0.2 (eta, epsilon) over `count` parameters:
 * acc += g.^2; theta -= eta * g ./ (sqrt.(acc) .+ epsilon), with g = grad * grad_scale.
 * params/acc/grad are device arrays of the dtype. */
enf_status enf_adagrad_step(enf_dtype dtype, int64_t count, void* params, void* acc,
                            const void* grad, double grad_scale, double eta, double epsilon,
                            void* hip_stream);
/* One single-GPU optimize_whitening minibatch step, fused (src/optimize_whitening.jl:36-42):
 * the negll and gradient of the N samples X (as enf_flow_negll_grad; the layer parameter pointers
 * point into theta), then *loss_out = negll / N (device double), ADAGrad (eta, epsilon) with
 * g = gradient / N on the nruns ranges [runs[2i], runs[2i+1]) of theta, and the re-normalisation
 * of the nhb Householder column batches (hbatches[3i..3i+2] = offset in theta, column count, column
 * stride; every column must start at a multiple of D in theta, as the parameter layout puts it). Identical
 * arithmetic to enf_flow_negll_grad + enf_adagrad_step per range + enf_householder_normalize_strided per batch
 * on one rank, in two launches (round 5: the gradient kernel, then one reduction launch in which every
 * parameter vector is summed over the gradient blocks, projected, updated and re-normalised by a block of its
 * own). Multi-GPU training: enf_whitening_step_dp (or enf_flow_negll_grad, the all-reduce, enf_whitening_apply). */
enf_status enf_whitening_step(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx,
                              const enf_layer* layers, int32_t nlayers, void* theta, void* acc,
                              const int64_t* runs, int32_t nruns, const int64_t* hbatches, int32_t nhb,
                              double eta, double epsilon, double* loss_out, void* workspace,
                              size_t workspace_bytes, void* hip_stream);
/* The single-GPU optimize_whitening steps of ONE EPOCH (src/optimize_whitening.jl:31-42: the minibatches
 * Iterators.partition(1:N, batchsize) in order, each an enf_whitening_step): step j covers columns
 * [j*batchsize, min((j+1)*batchsize, N)) of X and writes its loss to loss_out[j] (device, ceil(N/batchsize) doubles).
 * Identical arithmetic to that sequence of enf_whitening_step calls, bit for bit. Round 5: while a minibatch fits the
 * one-launch step (a batch of one gradient block, e.g. the reference examples' B = 100 / 1000 at D <= 2), the whole
 * epoch is ONE launch -- one block walks the minibatches, no launch per step; other flows and batch sizes run the
 * per-step path. workspace: enf_flow_negll_grad_workspace(batchsize) bytes. */
enf_status enf_whitening_epoch(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx, int64_t batchsize,
                               const enf_layer* layers, int32_t nlayers, void* theta, void* acc,
                               const int64_t* runs, int32_t nruns, const int64_t* hbatches, int32_t nhb,
                               double eta, double epsilon, double* loss_out, void* workspace,
                               size_t workspace_bytes, void* hip_stream);
/* The update half of a DATA-PARALLEL optimize_whitening minibatch step (src/optimize_whitening.jl:38-41),
 * run on every rank after the cross-GPU sum (enf_allreduce_sum / RCCL) of enf_flow_negll_grad's out
 * buffer g (1 + nparams values of the dtype, nparams = enf_flow_param_count): *loss_out = g[0] / B
 * (device double; B = global batch size), ADAGrad (eta, epsilon) with gradient g[1 + i] / B on the
 * nruns ranges [runs[2i], runs[2i+1]) of theta, and the re-normalisation of the nhb Householder column
 * batches, in one launch. Identical arithmetic to g[0] / B + enf_adagrad_step per range +
 * enf_householder_normalize_strided per batch; every rank applies the same update (no broadcast). */
enf_status enf_whitening_apply(enf_dtype dtype, int64_t D, int64_t nparams, const void* g, int64_t B,
                               void* theta, void* acc, const int64_t* runs, int32_t nruns,
                               const int64_t* hbatches, int32_t nhb, double eta, double epsilon,
                               double* loss_out, void* hip_stream);
/* HouseholderTrafo functor reconstruction (src/householder_trafo.jl:134-146): normalise each of
 * the k columns of the D x k device matrix V to unit 2-norm, in place. */
enf_status enf_householder_normalize(enf_dtype dtype, int64_t D, int64_t k, void* V,
                                     void* hip_stream);
/* The same for k columns at a column stride ldv >= D (column j at V + j*ldv): every
 * HouseholderTrafo vector of a flow's flat parameter vector in one launch. */
enf_status enf_householder_normalize_strided(enf_dtype dtype, int64_t D, int64_t k, void* V, int64_t ldv,
                                             void* hip_stream);

/* Measurement helper, not a reference operation: a hand-written streaming copy of `bytes` from src to dst
 * (16-byte aligned device buffers) -- the practical HBM ceiling bench.py reports the flow kernels against
 * (SURVEY.md §8(d)). variant: 0 = 4 x 16-byte fragments per lane per iteration, nontemporal; 1 = the same,
 * plain loads / stores; 2 = 8 fragments, nontemporal; 3 = one fragment per lane, one pass. */
enf_status enf_stream_copy(const void* src, void* dst, int64_t bytes, int32_t variant, void* hip_stream);

/* ------------------------------------------------------- JohnsonSU distribution -------- */
/* JohnsonSU(gamma, delta, xi, lambda) (src/johnson_trafo.jl:1-26) evaluated elementwise over n
 * device values of the dtype, out[i] = fn(x[i]) (out may equal x), with the reference's formulas
 * (src/johnson_trafo.jl:120-129):
 *   PDF      deriv_johnsontrafo(x) * pdf(Normal(), johnsontrafo(x))          (:120)
 *   LOGPDF   log of the same product                                         (:123)
 *   CDF      cdf(Normal(), johnsontrafo(x))                                  (:121)
 *   LOGCDF   logcdf(Normal(), johnsontrafo(x))                               (:124)
 *   CCDF     1 - cdf;  LOGCCDF  log(1 - cdf)                                 (:125-126)
 *   QUANTILE johnsontrafo_inv(quantile(Normal(), x)), x = probability       (:129)
 * Parameters are passed as doubles and rounded to the dtype. */
typedef enum {
  ENF_JSU_PDF = 0,
  ENF_JSU_LOGPDF = 1,
  ENF_JSU_CDF = 2,
  ENF_JSU_LOGCDF = 3,
  ENF_JSU_CCDF = 4,
  ENF_JSU_LOGCCDF = 5,
  ENF_JSU_QUANTILE = 6
} enf_jsu_fn;
enf_status enf_johnsonsu_eval(enf_dtype dtype, int32_t fn, int64_t n, const void* x, void* out,
                              double gamma, double delta, double xi, double lambda, void* hip_stream);
/* rand(JohnsonSU(...), n) (Distributions' inverse-CDF fallback through quantile, exercised by
 * test/test_johnson_trafo.jl:12-14): out[i] = quantile(u_i), u_i uniform on (0, 1) from
 * Philox4x32-10 with key = seed and counter = offset + i/4 (fp32: the four 32-bit words of a call
 * give samples 4c..4c+3) or offset + i/2 (fp64: two 64-bit draws per call). */
enf_status enf_johnsonsu_sample(enf_dtype dtype, int64_t n, void* out, double gamma, double delta,
                                double xi, double lambda, uint64_t seed, uint64_t offset,
                                void* hip_stream);

/* ---------------------------------------------------------------- RCCL ---------------- */
/* Opaque communicator for the gradient all-reduce (one rank per GPU, one process each). */
typedef struct enf_comm_s* enf_comm;
#define ENF_UNIQUE_ID_BYTES 128
/* Rank 0 creates the id and ships it to the other ranks out of band. */
enf_status enf_comm_unique_id(uint8_t id[ENF_UNIQUE_ID_BYTES]);
enf_status enf_comm_init(enf_comm* comm, int32_t nranks, const uint8_t id[ENF_UNIQUE_ID_BYTES],
                         int32_t rank);
enf_status enf_comm_destroy(enf_comm comm);
/* In-place sum all-reduce of `count` dtype elements over the communicator. */
enf_status enf_allreduce_sum(enf_comm comm, void* buf, int64_t count, enf_dtype dtype,
                             void* hip_stream);

/* One rank's DATA-PARALLEL optimize_whitening minibatch step in one call (round 4; src/optimize_whitening.jl:36-42):
 * the loss / gradient sums of this rank's N columns X (its share of a minibatch of B columns in all; N may be 0),
 * the cross-rank sum over `comm` (RCCL on hip_stream, of this rank's 1 + nparams double totals -- before any
 * rounding to the dtype; NULL comm: one rank, no all-reduce), then *loss_out = negll (sum / B), ADAGrad on the
 * runs with gradient / B and the Householder re-normalisation, as enf_whitening_step. Replaces
 * enf_flow_negll_grad + enf_allreduce_sum + enf_whitening_apply (and the zeroing of their buffer) with gradient +
 * totals + all-reduce + one update launch; on one rank (comm NULL or a 1-rank communicator, B = N) identical to
 * enf_whitening_step. A flow beyond one gradient launch's bounds (the chunked path of enf_flow_negll_grad) sums
 * each rank's gradient in the dtype before the all-reduce (its chunks accumulate into a buffer of T). Round 6: on the
 * fused fp32 (J o H)^n path with more than one rank (or N < B) the all-reduce carries the gradient kernel's partial
 * rows (every rank launches the grid of ceil(B / ranks) columns; about 5 KB per row at D = 32, 4 pairs) and the
 * update launch sums them -- no reduction launch in between -- while those rows total at most 64 KiB (larger
 * payloads are reduced to one row first: a ring all-reduce of R rows costs more than the launch it saves).
 * Results are the same bit for bit either way. workspace: enf_flow_negll_grad_workspace of
 * max(N, ceil(B / ranks)) columns (the global batch B always suffices). Every rank must call it with the same B,
 * runs and batches. */
enf_status enf_whitening_step_dp(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx,
                                 const enf_layer* layers, int32_t nlayers, void* theta, void* acc, const int64_t* runs,
                                 int32_t nruns, const int64_t* hbatches, int32_t nhb, double eta, double epsilon,
                                 int64_t B, double* loss_out, enf_comm comm, void* workspace, size_t workspace_bytes,
                                 void* hip_stream);


#ifdef __cplusplus
}
#endif
#endif /* ENF_H */
