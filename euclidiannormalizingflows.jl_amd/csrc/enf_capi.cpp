// enf_capi.cpp -- the C ABI of libenf.so (include/enf.h): argument validation, flattening of a
// composed flow into launch-sized step programs, device bookkeeping, error reporting, RCCL.
// No C++ exception crosses the ABI: every entry point catches everything.
#include "enf.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "enf_internal.h"
#include "enf_train.h"

namespace {

thread_local std::string g_last_error;

enf_status fail(enf_status st, const std::string& msg) {
  g_last_error = msg;
  return st;
}

enf_status hip_fail(hipError_t e, const char* what) {
  return fail(ENF_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define ENF_TRY try {
#define ENF_CATCH                                                   \
  }                                                                 \
  catch (const std::exception& ex) {                                \
    return fail(ENF_ERR_INVALID, std::string("exception: ") + ex.what()); \
  }                                                                 \
  catch (...) {                                                     \
    return fail(ENF_ERR_INVALID, "unknown exception");              \
  }

std::mutex g_dev_mu;
std::vector<enf::DeviceInfo> g_dev;

enf_status device_info(enf::DeviceInfo* out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  std::lock_guard<std::mutex> lk(g_dev_mu);
  if ((int)g_dev.size() <= dev) g_dev.resize(dev + 1);
  if (g_dev[dev].num_cu == 0) {
    int n = 0;
    e = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return hip_fail(e, "hipDeviceGetAttribute");
    g_dev[dev].num_cu = n > 0 ? n : 1;
  }
  *out = g_dev[dev];
  return ENF_OK;
}

int nparams_of(int op) {
  switch (op) {
    case ENF_OP_SCALESHIFT: return 2;
    case ENF_OP_CENTER_STRETCH:
    case ENF_OP_CENTER_CONTRACT: return 3;
    case ENF_OP_JOHNSON:
    case ENF_OP_JOHNSON_INV: return 4;
    case ENF_OP_HOUSEHOLDER: return 1;
    default: return -1;
  }
}

enf_status validate_layers(int64_t D, const enf_layer* layers, int32_t nlayers) {
  if (nlayers < 0) return fail(ENF_ERR_INVALID, "nlayers < 0");
  if (nlayers > 0 && !layers) return fail(ENF_ERR_INVALID, "layers is NULL");
  for (int32_t l = 0; l < nlayers; ++l) {
    const int np = nparams_of(layers[l].op);
    if (np < 0) return fail(ENF_ERR_INVALID, "layer " + std::to_string(l) + ": unknown op " + std::to_string(layers[l].op));
    if (layers[l].op == ENF_OP_HOUSEHOLDER && layers[l].k < 1)
      return fail(ENF_ERR_INVALID, "layer " + std::to_string(l) + ": HouseholderTrafo needs k >= 1 columns");
    if (layers[l].op == ENF_OP_SCALESHIFT && layers[l].k != 0 && layers[l].k != 1)
      return fail(ENF_ERR_INVALID, "layer " + std::to_string(l) + ": ScaleShiftTrafo k must be 0 (length-D a) or 1 (length-1 a)");
    if (D > 0)
      for (int q = 0; q < np; ++q)
        if (!layers[l].p[q])
          return fail(ENF_ERR_INVALID, "layer " + std::to_string(l) + ": parameter " + std::to_string(q) + " is NULL");
  }
  return ENF_OK;
}

}  // namespace

namespace enf {
// enf_cpu.cpp (host-only translation unit)
int usable_cpus();
enf_status flow_apply_cpu(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, void* Y, int64_t ldy,
                          void* ladj, int32_t accumulate, const enf_layer* layers, int32_t nlayers, int32_t nthreads);
// shared with enf_train.hip
enf_status set_error(enf_status st, const char* msg) { return fail(st, msg); }
thread_local int tl_negll_zygote = 0;
enf_status current_device_info(DeviceInfo* out) { return device_info(out); }
}  // namespace enf

namespace {
// ENF_NEGLL_ZYGOTE (include/enf.h) of a training entry point: stripped from the dtype, held for the call
struct ZygoteScope {
  explicit ZygoteScope(enf_dtype& dtype) {
    enf::tl_negll_zygote = ((int)dtype & ENF_NEGLL_ZYGOTE) ? 1 : 0;
    dtype = (enf_dtype)((int)dtype & ~ENF_NEGLL_ZYGOTE);
  }
  ~ZygoteScope() { enf::tl_negll_zygote = 0; }
};

}  // namespace

extern "C" {

const char* enf_version(void) {
  static char buf[64];
  std::snprintf(buf, sizeof buf, "%d.%d.%d gfx950", ENF_VERSION_MAJOR, ENF_VERSION_MINOR, ENF_VERSION_PATCH);
  return buf;
}

const char* enf_last_error(void) { return g_last_error.c_str(); }

enf_status enf_device_count(int32_t* count) {
  ENF_TRY
  if (!count) return fail(ENF_ERR_INVALID, "count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
  *count = n;
  return ENF_OK;
  ENF_CATCH
}

enf_status enf_set_device(int32_t device) {
  ENF_TRY
  hipError_t e = hipSetDevice(device);
  return e == hipSuccess ? ENF_OK : hip_fail(e, "hipSetDevice");
  ENF_CATCH
}

enf_status enf_get_device(int32_t* device) {
  ENF_TRY
  if (!device) return fail(ENF_ERR_INVALID, "device is NULL");
  int d = 0;
  hipError_t e = hipGetDevice(&d);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  *device = d;
  return ENF_OK;
  ENF_CATCH
}

enf_status enf_malloc(void** ptr, size_t bytes) {
  ENF_TRY
  if (!ptr) return fail(ENF_ERR_INVALID, "ptr is NULL");
  hipError_t e = hipMalloc(ptr, bytes);
  return e == hipSuccess ? ENF_OK : hip_fail(e, "hipMalloc");
  ENF_CATCH
}

enf_status enf_free(void* ptr) {
  ENF_TRY
  hipError_t e = hipFree(ptr);
  return e == hipSuccess ? ENF_OK : hip_fail(e, "hipFree");
  ENF_CATCH
}

enf_status enf_memcpy(void* dst, const void* src, size_t bytes, int32_t kind, void* hip_stream) {
  ENF_TRY
  if (bytes == 0) return ENF_OK;
  if (!dst || !src) return fail(ENF_ERR_INVALID, "memcpy: NULL pointer");
  hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                  : kind == 1 ? hipMemcpyDeviceToHost
                  : kind == 2 ? hipMemcpyDeviceToDevice : hipMemcpyDefault;
  hipError_t e = hipMemcpyAsync(dst, src, bytes, k, (hipStream_t)hip_stream);
  return e == hipSuccess ? ENF_OK : hip_fail(e, "hipMemcpyAsync");
  ENF_CATCH
}

enf_status enf_stream_synchronize(void* hip_stream) {
  ENF_TRY
  hipError_t e = hipStreamSynchronize((hipStream_t)hip_stream);
  return e == hipSuccess ? ENF_OK : hip_fail(e, "hipStreamSynchronize");
  ENF_CATCH
}

enf_status enf_flow_apply(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx, void* Y,
                          int64_t ldy, void* ladj, int32_t accumulate_ladj, const enf_layer* layers,
                          int32_t nlayers, void* hip_stream) {
  ENF_TRY
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "dtype must be ENF_F32 or ENF_F64");
  if (D < 0 || N < 0) return fail(ENF_ERR_INVALID, "D and N must be >= 0");
  if (D > (int64_t)1 << 30) return fail(ENF_ERR_UNSUPPORTED, "D too large");
  if (ldx < (D > 0 ? D : 1) || ldy < (D > 0 ? D : 1)) return fail(ENF_ERR_INVALID, "leading dimension < D");
  enf_status vs = validate_layers(D, layers, nlayers);
  if (vs != ENF_OK) return vs;
  if (N == 0) return ENF_OK;
  if (D > 0 && (!X || !Y)) return fail(ENF_ERR_INVALID, "X or Y is NULL");
  const size_t elem = dtype == ENF_F64 ? 8 : 4;
  hipStream_t st = (hipStream_t)hip_stream;
  if (D > 0 && X != Y) {  // partial overlap of X and Y is not supported (exact aliasing is)
    const char* xb = (const char*)X;
    const char* yb = (const char*)Y;
    const char* xe = xb + ((N - 1) * ldx + D) * elem;
    const char* ye = yb + ((N - 1) * ldy + D) * elem;
    if (xb < ye && yb < xe) return fail(ENF_ERR_INVALID, "X and Y overlap without being identical");
  } else if (D > 0 && ldx != ldy) {
    return fail(ENF_ERR_INVALID, "in-place call (X == Y) needs ldx == ldy");
  }

  // empty flow or empty samples: Y = X, ladj = 0 (ChangesOfVariables: identity has ladj 0)
  if (D == 0 || nlayers == 0) {
    if (D > 0 && X != Y) {
      hipError_t e = hipMemcpy2DAsync(Y, ldy * elem, X, ldx * elem, D * elem, N, hipMemcpyDeviceToDevice, st);
      if (e != hipSuccess) return hip_fail(e, "hipMemcpy2DAsync");
    }
    if (ladj && !accumulate_ladj) {
      hipError_t e = hipMemsetAsync(ladj, 0, N * elem, st);
      if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync");
    }
    return ENF_OK;
  }

  enf::DeviceInfo dev;
  enf_status ds = device_info(&dev);
  if (ds != ENF_OK) return ds;

  // flatten into steps: one per transform, one per Householder reflection column
  // (dense-Householder path: a chained HouseholderTrafo with k >= wy_min_k() reflections becomes
  // OP_DENSE steps of <= D reflections each, col = first column | count << 16)
  bool frag = enf::frag_path(D, ldx, ldy, X, Y, elem) && enf::frag_path(D, ldy, ldy, Y, Y, elem);
  // padded fragment path: D a multiple of 16/elem but not a power of two, laid out as the next power
  // of two (enf_internal.h frag_pad_dim); every op has neutral parameters that map 0 to 0 with ladj 0
  int64_t dk = 0;
  if (!frag) {
    dk = enf::frag_pad_dim(D, ldx, ldy, X, Y, elem);
    frag = dk != 0;
  }
  bool wy = false;
  if (!dk && enf::wy_supported(D, frag))
    for (int32_t l = 0; l < nlayers; ++l)
      if (layers[l].op == ENF_OP_HOUSEHOLDER && layers[l].k >= enf::wy_min_k()) wy = true;
  struct S { int32_t op, layer, col; };
  std::vector<S> steps;
  for (int32_t l = 0; l < nlayers; ++l) {
    if (layers[l].op == ENF_OP_HOUSEHOLDER && wy && layers[l].k >= enf::wy_min_k()) {
      for (int32_t c = 0; c < layers[l].k; c += (int32_t)D) {
        const int32_t cnt = std::min<int32_t>((int32_t)D, layers[l].k - c);
        steps.push_back({enf::OP_DENSE, l, c | (cnt << 16)});
      }
    } else if (layers[l].op == ENF_OP_HOUSEHOLDER) {
      for (int32_t c = 0; c < layers[l].k; ++c) steps.push_back({layers[l].op, l, c});
    } else {
      steps.push_back({layers[l].op, l, 0});
    }
  }

  // cut into launches bounded by the kernarg tables and the LDS parameter budget
  size_t i = 0;
  bool first = true;
  while (i < steps.size()) {
    enf::FlowArgs a;
    std::memset(&a, 0, sizeof a);
    a.D = (int32_t)D;
    a.N = N;
    a.frag = frag ? 1 : 0;
    a.dk = (int32_t)dk;
    a.wy = wy ? 1 : 0;
    size_t recs = 0;
    int last_layer = -1;
    while (i < steps.size() && a.nsteps < enf::kMaxSteps) {
      const S& s = steps[i];
      const size_t w = enf::record_elems(s.op, dk ? dk : D, elem, frag) * elem;
      const bool new_layer = s.layer != last_layer;
      if (new_layer && a.nlayers >= enf::kMaxLayers) break;
      if (recs + w > (wy ? enf::kLdsParamBudgetWY : enf::kLdsParamBudget)) {
        if (a.nsteps == 0)
          return fail(ENF_ERR_UNSUPPORTED, "D too large: one transform's parameter records exceed the LDS budget");
        break;
      }
      if (new_layer) {
        enf::LayerDesc& L = a.layers[a.nlayers++];
        L.op = layers[s.layer].op;
        L.k = layers[s.layer].k;
        for (int q = 0; q < 4; ++q) L.p[q] = layers[s.layer].p[q];
        last_layer = s.layer;
      }
      enf::Step& t = a.steps[a.nsteps++];
      t.op = s.op;
      t.layer = a.nlayers - 1;
      t.col = s.col;
      t.off = (int32_t)(recs / elem);
      a.desc[a.nsteps - 1] = t.op | (t.off << 4);
      recs += w;
      ++i;
    }
    a.X = first ? X : Y;
    a.ldx = first ? ldx : ldy;
    a.Y = Y;
    a.ldy = ldy;
    a.ladj = ladj;
    a.accumulate = first ? accumulate_ladj : 1;
#if ENF_BOUNDS
    a.csum = enf::flow_args_csum(a);
#endif
    hipError_t e = enf::launch_flow(a, dtype == ENF_F64, st, dev);
    if (e != hipSuccess) return hip_fail(e, "flow kernel launch");
    first = false;
  }
  return ENF_OK;
  ENF_CATCH
}

// ------------------------------------------------------------------- host-resident batches ----
namespace {

// Round 3: the ring no longer page-locks the caller's arrays (hipHostRegister / hipHostUnregister of
// arbitrary, non-page-aligned heap ranges). A process that had registered and released host arrays
// later hit hipErrorIllegalAddress in ordinary pageable torch copies of NEW heap arrays placed on the
// released pages (tools/pin_overlap_probe.py). The ring now owns its host staging:
// pinned slots from hipHostMalloc, filled from / drained to the caller's arrays by threaded host
// copies that overlap the device work of the other slots.
// The slot buffers (device ring and pinned host staging) are cached per process for the device of the
// last call and reused while large enough (pinning hundreds of MB costs far more than a chunk's copy);
// a concurrent call that finds the cache in use allocates its own and frees them on return. A slot is
// at most kStageCap bytes, so the cache stays small (6 x 32 MB pinned host, 3 x 32 MB device).
constexpr size_t kStageCap = (size_t)32 << 20;
constexpr int kRingSlots = 3;
struct RingBufs {
  void* buf[kRingSlots] = {};   // device: D x C chunk, then C ladj values
  void* hin[kRingSlots] = {};   // pinned host: the chunk going up
  void* hout[kRingSlots] = {};  // pinned host: the results coming down
  size_t bytes = 0;
  int dev = -1;
  void release() {
    for (int s = 0; s < kRingSlots; ++s) {
      if (buf[s]) (void)hipFree(buf[s]);
      if (hin[s]) (void)hipHostFree(hin[s]);
      if (hout[s]) (void)hipHostFree(hout[s]);
      buf[s] = hin[s] = hout[s] = nullptr;
    }
    bytes = 0;
    dev = -1;
  }
  hipError_t ensure(size_t need, int device) {
    if (bytes >= need && dev == device) return hipSuccess;
    release();
    for (int s = 0; s < kRingSlots; ++s) {
      hipError_t e = hipMalloc(&buf[s], need);
      if (e == hipSuccess) e = hipHostMalloc(&hin[s], need, hipHostMallocDefault);
      if (e == hipSuccess) e = hipHostMalloc(&hout[s], need, hipHostMallocDefault);
      if (e != hipSuccess) {
        release();
        return e;
      }
    }
    bytes = need;
    dev = device;
    return hipSuccess;
  }
};
std::mutex g_ring_mu;
RingBufs g_ring_cache;

struct Ring {
  static constexpr int kSlots = kRingSlots;
  std::unique_lock<std::mutex> lk{g_ring_mu, std::try_to_lock};
  RingBufs own;
  RingBufs& b = lk.owns_lock() ? g_ring_cache : own;
  hipEvent_t h2d[kSlots] = {}, comp[kSlots] = {}, d2h[kSlots] = {};
  hipStream_t up = nullptr, down = nullptr;
  hipStream_t caller = nullptr;  // set once the ring has queued work on the caller's stream
  bool queued = false;
  ~Ring() {
    // an error exit may leave flow kernels queued on the caller's stream that still use the slots: they
    // finish before the slots are released or handed to the next call
    if (queued) (void)hipStreamSynchronize(caller);
    if (up) (void)hipStreamSynchronize(up);
    if (down) (void)hipStreamSynchronize(down);
    for (int s = 0; s < kSlots; ++s) {
      if (h2d[s]) (void)hipEventDestroy(h2d[s]);
      if (comp[s]) (void)hipEventDestroy(comp[s]);
      if (d2h[s]) (void)hipEventDestroy(d2h[s]);
    }
    if (up) (void)hipStreamDestroy(up);
    if (down) (void)hipStreamDestroy(down);
    own.release();
  }
};

// cols columns of `width` bytes from src (column stride ss bytes) to dst (stride ds), split over up to 8
// host threads for large copies (a single thread moves ~10 GB/s; the PCIe link ~2-5x that)
void host_copy_cols(char* dst, size_t ds, const char* src, size_t ss, size_t width, int64_t cols) {
  const size_t bytes = width * (size_t)cols;
  const auto part = [&](int64_t c0, int64_t c1) {
    if (ds == width && ss == width) {
      std::memcpy(dst + (size_t)c0 * width, src + (size_t)c0 * width, (size_t)(c1 - c0) * width);
    } else {
      for (int64_t c = c0; c < c1; ++c) std::memcpy(dst + (size_t)c * ds, src + (size_t)c * ss, width);
    }
  };
  int nt = (int)std::min<size_t>(8, bytes >> 22);  // one thread per 4 MiB, at most 8
  const int hc = enf::usable_cpus();
  if (nt > hc) nt = hc;
  if (nt <= 1 || cols < nt) {
    part(0, cols);
    return;
  }
  std::vector<std::thread> pool;
  pool.reserve((size_t)nt);
  int started = 0;
  try {
    for (int t = 1; t < nt; ++t) {
      pool.emplace_back(part, cols * t / nt, cols * (t + 1) / nt);
      ++started;
    }
  } catch (...) {
  }
  part(0, cols / nt);
  // columns of threads that could not be started: on this thread
  if (started < nt - 1) part(cols * (started + 1) / nt, cols);
  for (auto& th : pool) th.join();
}

}  // namespace

enf_status enf_flow_apply_host(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx, void* Y,
                               int64_t ldy, void* ladj, int32_t accumulate_ladj, const enf_layer* layers,
                               int32_t nlayers, int64_t chunk_cols, void* hip_stream) {
  ENF_TRY
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "dtype must be ENF_F32 or ENF_F64");
  if (D < 1 || N < 0) return fail(ENF_ERR_INVALID, "D must be >= 1 and N >= 0");
  if (ldx < D || ldy < D) return fail(ENF_ERR_INVALID, "leading dimension < D");
  if (chunk_cols < 0) return fail(ENF_ERR_INVALID, "chunk_cols < 0");
  if (N == 0) return ENF_OK;
  if (!X || !Y) return fail(ENF_ERR_INVALID, "X or Y is NULL");
  if (X == Y && ldx != ldy) return fail(ENF_ERR_INVALID, "in-place call (X == Y) needs ldx == ldy");
  const size_t elem = dtype == ENF_F64 ? 8 : 4;
  // chunk: chunk_cols columns (0: as many as fill a slot), at most one slot of kStageCap bytes
  const int64_t cap = std::max<int64_t>(1, (int64_t)(kStageCap / ((size_t)(D + 1) * elem)));
  int64_t C = chunk_cols > 0 ? std::min(chunk_cols, cap) : cap;
  if (C > N) C = N;
  hipStream_t st = (hipStream_t)hip_stream;
  int device = 0;
  hipError_t e = hipGetDevice(&device);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  Ring r;
  const size_t slot_bytes = ((size_t)D * C + (size_t)C) * elem;
  if ((e = r.b.ensure(slot_bytes, device)) != hipSuccess) return hip_fail(e, "ingest ring / staging allocation");
  for (int s = 0; s < Ring::kSlots; ++s) {
    if ((e = hipEventCreateWithFlags(&r.h2d[s], hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&r.comp[s], hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&r.d2h[s], hipEventDisableTiming)) != hipSuccess)
      return hip_fail(e, "hipEventCreate");
  }
  if ((e = hipStreamCreateWithFlags(&r.up, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&r.down, hipStreamNonBlocking)) != hipSuccess)
    return hip_fail(e, "hipStreamCreate");
  // the ring starts after everything already queued on the caller's stream: the host copies out of X and
  // into Y / ladj are not stream-ordered, so the host waits for that work (e.g. an async copy into X) first
  if ((e = hipEventRecord(r.comp[0], st)) != hipSuccess) return hip_fail(e, "hipEventRecord");
  if ((e = hipEventSynchronize(r.comp[0])) != hipSuccess) return hip_fail(e, "hipEventSynchronize");
  r.caller = st;
  const char* Xc = (const char*)X;
  char* Yc = (char*)Y;
  char* Lc = (char*)ladj;
  const int64_t nchunks = (N + C - 1) / C;
  const size_t colb = (size_t)D * elem;
  // results of chunk j: staging -> the caller's Y (and ladj)
  auto drain = [&](int64_t j) -> hipError_t {
    const int s = (int)(j % Ring::kSlots);
    const int64_t c0 = j * C, cols = N - c0 < C ? N - c0 : C;
    hipError_t ee = hipEventSynchronize(r.d2h[s]);
    if (ee != hipSuccess) return ee;
    const char* h = (const char*)r.b.hout[s];
    host_copy_cols(Yc + (size_t)c0 * ldy * elem, (size_t)ldy * elem, h, colb, colb, cols);
    if (ladj) std::memcpy(Lc + (size_t)c0 * elem, h + (size_t)D * C * elem, (size_t)cols * elem);
    return hipSuccess;
  };
  for (int64_t i = 0; i < nchunks; ++i) {
    const int s = (int)(i % Ring::kSlots);
    const int64_t c0 = i * C, cols = N - c0 < C ? N - c0 : C;
    // slot reuse: chunk i - 3's results leave the staging first (its upload finished before them); in
    // place (Y == X), chunk i - 3's columns are not chunk i's, so the order of the host copies is free
    if (i >= Ring::kSlots && (e = drain(i - Ring::kSlots)) != hipSuccess) return hip_fail(e, "ingest drain");
    char* hi = (char*)r.b.hin[s];
    host_copy_cols(hi, colb, Xc + (size_t)c0 * ldx * elem, (size_t)ldx * elem, colb, cols);
    if (ladj && accumulate_ladj) std::memcpy(hi + (size_t)D * C * elem, Lc + (size_t)c0 * elem, (size_t)cols * elem);
    char* dX = (char*)r.b.buf[s];
    char* dL = dX + (size_t)D * C * elem;
    e = hipMemcpyAsync(dX, hi, (size_t)D * cols * elem, hipMemcpyHostToDevice, r.up);
    if (e == hipSuccess && ladj && accumulate_ladj)
      e = hipMemcpyAsync(dL, hi + (size_t)D * C * elem, cols * elem, hipMemcpyHostToDevice, r.up);
    if (e == hipSuccess) e = hipEventRecord(r.h2d[s], r.up);
    if (e == hipSuccess) e = hipStreamWaitEvent(st, r.h2d[s], 0);
    if (e != hipSuccess) return hip_fail(e, "ingest H2D");
    r.queued = true;
    enf_status fs = enf_flow_apply(dtype, D, cols, dX, D, dX, D, ladj ? dL : nullptr, accumulate_ladj, layers,
                                   nlayers, st);
    if (fs != ENF_OK) return fs;
    if ((e = hipEventRecord(r.comp[s], st)) != hipSuccess || (e = hipStreamWaitEvent(r.down, r.comp[s], 0)) != hipSuccess)
      return hip_fail(e, "ingest compute event");
    char* ho = (char*)r.b.hout[s];
    e = hipMemcpyAsync(ho, dX, (size_t)D * cols * elem, hipMemcpyDeviceToHost, r.down);
    if (e == hipSuccess && ladj) e = hipMemcpyAsync(ho + (size_t)D * C * elem, dL, cols * elem, hipMemcpyDeviceToHost, r.down);
    if (e == hipSuccess) e = hipEventRecord(r.d2h[s], r.down);
    if (e != hipSuccess) return hip_fail(e, "ingest D2H");
  }
  // synchronous: the last chunks' results are in the caller's arrays on return
  for (int64_t j = nchunks > Ring::kSlots ? nchunks - Ring::kSlots : 0; j < nchunks; ++j)
    if ((e = drain(j)) != hipSuccess) return hip_fail(e, "ingest drain");
  return ENF_OK;
  ENF_CATCH
}

enf_status enf_flow_param_count(int64_t D, const enf_layer* layers, int32_t nlayers, int64_t* count) {
  ENF_TRY
  if (!count) return fail(ENF_ERR_INVALID, "count is NULL");
  if (D < 0) return fail(ENF_ERR_INVALID, "D < 0");
  enf_status vs = validate_layers(D, layers, nlayers);
  if (vs != ENF_OK) return vs;
  int64_t n = 0;
  for (int32_t l = 0; l < nlayers; ++l)
    n += D * (layers[l].op == ENF_OP_HOUSEHOLDER ? layers[l].k : nparams_of(layers[l].op));
  *count = n;
  return ENF_OK;
  ENF_CATCH
}

enf_status enf_flow_apply_cpu(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx, void* Y, int64_t ldy,
                              void* ladj, int32_t accumulate_ladj, const enf_layer* layers, int32_t nlayers,
                              int32_t nthreads) {
  ENF_TRY
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (D < 0 || N < 0) return fail(ENF_ERR_INVALID, "D and N must be >= 0");
  if (ldx < (D > 0 ? D : 1) || ldy < (D > 0 ? D : 1)) return fail(ENF_ERR_INVALID, "ldx or ldy < D");
  enf_status vs = validate_layers(D, layers, nlayers);
  if (vs != ENF_OK) return vs;
  if (N == 0) return ENF_OK;
  if (D > 0 && (!X || !Y)) return fail(ENF_ERR_INVALID, "X or Y is NULL");
  const size_t elem = dtype == ENF_F64 ? 8 : 4;
  if (D > 0 && X != Y) {
    const char* xb = (const char*)X;
    const char* yb = (const char*)Y;
    const char* xe = xb + ((N - 1) * ldx + D) * elem;
    const char* ye = yb + ((N - 1) * ldy + D) * elem;
    if (xb < ye && yb < xe) return fail(ENF_ERR_INVALID, "X and Y overlap without being identical");
  } else if (D > 0 && ldx != ldy) {
    return fail(ENF_ERR_INVALID, "in-place call (X == Y) needs ldx == ldy");
  }
  return enf::flow_apply_cpu(dtype == ENF_F64, D, N, X, ldx, Y, ldy, ladj, accumulate_ladj, layers, D > 0 ? nlayers : 0,
                             nthreads);
  ENF_CATCH
}

enf_status enf_flow_negll_grad_workspace(enf_dtype dtype, int64_t D, int64_t N, const enf_layer* layers,
                                         int32_t nlayers, size_t* bytes) {
  ENF_TRY
  if (!bytes) return fail(ENF_ERR_INVALID, "bytes is NULL");
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (D < 0 || N < 0) return fail(ENF_ERR_INVALID, "D and N must be >= 0");
  enf_status vs = validate_layers(D, layers, nlayers);
  if (vs != ENF_OK) return vs;
  return enf::negll_grad_workspace(dtype == ENF_F64, D, N, layers, nlayers, bytes);
  ENF_CATCH
}

enf_status enf_flow_negll_grad(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx,
                               const enf_layer* layers, int32_t nlayers, void* out, void* workspace,
                               size_t workspace_bytes, void* hip_stream) {
  ENF_TRY
  ZygoteScope zygote(dtype);
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (D < 0 || N < 0) return fail(ENF_ERR_INVALID, "D and N must be >= 0");
  if (ldx < (D > 0 ? D : 1)) return fail(ENF_ERR_INVALID, "ldx < D");
  enf_status vs = validate_layers(D, layers, nlayers);
  if (vs != ENF_OK) return vs;
  if (!out) return fail(ENF_ERR_INVALID, "out is NULL");
  if (N == 0) return ENF_OK;
  if (D > 0 && !X) return fail(ENF_ERR_INVALID, "X is NULL");
  return enf::negll_grad(dtype == ENF_F64, D, N, X, ldx, layers, nlayers, out, workspace, workspace_bytes,
                         (hipStream_t)hip_stream);
  ENF_CATCH
}

enf_status enf_flow_negll_workspace(enf_dtype dtype, int64_t D, int64_t N, size_t* bytes) {
  ENF_TRY
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (D < 0 || N < 0) return fail(ENF_ERR_INVALID, "D and N must be >= 0");
  if (!bytes) return fail(ENF_ERR_INVALID, "bytes is NULL");
  return enf::negll_loss_workspace(dtype == ENF_F64, D, N, bytes);
  ENF_CATCH
}

enf_status enf_flow_negll(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx, const enf_layer* layers,
                          int32_t nlayers, void* out, void* workspace, size_t workspace_bytes, void* hip_stream) {
  ENF_TRY
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (D < 0 || N < 0) return fail(ENF_ERR_INVALID, "D and N must be >= 0");
  if (ldx < (D > 0 ? D : 1)) return fail(ENF_ERR_INVALID, "ldx < D");
  enf_status vs = validate_layers(D, layers, nlayers);
  if (vs != ENF_OK) return vs;
  if (!out) return fail(ENF_ERR_INVALID, "out is NULL");
  if (N == 0) return ENF_OK;
  if (D > 0 && !X) return fail(ENF_ERR_INVALID, "X is NULL");
  return enf::negll_loss(dtype == ENF_F64, D, N, X, ldx, layers, nlayers, out, workspace, workspace_bytes,
                         (hipStream_t)hip_stream);
  ENF_CATCH
}

enf_status enf_flow_vjp(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx, const void* dY,
                        int64_t lddy, const void* dladj, const enf_layer* layers, int32_t nlayers, void* dX,
                        int64_t lddx, void* dparams, void* workspace, size_t workspace_bytes, void* hip_stream) {
  ENF_TRY
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (D < 0 || N < 0) return fail(ENF_ERR_INVALID, "D and N must be >= 0");
  const int64_t d1 = D > 0 ? D : 1;
  if (ldx < d1 || lddy < d1 || lddx < d1) return fail(ENF_ERR_INVALID, "ldx, lddy or lddx < D");
  enf_status vs = validate_layers(D, layers, nlayers);
  if (vs != ENF_OK) return vs;
  if (N == 0 || D == 0) return ENF_OK;
  if (!X || !dY || !dX) return fail(ENF_ERR_INVALID, "X, dY or dX is NULL");
  if (dX == X) return fail(ENF_ERR_INVALID, "dX may not alias X");
  if (dX == dY && lddx != lddy) return fail(ENF_ERR_INVALID, "dX aliases dY with a different leading dimension");
  return enf::flow_vjp(dtype == ENF_F64, D, N, X, ldx, dY, lddy, dladj, layers, nlayers, dX, lddx, dparams, workspace,
                       workspace_bytes, (hipStream_t)hip_stream);
  ENF_CATCH
}

enf_status enf_whitening_step(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx,
                              const enf_layer* layers, int32_t nlayers, void* theta, void* acc, const int64_t* runs,
                              int32_t nruns, const int64_t* hbatches, int32_t nhb, double eta, double epsilon,
                              double* loss_out, void* workspace, size_t workspace_bytes, void* hip_stream) {
  ENF_TRY
  ZygoteScope zygote(dtype);
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (D < 1 || N < 1) return fail(ENF_ERR_INVALID, "D and N must be >= 1");
  if (ldx < D) return fail(ENF_ERR_INVALID, "ldx < D");
  enf_status vs = validate_layers(D, layers, nlayers);
  if (vs != ENF_OK) return vs;
  if (!X || !theta || !acc || !loss_out) return fail(ENF_ERR_INVALID, "X, theta, acc or loss_out is NULL");
  if ((nruns > 0 && !runs) || (nhb > 0 && !hbatches)) return fail(ENF_ERR_INVALID, "runs or hbatches is NULL");
  return enf::whitening_step(dtype == ENF_F64, D, N, X, ldx, layers, nlayers, theta, acc, runs, nruns, hbatches, nhb,
                             eta, epsilon, loss_out, workspace, workspace_bytes, (hipStream_t)hip_stream);
  ENF_CATCH
}

enf_status enf_whitening_epoch(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx, int64_t batchsize,
                               const enf_layer* layers, int32_t nlayers, void* theta, void* acc, const int64_t* runs,
                               int32_t nruns, const int64_t* hbatches, int32_t nhb, double eta, double epsilon,
                               double* loss_out, void* workspace, size_t workspace_bytes, void* hip_stream) {
  ENF_TRY
  ZygoteScope zygote(dtype);
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (D < 1 || N < 1 || batchsize < 1) return fail(ENF_ERR_INVALID, "D, N and batchsize must be >= 1");
  if (ldx < D) return fail(ENF_ERR_INVALID, "ldx < D");
  enf_status vs = validate_layers(D, layers, nlayers);
  if (vs != ENF_OK) return vs;
  if (!X || !theta || !acc || !loss_out) return fail(ENF_ERR_INVALID, "X, theta, acc or loss_out is NULL");
  if ((nruns > 0 && !runs) || (nhb > 0 && !hbatches)) return fail(ENF_ERR_INVALID, "runs or hbatches is NULL");
  return enf::whitening_epoch(dtype == ENF_F64, D, N, X, ldx, batchsize, layers, nlayers, theta, acc, runs, nruns,
                              hbatches, nhb, eta, epsilon, loss_out, workspace, workspace_bytes,
                              (hipStream_t)hip_stream);
  ENF_CATCH
}

enf_status enf_whitening_apply(enf_dtype dtype, int64_t D, int64_t nparams, const void* g, int64_t B, void* theta,
                               void* acc, const int64_t* runs, int32_t nruns, const int64_t* hbatches, int32_t nhb,
                               double eta, double epsilon, double* loss_out, void* hip_stream) {
  ENF_TRY
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (D < 1 || nparams < 0 || B < 1) return fail(ENF_ERR_INVALID, "D and B must be >= 1, nparams >= 0");
  if (!g || !theta || !acc || !loss_out) return fail(ENF_ERR_INVALID, "g, theta, acc or loss_out is NULL");
  if ((nruns > 0 && !runs) || (nhb > 0 && !hbatches)) return fail(ENF_ERR_INVALID, "runs or hbatches is NULL");
  return enf::whitening_apply(dtype == ENF_F64, D, nparams, g, B, theta, acc, runs, nruns, hbatches, nhb, eta, epsilon,
                              loss_out, (hipStream_t)hip_stream);
  ENF_CATCH
}

enf_status enf_adagrad_step(enf_dtype dtype, int64_t count, void* params, void* acc, const void* grad,
                            double grad_scale, double eta, double epsilon, void* hip_stream) {
  ENF_TRY
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (count < 0) return fail(ENF_ERR_INVALID, "count < 0");
  if (count == 0) return ENF_OK;
  if (!params || !acc || !grad) return fail(ENF_ERR_INVALID, "NULL pointer");
  return enf::adagrad_step(dtype == ENF_F64, count, params, acc, grad, grad_scale, eta, epsilon,
                           (hipStream_t)hip_stream);
  ENF_CATCH
}

enf_status enf_householder_normalize(enf_dtype dtype, int64_t D, int64_t k, void* V, void* hip_stream) {
  ENF_TRY
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (D < 0 || k < 0) return fail(ENF_ERR_INVALID, "D and k must be >= 0");
  if (D == 0 || k == 0) return ENF_OK;
  if (!V) return fail(ENF_ERR_INVALID, "V is NULL");
  return enf::householder_normalize(dtype == ENF_F64, D, k, V, D, (hipStream_t)hip_stream);
  ENF_CATCH
}

enf_status enf_householder_normalize_strided(enf_dtype dtype, int64_t D, int64_t k, void* V, int64_t ldv,
                                             void* hip_stream) {
  ENF_TRY
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (D < 0 || k < 0) return fail(ENF_ERR_INVALID, "D and k must be >= 0");
  if (k > 1 && ldv < D) return fail(ENF_ERR_INVALID, "ldv < D");
  if (D == 0 || k == 0) return ENF_OK;
  if (!V) return fail(ENF_ERR_INVALID, "V is NULL");
  return enf::householder_normalize(dtype == ENF_F64, D, k, V, ldv, (hipStream_t)hip_stream);
  ENF_CATCH
}

enf_status enf_stream_copy(const void* src, void* dst, int64_t bytes, int32_t variant, void* hip_stream) {
  ENF_TRY
  if (bytes < 0) return fail(ENF_ERR_INVALID, "bytes < 0");
  if (bytes > 0 && (!src || !dst)) return fail(ENF_ERR_INVALID, "src or dst is NULL");
  return enf::stream_copy(src, dst, bytes, variant, (hipStream_t)hip_stream);
  ENF_CATCH
}

// ------------------------------------------------------------------------ JohnsonSU ----
enf_status enf_johnsonsu_eval(enf_dtype dtype, int32_t fn, int64_t n, const void* x, void* out, double gamma,
                              double delta, double xi, double lambda, void* hip_stream) {
  ENF_TRY
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (fn < ENF_JSU_PDF || fn > ENF_JSU_QUANTILE) return fail(ENF_ERR_INVALID, "unknown JohnsonSU function");
  if (n < 0) return fail(ENF_ERR_INVALID, "n must be >= 0");
  if (n == 0) return ENF_OK;
  if (!x || !out) return fail(ENF_ERR_INVALID, "x or out is NULL");
  enf::DeviceInfo dev;
  enf_status ds = device_info(&dev);
  if (ds != ENF_OK) return ds;
  const double prm[4] = {gamma, delta, xi, lambda};
  hipError_t e = enf::launch_jsu_eval(dtype == ENF_F64, fn, n, x, out, prm, (hipStream_t)hip_stream, dev);
  return e == hipSuccess ? ENF_OK : hip_fail(e, "JohnsonSU kernel launch");
  ENF_CATCH
}

enf_status enf_johnsonsu_sample(enf_dtype dtype, int64_t n, void* out, double gamma, double delta, double xi,
                                double lambda, uint64_t seed, uint64_t offset, void* hip_stream) {
  ENF_TRY
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (n < 0) return fail(ENF_ERR_INVALID, "n must be >= 0");
  if (n == 0) return ENF_OK;
  if (!out) return fail(ENF_ERR_INVALID, "out is NULL");
  enf::DeviceInfo dev;
  enf_status ds = device_info(&dev);
  if (ds != ENF_OK) return ds;
  const double prm[4] = {gamma, delta, xi, lambda};
  hipError_t e = enf::launch_jsu_sample(dtype == ENF_F64, n, out, prm, seed, offset, (hipStream_t)hip_stream, dev);
  return e == hipSuccess ? ENF_OK : hip_fail(e, "JohnsonSU sampling kernel launch");
  ENF_CATCH
}

// ---------------------------------------------------------------------------------- RCCL ----
struct enf_comm_s {
  ncclComm_t comm;
};

static_assert(sizeof(ncclUniqueId) == ENF_UNIQUE_ID_BYTES, "ncclUniqueId size");

enf_status enf_comm_unique_id(uint8_t id[ENF_UNIQUE_ID_BYTES]) {
  ENF_TRY
  if (!id) return fail(ENF_ERR_INVALID, "id is NULL");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return fail(ENF_ERR_RCCL, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(id, &u, sizeof u);
  return ENF_OK;
  ENF_CATCH
}

enf_status enf_comm_init(enf_comm* comm, int32_t nranks, const uint8_t id[ENF_UNIQUE_ID_BYTES], int32_t rank) {
  ENF_TRY
  if (!comm || !id) return fail(ENF_ERR_INVALID, "NULL pointer");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(ENF_ERR_INVALID, "bad rank / nranks");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  auto* c = new enf_comm_s;
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail(ENF_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  *comm = c;
  return ENF_OK;
  ENF_CATCH
}

enf_status enf_comm_destroy(enf_comm comm) {
  ENF_TRY
  if (!comm) return ENF_OK;
  // the documented teardown: ncclCommFinalize flushes every collective issued on the communicator
  // (blocking communicator), then ncclCommDestroy frees its local resources
  ncclResult_t r = ncclCommFinalize(comm->comm);
  const ncclResult_t rd = ncclCommDestroy(comm->comm);
  if (r == ncclSuccess) r = rd;
  delete comm;
  if (r != ncclSuccess) return fail(ENF_ERR_RCCL, std::string("ncclCommDestroy: ") + ncclGetErrorString(r));
  return ENF_OK;
  ENF_CATCH
}

enf_status enf_allreduce_sum(enf_comm comm, void* buf, int64_t count, enf_dtype dtype, void* hip_stream) {
  ENF_TRY
  if (!comm) return fail(ENF_ERR_INVALID, "comm is NULL");
  if (count < 0) return fail(ENF_ERR_INVALID, "count < 0");
  if (count == 0) return ENF_OK;
  if (!buf) return fail(ENF_ERR_INVALID, "buf is NULL");
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, dtype == ENF_F64 ? ncclFloat64 : ncclFloat32, ncclSum,
                                 comm->comm, (hipStream_t)hip_stream);
  if (r != ncclSuccess) return fail(ENF_ERR_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
  return ENF_OK;
  ENF_CATCH
}

// ------------------------------------------------------------- data-parallel training step ----
static enf_status rccl_allreduce(void* ctx, void* buf, int64_t count, bool f64, hipStream_t st) {
  const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, f64 ? ncclFloat64 : ncclFloat32, ncclSum,
                                       static_cast<enf_comm_s*>(ctx)->comm, st);
  return r == ncclSuccess ? ENF_OK : fail(ENF_ERR_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
}

enf_status enf_whitening_step_dp(enf_dtype dtype, int64_t D, int64_t N, const void* X, int64_t ldx,
                                 const enf_layer* layers, int32_t nlayers, void* theta, void* acc, const int64_t* runs,
                                 int32_t nruns, const int64_t* hbatches, int32_t nhb, double eta, double epsilon,
                                 int64_t B, double* loss_out, enf_comm comm, void* workspace, size_t workspace_bytes,
                                 void* hip_stream) {
  ENF_TRY
  ZygoteScope zygote(dtype);
  if (dtype != ENF_F32 && dtype != ENF_F64) return fail(ENF_ERR_INVALID, "bad dtype");
  if (D < 1 || N < 0 || B < 1 || N > B) return fail(ENF_ERR_INVALID, "D and B must be >= 1, 0 <= N <= B");
  if (ldx < D) return fail(ENF_ERR_INVALID, "ldx < D");
  enf_status vs = validate_layers(D, layers, nlayers);
  if (vs != ENF_OK) return vs;
  if ((N > 0 && !X) || !theta || !acc || !loss_out) return fail(ENF_ERR_INVALID, "X, theta, acc or loss_out is NULL");
  if ((nruns > 0 && !runs) || (nhb > 0 && !hbatches)) return fail(ENF_ERR_INVALID, "runs or hbatches is NULL");
  int nranks = 1;
  if (comm && ncclCommCount(comm->comm, &nranks) != ncclSuccess) return fail(ENF_ERR_RCCL, "ncclCommCount failed");
  return enf::whitening_step_dp(dtype == ENF_F64, D, N, X, ldx, layers, nlayers, theta, acc, runs, nruns, hbatches, nhb,
                                eta, epsilon, B, loss_out, comm ? rccl_allreduce : nullptr, comm, workspace,
                                workspace_bytes, (hipStream_t)hip_stream, nranks);
  ENF_CATCH
}

}  // extern "C"
