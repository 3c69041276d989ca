// enf_cpu.cpp -- host (CPU) execution of a composed flow: enf_flow_apply_cpu (include/enf.h).
//
// SURVEY.md §8 config 1 ("ScaleShiftTrafo D=1, N=1e3 fp64 on CPU, no GPU"): data that lives in host
// memory runs here, as a Julia Array runs the reference's CPU methods; device data runs the HIP
// kernels. The host mirror selects the path by where the data is, never as a fallback.
//
// Arithmetic is the reference's, in the data type T, written out as Julia evaluates it (no implicit
// FMA contraction: this file is compiled with -ffp-contract=off; std::fma only where the reference
// calls muladd):
//   ScaleShiftTrafo  y = muladd(x, a, b); ladj = sum(log.(abs.(a))) per column   scale_shift_trafo.jl:16,22
//   CenterStretch    center_stretch(x); ladj = -sum(center_contract_ladj.(y))  center_stretch.jl:4-8,39-43
//   CenterContract   center_contract(x); ladj = sum(center_contract_ladj.(x))  center_stretch.jl:11-22,63-67
//   JohnsonTrafo     gamma + delta*asinh((x-xi)/lambda); ladj = sum(johnsontrafo_ladj.(x))
//                                                                               johnson_trafo.jl:29-32,49-52,76-80
//   JohnsonTrafoInv  lambda*sinh((x-gamma)/delta) + xi; ladj = -sum(johnsontrafo_ladj.(y))
//                                                                               johnson_trafo.jl:34-37,101-105
//   HouseholderTrafo k = (v'x)/(v'v); y = muladd(-2k, v, x), column by column of V; ladj 0
//                                                                               householder_trafo.jl:8-11,71-78
// Per-layer ladj are column sums in T (sum_ladjs, abstract_trafo.jl:9); the layers' totals combine in
// the order ChangesOfVariables' ComposedFunction method adds them for the usual left-associated
// f_n ∘ ... ∘ f_1: l_1 + (l_2 + (... + l_n)) (inner plus outer at every ∘ node).
//
// Execution: column blocks of kBlock samples, each block through all layers while it sits in cache;
// blocks are shared by worker threads (std::thread, static round-robin).
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "enf.h"

namespace enf {

enf_status set_error(enf_status st, const char* msg);

// CPUs this process may actually use: the affinity set, capped by the cgroup CPU quota (cgroup v2 cpu.max,
// or v1 cpu.cfs_quota_us / cpu.cfs_period_us) rounded up. std::thread::hardware_concurrency() counts every
// hardware thread of the machine (256 on the GPU box, whose cgroup grants 16): a pool that size time-slices
// on the quota. Queried once per process.
int usable_cpus() {
  static const int n = [] {
    int cpus = 0;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) cpus = CPU_COUNT(&set);
    if (cpus <= 0) cpus = (int)std::thread::hardware_concurrency();
    if (cpus <= 0) cpus = 1;
    double quota = -1.0;
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long long period = 0;
      if (std::fscanf(f, "%31s %lld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0)
        quota = std::atof(q) / (double)period;
      std::fclose(f);
    } else if (FILE* fq = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
      long long q = -1, period = 0;
      if (std::fscanf(fq, "%lld", &q) != 1) q = -1;
      std::fclose(fq);
      if (FILE* fp = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
        if (std::fscanf(fp, "%lld", &period) != 1) period = 0;
        std::fclose(fp);
      }
      if (q > 0 && period > 0) quota = (double)q / (double)period;
    }
    if (quota > 0.0) {
      const int qc = std::max(1, (int)std::ceil(quota - 1e-9));
      if (qc < cpus) cpus = qc;
    }
    return cpus;
  }();
  return n;
}

namespace {

constexpr int64_t kBlock = 64;

template <typename T>
inline T sgn(T x) { return x > T(0) ? T(1) : (x < T(0) ? T(-1) : x); }  // Julia sign (keeps +-0, NaN)

template <typename T>
inline T center_stretch_s(T x, T a, T b, T c) {
  const T e = std::exp(std::fabs(b * x));
  const T ome = T(1) - e;
  return sgn(x) * std::log((std::sqrt(ome * ome * std::exp(T(2) * b * a) + T(4) * e) - ome * std::exp(b * a)) / T(2)) / b + c;
}

template <typename T>
inline T center_contract_s(T x, T a, T b, T c) {
  const T xu = x - c;
  return (std::log(T(1) + std::exp(b * (xu - a))) - std::log(T(1) + std::exp(-b * (xu + a)))) / b;
}

template <typename T>
inline T center_contract_ladj_s(T x, T a, T b, T c) {
  const T xu = x - c;
  const T dy = T(1) / (T(1) + std::exp(-b * (xu - a))) + T(1) / (T(1) + std::exp(b * (xu + a)));
  return std::log(std::fabs(dy));
}

template <typename T>
inline T johnson_ladj_s(T x, T d, T xi, T l) {
  const T z = (x - xi) / l;
  return std::log(std::fabs((d / l) * (T(1) / std::sqrt(T(1) + z * z))));
}

struct HostLayer {
  int op;
  int k;
  const void* p[4];
};

// One layer on columns [0, nc) of the block Y (leading dimension ld); per-column ladj into lt.
template <typename T>
void layer_block(const HostLayer& L, int64_t D, int64_t nc, T* Y, int64_t ld, T* lt, const std::vector<T>& vv) {
  const T* p0 = (const T*)L.p[0];
  const T* p1 = (const T*)L.p[1];
  const T* p2 = (const T*)L.p[2];
  const T* p3 = (const T*)L.p[3];
  switch (L.op) {
    case ENF_OP_SCALESHIFT: {
      const T s = vv[0];  // sum(log.(abs.(f.a))), once per call (run_cpu)
      for (int64_t j = 0; j < nc; ++j) {
        T* y = Y + j * ld;
        for (int64_t d = 0; d < D; ++d) y[d] = std::fma(y[d], p0[d], p1[d]);
        lt[j] = s;
      }
      break;
    }
    case ENF_OP_CENTER_STRETCH:
      for (int64_t j = 0; j < nc; ++j) {
        T* y = Y + j * ld;
        T s = T(0);
        for (int64_t d = 0; d < D; ++d) {
          y[d] = center_stretch_s(y[d], p0[d], p1[d], p2[d]);
          s += center_contract_ladj_s(y[d], p0[d], p1[d], p2[d]);
        }
        lt[j] = -s;
      }
      break;
    case ENF_OP_CENTER_CONTRACT:
      for (int64_t j = 0; j < nc; ++j) {
        T* y = Y + j * ld;
        T s = T(0);
        for (int64_t d = 0; d < D; ++d) {
          s += center_contract_ladj_s(y[d], p0[d], p1[d], p2[d]);
          y[d] = center_contract_s(y[d], p0[d], p1[d], p2[d]);
        }
        lt[j] = s;
      }
      break;
    case ENF_OP_JOHNSON:
      for (int64_t j = 0; j < nc; ++j) {
        T* y = Y + j * ld;
        T s = T(0);
        for (int64_t d = 0; d < D; ++d) {
          const T x = y[d];
          s += johnson_ladj_s(x, p1[d], p2[d], p3[d]);
          y[d] = p0[d] + p1[d] * std::asinh((x - p2[d]) / p3[d]);
        }
        lt[j] = s;
      }
      break;
    case ENF_OP_JOHNSON_INV:
      for (int64_t j = 0; j < nc; ++j) {
        T* y = Y + j * ld;
        T s = T(0);
        for (int64_t d = 0; d < D; ++d) {
          y[d] = p3[d] * std::sinh((y[d] - p0[d]) / p1[d]) + p2[d];
          s += johnson_ladj_s(y[d], p1[d], p2[d], p3[d]);
        }
        lt[j] = -s;
      }
      break;
    case ENF_OP_HOUSEHOLDER:
      for (int64_t j = 0; j < nc; ++j) {
        T* y = Y + j * ld;
        for (int c = 0; c < L.k; ++c) {
          const T* v = p0 + (int64_t)c * D;
          T dot = T(0);
          for (int64_t d = 0; d < D; ++d) dot = std::fma(v[d], y[d], dot);
          const T m2k = T(-2) * (dot / vv[c]);
          for (int64_t d = 0; d < D; ++d) y[d] = std::fma(m2k, v[d], y[d]);
        }
        lt[j] = T(0);
      }
      break;
    default: break;
  }
}

template <typename T>
void run_cpu(int64_t D, int64_t N, const T* X, int64_t ldx, T* Y, int64_t ldy, T* ladj, bool accumulate,
             const std::vector<HostLayer>& layers, int nthreads) {
  const int nl = (int)layers.size();
  // v'v of every reflection vector once per call (the reference's _dot(v, v) per reflection)
  std::vector<std::vector<T>> vv(nl);
  for (int l = 0; l < nl; ++l) {
    if (layers[l].op == ENF_OP_SCALESHIFT) {
      // sum(log.(abs.(f.a))) over a's own length (k = 1: a length-1 `a` broadcast to the D rows), in the
      // reference's order; one value per call instead of one per column block
      const T* a = (const T*)layers[l].p[0];
      T s = T(0);
      for (int64_t d = 0; d < (layers[l].k == 1 ? std::min<int64_t>(D, 1) : D); ++d) s += std::log(std::fabs(a[d]));
      vv[l].assign(1, s);
      continue;
    }
    if (layers[l].op != ENF_OP_HOUSEHOLDER) continue;
    vv[l].resize(layers[l].k);
    for (int c = 0; c < layers[l].k; ++c) {
      const T* v = (const T*)layers[l].p[0] + (int64_t)c * D;
      T s = T(0);
      for (int64_t d = 0; d < D; ++d) s = std::fma(v[d], v[d], s);
      vv[l][c] = s;
    }
  }
  const int64_t nblocks = (N + kBlock - 1) / kBlock;
  // blocks are claimed from a shared counter, so the blocks of a worker that could not be started run on
  // the others (each block's arithmetic is independent of which thread runs it)
  std::atomic<int64_t> next{0};
  auto worker = [&](int) {
    std::vector<T> lt((size_t)nl * kBlock);
    for (int64_t b = next.fetch_add(1); b < nblocks; b = next.fetch_add(1)) {
      const int64_t c0 = b * kBlock, nc = N - c0 < kBlock ? N - c0 : kBlock;
      T* Yb = Y + c0 * ldy;
      const T* Xb = X + c0 * ldx;
      if (Yb != Xb) {
        if (ldx == D && ldy == D) std::memmove(Yb, Xb, (size_t)(D * nc) * sizeof(T));  // dense: one copy
        else
          for (int64_t j = 0; j < nc; ++j) std::memmove(Yb + j * ldy, Xb + j * ldx, (size_t)D * sizeof(T));
      }
      for (int l = 0; l < nl; ++l) layer_block<T>(layers[l], D, nc, Yb, ldy, lt.data() + (size_t)l * kBlock, vv[l]);
      if (ladj) {
        for (int64_t j = 0; j < nc; ++j) {
          T tot = nl > 0 ? lt[(size_t)(nl - 1) * kBlock + j] : T(0);
          for (int l = nl - 2; l >= 0; --l) tot = lt[(size_t)l * kBlock + j] + tot;
          ladj[c0 + j] = accumulate ? ladj[c0 + j] + tot : tot;
        }
      }
    }
  };
  if (nthreads <= 1 || nblocks <= 1) {
    nthreads = 1;
    worker(0);
    return;
  }
  std::vector<std::thread> pool;
  pool.reserve((size_t)nthreads);
  try {
    for (int w = 1; w < nthreads; ++w) pool.emplace_back(worker, w);
  } catch (...) {
    // thread or resource limit: go on with the workers already started (never leave a joinable thread
    // to a destructor, which would terminate the process)
  }
  worker(0);
  for (auto& t : pool) t.join();
}

}  // namespace

enf_status flow_apply_cpu(bool f64, int64_t D, int64_t N, const void* X, int64_t ldx, void* Y, int64_t ldy,
                          void* ladj, int32_t accumulate, const enf_layer* layers, int32_t nlayers, int32_t nthreads) {
  std::vector<HostLayer> hl((size_t)nlayers);
  for (int l = 0; l < nlayers; ++l) {
    hl[l].op = layers[l].op;
    hl[l].k = (layers[l].op == ENF_OP_HOUSEHOLDER || layers[l].op == ENF_OP_SCALESHIFT) ? layers[l].k : 0;
    for (int q = 0; q < 4; ++q) hl[l].p[q] = layers[l].p[q];
  }
  int nt = nthreads;
  if (nt <= 0) {  // every CPU the process may use (usable_cpus: affinity and cgroup quota), but at least
                  // ~2^16 element-steps per thread (a thread's start costs tens of microseconds: config 1's
                  // 1000 x 1 batch runs on the calling thread)
    const int h = usable_cpus();
    int64_t steps = 0;
    for (int l = 0; l < nlayers; ++l) steps += layers[l].op == ENF_OP_HOUSEHOLDER ? 2 * (int64_t)layers[l].k : 1;
    const int64_t work = N * (D > 0 ? D : 1) * (steps > 0 ? steps : 1);
    const int64_t want = 1 + work / (1 << 16);
    nt = h > 0 ? h : 1;
    if (want < nt) nt = (int)want;
  }
  const int64_t nblocks = (N + kBlock - 1) / kBlock;
  if (nt > nblocks) nt = (int)(nblocks > 0 ? nblocks : 1);
  try {
    if (f64) run_cpu<double>(D, N, (const double*)X, ldx, (double*)Y, ldy, (double*)ladj, accumulate != 0, hl, nt);
    else run_cpu<float>(D, N, (const float*)X, ldx, (float*)Y, ldy, (float*)ladj, accumulate != 0, hl, nt);
  } catch (const std::exception& e) {
    return set_error(ENF_ERR_INVALID, e.what());
  }
  return ENF_OK;
}

}  // namespace enf
