// enf_grad_tail.h -- the reduction side of the whitening-loss gradient (config 5), shared by the generic
// gradient kernel (enf_grad.hip) and the fused (J o H)^n kernels (enf_grad_hj.hip).
//
// Every gradient block writes one partial row [loss, gradient...] (double). grad_reduce_kernel sums them and
// finishes the step in ONE launch (round 5; rounds 1-4 ran a slice-sum launch and a one-block tail that walked
// every parameter in turn: 4.7 + 7.8 us per config-5 step):
//
//   block 0            the loss entry: the partial rows' sum, minus N times the flow's constant ladj when the
//                      fused (J o H)^n kernel computed it once instead of per column (enf_grad_hj.hip);
//   block 1 + b        the gradient entries of `upb` consecutive parameter vectors ("units": every vector of the
//                      gradient layout is D entries -- a Householder column, a Johnson gamma, ...): their sums
//                      over the partial rows, then per mode
//     MODE_SUM         the raw sums to tot (a data-parallel rank's contribution, before the cross-rank sum);
//     MODE_OUT         the Householder direction projection (householder_trafo.jl:22-40) and out += (T) sum
//                      (enf_flow_negll_grad, enf_flow_vjp);
//     MODE_STEP        the projection, ADAGrad (Optimisers.update, optimize_whitening.jl:36-42) on the entries in
//                      the trainable runs and the re-normalisation of the Householder columns among the block's
//                      units -- no unit depends on another, so the blocks need no synchronisation.
//
// The sum of an entry is a fixed tree (J lanes per entry, each over partial rows j, j + J, ... with 8
// accumulators, then the J lanes in order): deterministic, and the same in every mode, so the fused
// single-rank step, the one-call data-parallel step on one rank (MODE_SUM, the identity all-reduce, MODE_STEP
// over that one row) and the three-call step (MODE_OUT, all-reduce, enf_whitening_apply) agree bit for bit.
//
// Round 3 measured running the finalisation inside the gradient kernel (a ticket taken after a device-scope
// fence, the last block runs the rest): slower, each device-scope fence writes back and invalidates the XCD's L2
// (profiles/r03_train_sum_tail_ab.txt, r03_train_fused_tail_in_gradient_ab.txt). Round 5 measured it again without
// any fence: rows stored write-through at agent scope, per-row epoch flags, the reduction's blocks reading flags and
// rows with agent-scope loads. Waiting alone cost nothing (32.7 us per config-5 step at B = 1e5, no reduction), the
// reduction alone 5.7 us (38.4, not waiting), both together 61.6 against 40.3 for the two launches
// (profiles/r05/c5_fuse_ab_v2.jsonl): the agent-scope loads of rows other XCDs have just written are slow, and the
// best case (38.4) would save 2 us. The reduction stays a launch of its own.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "enf_internal.h"
#include "enf_train.h"

namespace enf {

constexpr int kMaxGradSteps = 32;
// rows of totals the workspace reserves after the partial rows (one is used: tot, then the constant ladj)
constexpr int kSumSlices = 8;
constexpr int kRedThreads = 512;
constexpr int kRedMaxEntries = 1024;  // entries of one reduction block: max(D, 32) <= 1024

enum ReduceMode { MODE_SUM = 0, MODE_OUT = 1, MODE_STEP = 2 };

struct ReduceArgs {
  const double* partial;  // [nblocks][1 + nparams] (nblocks == 1: an already reduced row)
  int32_t nblocks;
  int32_t nparams;
  int32_t D;
  int32_t nh;         // Householder columns
  int32_t skip_loss;  // MODE_OUT for enf_flow_vjp: out has no loss slot (out[i] += tot[1 + i])
  int32_t upb;        // units (vectors of D entries) per reduction block
  const double* ctot;  // nullable: the flow's constant ladj per column; the loss gets -nloc * ctot
  int64_t nloc;
  void* out;    // MODE_OUT
  double* tot;  // MODE_SUM: 1 + nparams
  // per Householder column: offset of its gradient vector and its device column pointer
  int32_t hoff[kMaxGradSteps];
  const void* hcol[kMaxGradSteps];
};

// MODE_STEP: the rest of a single-rank optimize_whitening step (enf_whitening_step) / the update half of a
// data-parallel one (enf_whitening_step_dp after the cross-rank sum).
struct StepArgs {
  void* theta;
  void* acc;
  double* loss_out;
  double scale, eta, eps;
  int64_t D, nsamp;
  int32_t nruns, nhb;
  int64_t runs[kMaxStepRuns][2];
  int64_t hb[kMaxStepHB][3];  // offset, k, ldv
};

inline int reduce_units_per_block(int64_t D) { return D >= 32 ? 1 : (int)(32 / D); }
inline int reduce_grid(int64_t D, int64_t nparams) {
  const int64_t units = nparams / D;
  const int upb = reduce_units_per_block(D);
  return 1 + (int)((units + upb - 1) / upb);
}

// Sum of entry column c over the partial rows j, j + J, j + 2J, ... (rows of n doubles), with up to kBatch loads in
// flight per batch (the rows were written by the previous launch: every batch is one round trip to the caches),
// added into 8 accumulators in a fixed order.
constexpr int kBatch = 32;
__device__ __forceinline__ double rows_sum(const double* __restrict__ P, int nb, int64_t n, int64_t c, int j, int J) {
  double s8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int b0 = j; b0 < nb; b0 += kBatch * J) {
    double v[kBatch];
#pragma unroll
    for (int k = 0; k < kBatch; ++k) {
      const int b = b0 + k * J;
      v[k] = b < nb ? P[(int64_t)b * n + c] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kBatch; ++k) s8[k & 7] += v[k];
  }
  return ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
}

// Sums entries [e0, e0 + E) of the rows (column offset c0 + i) into gl[0 .. E) (LDS), block-wide: J = kRedThreads / E
// lanes per entry over interleaved rows, then the J partial sums in order. The lanes are kRedThreads virtual threads
// whatever the block size (a block of fewer threads runs several), so every caller sums in the same order.
// nblocks == 1: the row itself.
__device__ __forceinline__ void block_sums(const ReduceArgs& r, int64_t c0, int E, double* __restrict__ gl,
                                           double* __restrict__ red) {
  const int tid = threadIdx.x, NT = blockDim.x;
  const int64_t n = 1 + (int64_t)r.nparams;
  const double* P = r.partial;
  if (r.nblocks == 1) {
    for (int i = tid; i < E; i += NT) gl[i] = P[c0 + i];
    __syncthreads();
    return;
  }
  if (2 * E <= kRedThreads) {
    const int J = kRedThreads / E;
#pragma unroll 1
    for (int vt = tid; vt < kRedThreads; vt += NT) {
      const int i = vt % E, j = vt / E;
      if (j < J) red[j * E + i] = rows_sum(P, r.nblocks, n, c0 + i, j, J);
    }
    __syncthreads();
    for (int i = tid; i < E; i += NT) {
      double s = red[i];
      for (int q = 1; q < J; ++q) s += red[q * E + i];
      gl[i] = s;
    }
  } else {
    for (int i = tid; i < E; i += NT) gl[i] = rows_sum(P, r.nblocks, n, c0 + i, 0, 1);
  }
  __syncthreads();
}

// Householder index of the unit starting at gradient offset off, or -1
__device__ __forceinline__ int unit_householder(const ReduceArgs& r, int64_t off) {
  for (int h = 0; h < r.nh; ++h)
    if (r.hoff[h] == off) return h;
  return -1;
}

// dS/dv from the direction sums G of one column (in gl, D entries) and the column v (vc, double):
//   dS/dw = -sqrt2 G, dS/dv = (dS/dw - w (dS/dw . w)) / |v|, w = v / |v|  (householder_trafo.jl:22-40)
// by one wave (sums over the lanes: d = lane, lane + 64, ..., then the xor tree).
// project_lane: the same for D <= 64 with this lane's entry (g, vc) in registers (zeros past the column): the column
// is the group of lanes the xor tree of lane_sum(., D) spans, so a wave can hold several columns of a power-of-two D
// side by side (block_step_update), and every caller runs these same operations
__device__ __forceinline__ double project_lane(double g, double vc, int D) {
  double vv = 0.0;
  vv += vc * vc;
  vv = lane_sum(vv, D);
  const double nrm = sqrt(vv);
  double wd = 0.0;
  wd += -1.4142135623730951 * g * (vc / nrm);
  wd = lane_sum(wd, D);
  return (-1.4142135623730951 * g - (vc / nrm) * wd) / nrm;
}
__device__ __forceinline__ void project_column(double* __restrict__ g, const double* __restrict__ vc, int D, int lane) {
  if (D <= 64) {
    const double r = project_lane(lane < D ? g[lane] : 0.0, lane < D ? vc[lane] : 0.0, D);
    if (lane < D) g[lane] = r;
    return;
  }
  double vv = 0.0;
  for (int d = lane; d < D; d += 64) vv += vc[d] * vc[d];
  vv = lane_sum(vv, D);
  const double nrm = sqrt(vv);
  double wd = 0.0;
  for (int d = lane; d < D; d += 64) wd += -1.4142135623730951 * g[d] * (vc[d] / nrm);
  wd = lane_sum(wd, D);
  for (int d = lane; d < D; d += 64) g[d] = (-1.4142135623730951 * g[d] - (vc[d] / nrm) * wd) / nrm;
}

// LinearAlgebra.normalize! of one column held in LDS (src/householder_trafo.jl:135-139), by one wave: the sum of
// squares in double over d = lane, lane + 64, ..., the xor tree, then v *= (T)(1/sqrt) -- normalize_column's
// arithmetic (enf_train.h), so the separate enf_householder_normalize call rounds the same
template <typename T>
__device__ __forceinline__ T normalize_lane(T v, int D) {  // D <= 64, as project_lane
  double ss = 0.0;
  ss += (double)v * (double)v;
  ss = lane_sum(ss, D);
  const T inv = (T)(1.0 / sqrt(ss));
  return v * inv;
}
template <typename T>
__device__ __forceinline__ void normalize_lds(T* __restrict__ v, int D, int lane) {
  if (D <= 64) {
    const T r = normalize_lane<T>(lane < D ? v[lane] : (T)0, D);
    if (lane < D) v[lane] = r;
    return;
  }
  double ss = 0.0;
  for (int d = lane; d < D; d += 64) ss += (double)v[d] * (double)v[d];
  ss = lane_sum(ss, D);
  const T inv = (T)(1.0 / sqrt(ss));
  for (int d = lane; d < D; d += 64) v[d] *= inv;
}

// The update of a whole flow by ONE block (the single-block fused step, round 5): tot (LDS: 1 + np doubles, the
// block's loss and gradient sums) -> loss, Householder projection, ADAGrad, re-normalisation -- the operations and
// roundings of grad_reduce_kernel's MODE_STEP over one partial row, so the one-launch and the two-launch steps agree
// bit for bit. scratch (LDS, 16-byte aligned): np doubles + 2 np T + np ints.
// What the update of entry i reads that does not depend on the gradient: the Householder column value, the
// entry's flags (bit 0 trainable, bit 1 in a normalised column), theta and the ADAGrad state. The one-block step
// loads it for i = threadIdx.x before its tiles (round 5), so the loads' round trip is off the step's critical path.
template <typename T>
struct StepPre {
  double hv = 0.0;
  T th = (T)0, ac = (T)0;
  int f = 0;
};
template <typename T>
__device__ __forceinline__ StepPre<T> step_prefetch(int64_t i, int D, const ReduceArgs& r, const StepArgs& s) {
  StepPre<T> p;
  const int64_t uo = (i / D) * D;
  const int h = unit_householder(r, uo);
  if (h >= 0) p.hv = (double)((const T*)r.hcol[h])[i % D];
  for (int q = 0; q < s.nruns; ++q) p.f |= (i >= s.runs[q][0] && i < s.runs[q][1]) ? 1 : 0;
  for (int q = 0; q < s.nhb; ++q) {
    const int64_t rel = uo - s.hb[q][0];
    if (rel >= 0 && rel % s.hb[q][2] == 0 && rel / s.hb[q][2] < s.hb[q][1]) p.f |= 2;
  }
  if (p.f) p.th = ((const T*)s.theta)[i];
  if (p.f & 1) p.ac = ((const T*)s.acc)[i];
  return p;
}

// The update with one entry per thread (entry i = threadIdx.x) for a power-of-two D <= 64 (and np <= the block's
// threads, have_pre): the D lanes of a column unit are one group of lane_sum's xor tree, so each unit is finished by
// its own lanes -- projection, ADAGrad, re-normalisation and the stores -- with the operations of
// block_step_update's phases and no block barrier. g: entry i's gradient sum (0 past np).
__device__ __forceinline__ bool step_update_lanes(bool have_pre, int D) { return have_pre && D <= 64 && (D & (D - 1)) == 0; }
template <typename T>
__device__ __forceinline__ void step_update_lane(double g, int64_t np, int D, const ReduceArgs& r, const StepArgs& s,
                                                 const StepPre<T>& pre, double scale) {
  const int64_t i = threadIdx.x;
  const bool act = i < np;
  const bool hh = act && unit_householder(r, (i / D) * D) >= 0;
  const double gp = project_lane(g, pre.hv, D);
  if (hh) g = gp;
  T th = pre.th, ac = pre.ac;
  if (act && (pre.f & 1)) adagrad_update<T>(th, ac, (T)g, (T)scale, (T)s.eta, (T)s.eps);
  const T tn = normalize_lane<T>(th, D);
  if (act && (pre.f & 2)) th = tn;
  if (act && pre.f) ((T*)s.theta)[i] = th;
  if (act && (pre.f & 1)) ((T*)s.acc)[i] = ac;
}

// pre: this thread's step_prefetch(threadIdx.x) when have_pre (np <= blockDim.x), else loaded here. loss_out, nsamp
// and scale: this minibatch's (s.loss_out / s.nsamp / s.scale for one step; the epoch kernel's j-th batch).
template <typename T>
__device__ __forceinline__ void block_step_update(double* __restrict__ tot, int64_t np, int D, const ReduceArgs& r,
                                                  const StepArgs& s, unsigned char* __restrict__ scratch,
                                                  const StepPre<T>& pre, bool have_pre, double* loss_out,
                                                  int64_t nsamp, double scale) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6, NT = blockDim.x;
  double* vcol = reinterpret_cast<double*>(scratch);
  T* thl = reinterpret_cast<T*>(vcol + np);
  T* acl = thl + np;
  int* flags = reinterpret_cast<int*>(acl + np);
  double* gl = tot + 1;
  if (tid == 0) *loss_out = (double)((T)tot[0] / (T)nsamp);
  if (step_update_lanes(have_pre, D)) {
    step_update_lane<T>(tid < np ? gl[tid] : 0.0, np, D, r, s, pre, scale);
    return;
  }
  for (int64_t i = tid; i < np; i += NT) {
    const StepPre<T> p = have_pre ? pre : step_prefetch<T>(i, D, r, s);
    vcol[i] = p.hv;
    flags[i] = p.f;
    thl[i] = p.th;
    acl[i] = p.ac;
  }
  __syncthreads();
  const int64_t units = np / D;
  for (int64_t u = wave; u < units; u += nw)
    if (unit_householder(r, u * D) >= 0) project_column(gl + u * D, vcol + u * D, D, lane);  // wave-uniform
  __syncthreads();
  for (int64_t i = tid; i < np; i += NT)
    if (flags[i] & 1) adagrad_update<T>(thl[i], acl[i], (T)gl[i], (T)scale, (T)s.eta, (T)s.eps);
  __syncthreads();
  for (int64_t u = wave; u < units; u += nw)
    if (flags[u * D] & 2) normalize_lds<T>(thl + u * D, D, lane);  // wave-uniform
  __syncthreads();
  T* th = (T*)s.theta;
  T* ac = (T*)s.acc;
  for (int64_t i = tid; i < np; i += NT) {
    const int f = flags[i];
    if (f) th[i] = thl[i];
    if (f & 1) ac[i] = acl[i];
  }
}

// LDS of one reduction block: red[kRedThreads] doubles, then gl / vcol (E doubles each), thl / acl (E T each,
// MODE_STEP), flags (E ints); red_lds_bytes(E) in all
template <typename T>
struct RedLds {
  double* red;
  double* gl;
  double* vcol;
  T* thl;
  T* acl;
  int* flags;
  __device__ static RedLds at(unsigned char* base, int E) {
    RedLds l;
    l.red = reinterpret_cast<double*>(base);
    l.gl = l.red + kRedThreads;
    l.vcol = l.gl + E;
    l.thl = reinterpret_cast<T*>(l.vcol + E);
    l.acl = l.thl + E;
    l.flags = reinterpret_cast<int*>(l.acl + E);
    return l;
  }
};
template <typename T>
__host__ __device__ constexpr size_t red_lds_bytes(int E) {
  return (size_t)kRedThreads * 8 + (size_t)E * (16 + 2 * sizeof(T) + 4);
}

// Reduction block `bid` of the grid described in the file comment, any block size >= 64 (the entry sums are fixed
// trees of kRedThreads virtual lanes, block_sums). Returns after its last store; no grid synchronisation.
template <typename T, int MODE>
__device__ __forceinline__ void reduce_block(const ReduceArgs& r, const StepArgs& s, int bid, const RedLds<T>& L) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, NT = blockDim.x, nw = NT >> 6;
  const int64_t n = 1 + (int64_t)r.nparams;
  if (bid == 0) {  // the loss entry: one wave
    if (tid < 64) {
      double v;
      if (r.nblocks == 1) {
        v = r.partial[0];
      } else {
        v = rows_sum(r.partial, r.nblocks, n, 0, tid, 64);
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
      }
      if (tid == 0) {
        if (r.ctot) v -= (double)r.nloc * *r.ctot;
        if constexpr (MODE == MODE_SUM) r.tot[0] = v;
        else if constexpr (MODE == MODE_OUT) {
          if (!r.skip_loss) ((T*)r.out)[0] += (T)v;
        } else {
          *s.loss_out = (double)((T)v / (T)s.nsamp);
        }
      }
    }
    return;
  }
  const int D = r.D;
  const int64_t units = r.nparams / D;
  const int64_t u0 = (int64_t)(bid - 1) * r.upb;
  const int64_t u1 = u0 + r.upb < units ? u0 + r.upb : units;
  const int64_t e0 = u0 * D;  // first gradient entry of the block
  const int E = (int)((u1 - u0) * D);
  double* __restrict__ gl = L.gl;
  double* __restrict__ vcol = L.vcol;
  T* __restrict__ thl = L.thl;
  T* __restrict__ acl = L.acl;
  int* __restrict__ flags = L.flags;
  // What does not depend on the sums is loaded first, into registers (one entry per thread when E <= the block's
  // threads), so its round trip overlaps the sums' loads: the Householder columns, theta and the ADAGrad state.
  auto prefetch = [&](int i, double& hv, T& thv, T& acv, int& f) {
    hv = 0.0;
    thv = acv = (T)0;
    f = 0;
    const int64_t e = e0 + i;
    const int64_t uo = e0 + (i / D) * D;
    const int h = unit_householder(r, uo);
    if (h >= 0) hv = (double)((const T*)r.hcol[h])[i % D];
    if constexpr (MODE == MODE_STEP) {
      for (int q = 0; q < s.nruns; ++q) f |= (e >= s.runs[q][0] && e < s.runs[q][1]) ? 1 : 0;
      for (int q = 0; q < s.nhb; ++q) {
        const int64_t rel = uo - s.hb[q][0];
        if (rel >= 0 && rel % s.hb[q][2] == 0 && rel / s.hb[q][2] < s.hb[q][1]) f |= 2;
      }
      if (f) thv = ((const T*)s.theta)[e];
      if (f & 1) acv = ((const T*)s.acc)[e];
    }
  };
  auto stage = [&](int i, double hv, T thv, T acv, int f) {
    vcol[i] = hv;
    if constexpr (MODE == MODE_STEP) {
      flags[i] = f;
      thl[i] = thv;
      acl[i] = acv;
    }
  };
  if constexpr (MODE == MODE_SUM) {
    block_sums(r, 1 + e0, E, gl, L.red);
  } else if (E <= NT) {  // (block-uniform) the prefetched values are staged after the sums' loads
    double hv = 0.0;
    T thv = (T)0, acv = (T)0;
    int f = 0;
    if (tid < E) prefetch(tid, hv, thv, acv, f);
    block_sums(r, 1 + e0, E, gl, L.red);
    if (tid < E) stage(tid, hv, thv, acv, f);
  } else {
    for (int i = tid; i < E; i += NT) {
      double hv;
      T thv, acv;
      int f;
      prefetch(i, hv, thv, acv, f);
      stage(i, hv, thv, acv, f);
    }
    block_sums(r, 1 + e0, E, gl, L.red);
  }
  if constexpr (MODE == MODE_SUM) {
    for (int i = tid; i < E; i += NT) r.tot[1 + e0 + i] = gl[i];
    return;
  }
  __syncthreads();  // (the staged values)
  // Householder direction projection, one wave per column unit
  for (int64_t u = u0 + wave; u < u1; u += nw) {
    if (unit_householder(r, u * D) < 0) continue;  // wave-uniform
    const int o = (int)((u - u0) * D);
    project_column(gl + o, vcol + o, D, lane);
  }
  __syncthreads();
  if constexpr (MODE == MODE_OUT) {
    T* out = (T*)r.out;
    const int64_t base = r.skip_loss ? 0 : 1;
    for (int i = tid; i < E; i += NT) out[base + e0 + i] += (T)gl[i];
    return;
  }
  if constexpr (MODE == MODE_STEP) {
    for (int i = tid; i < E; i += NT)
      if (flags[i] & 1) adagrad_update<T>(thl[i], acl[i], (T)gl[i], (T)s.scale, (T)s.eta, (T)s.eps);
    __syncthreads();
    for (int64_t u = u0 + wave; u < u1; u += nw) {
      const int o = (int)((u - u0) * D);
      if (flags[o] & 2) normalize_lds<T>(thl + o, D, lane);  // wave-uniform
    }
    __syncthreads();
    T* th = (T*)s.theta;
    T* ac = (T*)s.acc;
    for (int i = tid; i < E; i += NT) {
      const int f = flags[i];
      if (f) th[e0 + i] = thl[i];
      if (f & 1) ac[e0 + i] = acl[i];
    }
  }
}

template <typename T, int MODE>
__global__ __launch_bounds__(kRedThreads) void grad_reduce_kernel(ReduceArgs r, StepArgs s) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[red_lds_bytes<T>(kRedMaxEntries)];
  const int upb_e = r.D * r.upb;  // entries of a full block
  reduce_block<T, MODE>(r, s, blockIdx.x, RedLds<T>::at(lds, upb_e));
}

}  // namespace enf
