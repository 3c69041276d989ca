// enf_flow_wy.hip -- chained HouseholderTrafo on the matrix cores.
//
// A HouseholderTrafo with a D x k matrix V applies k reflections in column order,
// y = H_k ... H_1 x with H_c = I - 2 v_c v_c' / (v_c'v_c) (chained_householder_trafo,
// src/householder_trafo.jl:71-78). Applied reflection by reflection that is 2k FMAs per element
// plus k column reductions; for large k it is cheaper to form the orthogonal product
// Q = H_k ... H_1 once per block (in double) and apply it as a D x D matrix product, Y = Q X,
// on the MFMA units: fp32 v_mfma_f32_32x32x2_f32 (exact f32 FMA chains), fp64
// v_mfma_f64_16x16x4_f64. ladj of a Householder step is 0 (householder_trafo.jl:157-160).
//
// Layout. A lane owns R = D / KH contiguous rows of one column (KH = lanes per column: 2 for the
// fp32 32x32x2 MFMA, 4 for the fp64 16x16x4 MFMA); lane l holds column l % COLS, rows
// R*(l / COLS) ... R*(l / COLS) + R - 1, loaded and stored as R*sizeof(T)/16 16-byte vectors.
// The MFMA's k index runs over the lane's own rows: step s takes k = R*q + s from part q, and the
// A operand (the rows of Q) is permuted so that accumulator register r of row block m lands on row
// R*q + RPB*m + r -- the product is produced in exactly the layout it was consumed in, so several
// dense steps and the elementwise steps of the rest of the flow (Johnson, ScaleShift, Center, single
// reflections: enf_steps.h bodies on one 16-byte fragment at a time) run back to back in registers.
// The A operand image of each dense step lives in LDS as [block m][s / V][lane][V] (one 16-byte
// read per V MFMAs).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <type_traits>

#include "enf_frag.h"
#include "enf_internal.h"
#include "enf_steps.h"

namespace enf {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <typename T, int D>
struct WYL;

// fp32: v_mfma_f32_32x32x2_f32. C row slot of (part q, register r): (r&3) + 8(r>>2) + 4q.
template <int D>
struct WYL<float, D> {
  static constexpr int COLS = 32, KH = 2, RPB = 16, V = 4;
  using Acc = f32x16;
  __device__ static __forceinline__ Acc mfma(float a, float b, Acc c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
  __host__ __device__ static constexpr int slot(int q, int r) { return (r & 3) + 8 * (r >> 2) + 4 * q; }
};

// fp64: v_mfma_f64_16x16x4_f64. C row slot of (part q, register r): q + 4r.
template <int D>
struct WYL<double, D> {
  static constexpr int COLS = 16, KH = 4, RPB = 4, V = 2;
  using Acc = f64x4;
  __device__ static __forceinline__ Acc mfma(double a, double b, Acc c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  __host__ __device__ static constexpr int slot(int q, int r) { return q + 4 * r; }
};

template <typename T, int D>
struct WYC : WYL<T, D> {
  using B = WYL<T, D>;
  static constexpr int R = D / B::KH;       // rows per lane
  static constexpr int NB = R / B::RPB;     // MFMA row blocks
  static constexpr int NF = R / B::V;       // 16-byte fragments per lane
  static_assert(NB * B::RPB * B::KH == D && NB >= 1, "D must be a multiple of the MFMA tile");
};

// image index of Q[row][col] in the A-operand layout [m][s / V][lane][V]
template <typename T, int D>
__device__ __forceinline__ int a_index(int row, int col) {
  using W = WYC<T, D>;
  constexpr int R = W::R, RPB = W::RPB, V = W::V;
  const int q = row / R, m = (row % R) / RPB, r = row % RPB;
  const int lane = W::slot(q, r) + W::COLS * (col / R);
  const int s = col % R;
  return ((m * (R / V) + s / V) * 64 + lane) * V + s % V;
}

// Block prologue of one dense step: Q = H_k ... H_1 in double, built by right-multiplying the
// identity with H_k, ..., H_1 (Q <- Q H_c = Q - (Q vh) vh', vh = v_c sqrt(2 / v_c'v_c)). Thread t
// owns D / P entries of row t / P (P = 256 / D threads per row, adjacent lanes), so the row dot
// Q vh is an in-lane sum plus a DPP group sum. V is staged in the step's own LDS record area
// (k * D <= D * D values of T) and overwritten by the A image at the end.
template <typename T, int D>
__device__ void build_dense(const FlowArgs& a, const Step& st, T* __restrict__ img, double* __restrict__ hs) {
  constexpr int P = 256 / D, NC = D / P;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int k = st.col >> 16;  // reflections [start, start + k) of V, k <= D
  const T* __restrict__ Vg = (const T*)a.layers[st.layer].p[0] + (int64_t)(st.col & 0xFFFF) * D;
  for (int i = t; i < k * D; i += 256) img[i] = Vg[i];
  __syncthreads();
  for (int c = wave; c < k; c += 4) {
    double vv = 0.0;
    for (int d = lane; d < D; d += 64) vv += (double)img[c * D + d] * (double)img[c * D + d];
    for (int m = 32; m >= 1; m >>= 1) vv += __shfl_xor(vv, m);
    if (lane == 0) hs[c] = sqrt(2.0 / vv);
  }
  __syncthreads();
  const int row = t / P, c0 = (t % P) * NC;
  double q[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) q[i] = (c0 + i == row) ? 1.0 : 0.0;
  for (int c = k - 1; c >= 0; --c) {
    const double h = hs[c];
    double vh[NC];
    double p0 = 0.0, p1 = 0.0;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      vh[i] = (double)img[c * D + c0 + i] * h;
      if (i & 1) p1 = fma(q[i], vh[i], p1);
      else p0 = fma(q[i], vh[i], p0);
    }
    const double dot = group_sum<P>(p0 + p1);
#pragma unroll
    for (int i = 0; i < NC; ++i) q[i] = fma(-dot, vh[i], q[i]);
  }
  __syncthreads();  // every thread is done reading the staged V
#pragma unroll
  for (int i = 0; i < NC; ++i) img[a_index<T, D>(row, c0 + i)] = (T)q[i];
}

// sum over the KH lanes of a column
template <typename T, int KH, int COLS>
__device__ __forceinline__ T part_sum(T v) {
  if constexpr (KH >= 2) v += __shfl_xor(v, COLS);
  if constexpr (KH >= 4) v += __shfl_xor(v, 2 * COLS);
  return v;
}

// Y = Q x for the lane's rows: NB accumulators, R k-steps each, A read from LDS per V steps.
template <typename T, int D>
__device__ __forceinline__ void dense_apply(const T* __restrict__ img, T (&x)[WYC<T, D>::NF][1][WYC<T, D>::V]) {
  using W = WYC<T, D>;
  constexpr int NB = W::NB, R = W::R, V = W::V, RPB = W::RPB;
  const int lane = threadIdx.x & 63;
  typename W::Acc acc[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) acc[m] = typename W::Acc{};
#pragma unroll
  for (int sv = 0; sv < R / V; ++sv) {
    T av[NB][V];
#pragma unroll
    for (int m = 0; m < NB; ++m) lds_vec<T, V>(img + ((m * (R / V) + sv) * 64 + lane) * V, av[m]);
#pragma unroll
    for (int e = 0; e < V; ++e)
#pragma unroll
      for (int m = 0; m < NB; ++m) acc[m] = W::mfma(av[m][e], x[sv][0][e], acc[m]);
  }
  // Non-finite input: reflection by reflection (the reference), an Inf makes the first dot +-Inf,
  // its own row Inf - Inf = NaN and, from the second reflection on, every row NaN; Q x would give
  // a mix of +-Inf and NaN. nf = sum of x*0 over the column is 0, or NaN if any input is Inf/NaN,
  // and adding it reproduces the all-NaN column (a step holds >= 2 reflections unless it is the
  // tail chunk of a longer chain, whose input is then already all-finite or all-NaN).
  T nf = (T)0;
#pragma unroll
  for (int f = 0; f < R / V; ++f)
#pragma unroll
    for (int e = 0; e < V; ++e) nf = fma(x[f][0][e], (T)0, nf);
  nf = part_sum<T, W::KH, W::COLS>(nf);
#pragma unroll
  for (int m = 0; m < NB; ++m)
#pragma unroll
    for (int r = 0; r < RPB; ++r) {
      const int row = m * RPB + r;
      x[row / V][0][row % V] = acc[m][r] + nf;
    }
}

// one reflection y = x - vh (vh'x) (householder_trafo.jl:8-11) on the lane's R rows
template <typename T, int D>
__device__ __forceinline__ void reflect(const T* __restrict__ r, int g0, T (&x)[WYC<T, D>::NF][1][WYC<T, D>::V]) {
  using W = WYC<T, D>;
  constexpr int NF = W::NF, V = W::V;
  T vh[NF][V];
  T p0 = (T)0, p1 = (T)0;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    lds_vec<T, V>(r + (g0 + f) * V, vh[f]);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      if (f & 1) p1 = fma(vh[f][e], x[f][0][e], p1);
      else p0 = fma(vh[f][e], x[f][0][e], p0);
    }
  }
  const T dot = part_sum<T, W::KH, W::COLS>(p0 + p1);
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int e = 0; e < V; ++e) x[f][0][e] = fma(-dot, vh[f][e], x[f][0][e]);
}

template <typename T, int D, int LM>
__device__ __forceinline__ void wy_steps(const FlowArgs& a, const T* __restrict__ rec, T ctot, int64_t col0,
                                        T (&x)[WYC<T, D>::NF][1][WYC<T, D>::V]) {
  using W = WYC<T, D>;
  constexpr int NF = W::NF, V = W::V;
  constexpr bool LADJ = LM > 0;
  const int lane = threadIdx.x & 63;
  const int q = lane / W::COLS;
  const int g0 = W::R * q / V;  // record group of the lane's first fragment
  T acc[1][1] = {{(T)0}};
  for (int s = 0; s < a.nsteps; ++s) {
    const int desc = a.desc[s];
    const int op = desc & 15;
    const T* __restrict__ r = rec + (desc >> 4);
    if (op == OP_DENSE) {
      dense_apply<T, D>(r, x);
    } else if (op == OP_HOUSEHOLDER) {
      reflect<T, D>(r, g0, x);
    } else {
      const int wv = record_width(op) * V;
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const T* __restrict__ rf = r + (g0 + f) * wv;
        if (op == OP_JOHNSON) step_johnson<T, D, 1, LADJ>(x[f], acc, rf);
        else if (op == OP_JOHNSON_INV) step_johnson_inv<T, D, 1, LADJ>(x[f], acc, rf);
        else if (op == OP_SCALESHIFT) step_scaleshift<T, D, 1>(x[f], rf);
        else if (op == OP_CENTER_STRETCH) step_center_stretch<T, D, 1, LADJ>(x[f], acc, rf);
        else step_center_contract<T, D, 1, LADJ>(x[f], acc, rf);
      }
    }
  }
  const int64_t col = col0 + lane % W::COLS;
  const bool valid = col < a.N;
  if (LADJ) {
    const T tot = part_sum<T, W::KH, W::COLS>(acc[0][0]);
    if (valid && q == 0) {
      T* __restrict__ ladj = (T*)a.ladj;
      const T v = fma(Unit<T>::v, tot, ctot);
      ladj[col] = LM == 2 ? ladj[col] + v : v;
    }
  }
}

// Global <-> MFMA layout through a per-wave LDS image. HBM is read and written with fully
// coalesced wave-instructions (instruction f, lane l: 16-byte chunk f*64 + l of the contiguous
// COLS x D tile); the image holds the tile in MFMA layout, entry (fragment f', lane') at
// f' * PITCH + lane' (PITCH = 65 entries: the chunks a lane writes in one instruction land in
// different banks). (A lane reading its own R contiguous rows straight from HBM touches 16 of every
// R*sizeof(T) bytes per instruction: measured 0.53 / 0.47 of HBM peak at D = 32 / 64, fp32.)
template <typename T, int D>
struct WYT {
  using W = WYC<T, D>;
  static constexpr int NF = W::NF, PITCH = 65;
  static constexpr int CPC = D * (int)sizeof(T) / 16;  // 16-byte chunks per column
  static constexpr size_t kBytesPerWave = (size_t)NF * PITCH * 16;
  __device__ static __forceinline__ int entry(int c) {  // chunk c of the tile -> image entry
    const int j = c / CPC, cc = c % CPC;
    return (cc % NF) * PITCH + j + W::COLS * (cc / NF);
  }
};

template <typename T, int D>
__device__ __forceinline__ void wy_load(const FlowArgs& a, int64_t col0, u32x4 (&raw)[WYT<T, D>::NF]) {
  using Tt = WYT<T, D>;
  const int lane = threadIdx.x & 63;
  const u32x4* __restrict__ X = reinterpret_cast<const u32x4*>((const T*)a.X + col0 * D);
#pragma unroll
  for (int f = 0; f < Tt::NF; ++f) {
    const int c = f * 64 + lane;
    if (col0 + c / Tt::CPC < a.N) raw[f] = __builtin_nontemporal_load(X + c);
    else raw[f] = u32x4{0u, 0u, 0u, 0u};
  }
}

template <typename T, int D>
__device__ __forceinline__ void wy_to_mfma(u32x4* __restrict__ img, const u32x4 (&raw)[WYT<T, D>::NF],
                                           T (&x)[WYC<T, D>::NF][1][WYC<T, D>::V]) {
  using Tt = WYT<T, D>;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int f = 0; f < Tt::NF; ++f) img[Tt::entry(f * 64 + lane)] = raw[f];
#pragma unroll
  for (int f = 0; f < Tt::NF; ++f) {
    const u32x4 v = img[f * Tt::PITCH + lane];
    __builtin_memcpy(&x[f][0][0], &v, 16);
  }
}

template <typename T, int D>
__device__ __forceinline__ void wy_store(const FlowArgs& a, int64_t col0, u32x4* __restrict__ img,
                                         const T (&x)[WYC<T, D>::NF][1][WYC<T, D>::V]) {
  using Tt = WYT<T, D>;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int f = 0; f < Tt::NF; ++f) {
    u32x4 v;
    __builtin_memcpy(&v, &x[f][0][0], 16);
    img[f * Tt::PITCH + lane] = v;
  }
  u32x4* __restrict__ Y = reinterpret_cast<u32x4*>((T*)a.Y + col0 * D);
#pragma unroll
  for (int f = 0; f < Tt::NF; ++f) {
    const int c = f * 64 + lane;
    const u32x4 v = img[Tt::entry(c)];
    if (col0 + c / Tt::CPC < a.N) __builtin_nontemporal_store(v, Y + c);
  }
}

template <typename T, int D, int LM>
__global__ __launch_bounds__(256) void flow_wy_kernel(FlowArgs a) {
  using W = WYC<T, D>;
  using Tt = WYT<T, D>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* stepc = reinterpret_cast<double*>(smem);
  double* ctotp = stepc + kMaxSteps;
  double* hs = reinterpret_cast<double*>(smem + kLdsScalars);  // dense-prologue scratch (the stage area)
  T* rec = reinterpret_cast<T*>(smem + kLdsHeader);
  (void)ctotp;
  ENF_KARG_CHECK(a);
  const double ctot_d = build_program<T, D, Frag<T, D>::V>(a, rec, stepc);
  for (int s = 0; s < a.nsteps; ++s)
    if (a.steps[s].op == OP_DENSE) {
      build_dense<T, D>(a, a.steps[s], rec + a.steps[s].off, hs);
      __syncthreads();
    }
  const T ctot = (T)ctot_d;
  // the waves' transpose images follow the records (program_lds_bytes, 16-byte aligned)
  u32x4* img = reinterpret_cast<u32x4*>(smem + a.img_off + (threadIdx.x >> 6) * Tt::kBytesPerWave);
  const int64_t ntiles = (a.N + W::COLS - 1) / W::COLS;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t t = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u32x4 raw[Tt::NF];
  T x[W::NF][1][W::V];
  if (t < ntiles) {
    wy_load<T, D>(a, t * W::COLS, raw);
    wy_to_mfma<T, D>(img, raw, x);
  }
  for (; t < ntiles; t += nw) {
    const bool more = t + nw < ntiles;
    if (more) wy_load<T, D>(a, (t + nw) * W::COLS, raw);  // next tile in flight
    wy_steps<T, D, LM>(a, rec, ctot, t * W::COLS, x);
    wy_store<T, D>(a, t * W::COLS, img, x);
    if (more) wy_to_mfma<T, D>(img, raw, x);
  }
}

template <typename T, int D, int LM>
hipError_t launch_wy_t(const FlowArgs& a, size_t lds, hipStream_t st, const DeviceInfo& dev) {
  const void* k = reinterpret_cast<const void*>(&flow_wy_kernel<T, D, LM>);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  int64_t blocks = 0;
  hipError_t e = frag_grid(k, a.N, (int64_t)WYL<T, D>::COLS * 4, lds, dev, &blocks);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((flow_wy_kernel<T, D, LM>), dim3((unsigned)blocks), dim3(256), lds, st, a);
  return hipGetLastError();
}

template <typename T, int LM>
hipError_t dispatch_wy(const FlowArgs& a0, size_t lds, hipStream_t st, const DeviceInfo& dev) {
  FlowArgs a = a0;
  a.img_off = (int32_t)((lds + 15) / 16 * 16);
#if ENF_BOUNDS
  a.csum = flow_args_csum(a);
#endif
  if (a.D == 32) return launch_wy_t<T, 32, LM>(a, a.img_off + 4 * WYT<T, 32>::kBytesPerWave, st, dev);
  if (a.D == 64) return launch_wy_t<T, 64, LM>(a, a.img_off + 4 * WYT<T, 64>::kBytesPerWave, st, dev);
  return hipErrorInvalidValue;
}

}  // namespace

bool wy_supported(int64_t D, bool frag) { return frag && (D == 32 || D == 64); }

// ENF_WY_MIN_K: smallest reflection count of a chained HouseholderTrafo that runs as a dense product
int wy_min_k() {
  static const int k = ENF_KNOB("ENF_WY_MIN_K", 8);
  return k;
}

hipError_t launch_wy(const FlowArgs& a, bool f64, hipStream_t st, const DeviceInfo& dev) {
  const size_t lds = program_lds_bytes(a, f64 ? 8 : 4);
  const int lm = a.ladj == nullptr ? 0 : (a.accumulate ? 2 : 1);
  if (f64) return lm == 0 ? dispatch_wy<double, 0>(a, lds, st, dev)
                : lm == 1 ? dispatch_wy<double, 1>(a, lds, st, dev) : dispatch_wy<double, 2>(a, lds, st, dev);
  return lm == 0 ? dispatch_wy<float, 0>(a, lds, st, dev)
       : lm == 1 ? dispatch_wy<float, 1>(a, lds, st, dev) : dispatch_wy<float, 2>(a, lds, st, dev);
}

}  // namespace enf
