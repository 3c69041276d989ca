// enf_flow.hip -- gfx950 kernels for the batched forward / inverse + log|det J| path of
// bat/EuclidianNormalizingFlows.jl (v0.1.0).
//
// One launch applies a whole composed flow (Julia `f_n o ... o f_1`) to a column-major D x N
// batch: X is read from HBM once, every layer runs on registers, Y and the per-sample ladj are
// written once ((2D+1)*sizeof(T) algorithmic bytes per sample).
//
// Data layout ("fragment" layout, fast path). A lane owns 16-byte fragments: V = 16/sizeof(T)
// consecutive rows of one column (D >= V), or V/D whole columns (D < V). One wave-instruction
// loads/stores 64 fragments = 1 KiB of contiguous HBM, fully coalesced; a wave tile is U such
// instructions. The G = D/V lanes that share a column are adjacent, so the Householder dot
// product v'x (src/householder_trafo.jl:4,9) is a per-lane partial sum plus log2(G) DPP
// cross-lane adds (quad_perm / row_half_mirror / row_mirror), and the ladj column sum
// (sum_ladjs, src/abstract_trafo.jl:9) is one such reduction per column at the end.
//
// Program. The host flattens the composition into "steps" (one per transform; one per
// reflection of a chained HouseholderTrafo, src/householder_trafo.jl:71-78) and passes the
// step table in the kernarg segment, so the per-step dispatch is a uniform scalar branch.
// Each block's prologue derives per-row parameter records (1/lambda, delta*ln2, normalised
// reflection vectors, exp(b*a) ...) from the raw device parameter vectors into LDS, plus the
// constant part of the ladj (sum log|delta/lambda|, sum log|a|) in double precision.
//
// Arithmetic. fp64 follows the reference formulas with ocml's accurate double functions.
// fp32 uses the hardware transcendental unit (v_log_f32 / v_exp_f32 / v_sqrt_f32 / v_rcp_f32,
// each <= 1.4 ulp, measured on MI355X: profiles/r01_microbench.txt) with log2-domain
// constants folded into the parameter records; errors are normwise few-ulp.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "enf_internal.h"

#include "enf_frag.h"
#include "enf_steps.h"

namespace enf {

// Op sets of the interpreter instantiations: every op, or only reflections and Johnson layers (the
// flows of configs 2-5). The step dispatch compiles only the ops of OPS, so a narrower set needs
// fewer registers (fp64 D = 2: 208 VGPRs -> fewer, i.e. more waves per SIMD to hide fp64 latency).
constexpr int kOpsAll = 0x3F;
constexpr int kOpsHJ = (1 << OP_HOUSEHOLDER) | (1 << OP_JOHNSON);

// Interpreter: runs the step table of the kernel arguments on one register tile, then stores it.
template <typename T, int D, int U, int LM, bool TAIL, int DBG, int OPS = kOpsAll, bool PAD = false>
__device__ __forceinline__ void flow_tile(const FlowArgs& a, const T* __restrict__ rec, T ctot,
                                          int64_t col0, Tile<T, D, U>& x,
                                          const T (&old)[LadjOut<T, D, U>::NLS][LadjOut<T, D, U>::W],
                                          T* __restrict__ stage) {
  ENF_FRAG_CONSTS
  constexpr bool LADJ = LM > 0;
  const int lane = threadIdx.x & 63;
  const int grp = D >= V ? lane % G : 0;  // parameter-record group of this lane
  T acc[U][CPF];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int c = 0; c < CPF; ++c) acc[u][c] = (T)0;
  // make the vmcnt wait for THIS tile's loads happen here, with the next tile's loads still in
  // flight (inside a runtime step loop the compiler would otherwise drain vmcnt to 0)
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < V; ++e) asm volatile("" : "+v"(x[u][e]));

  int desc = a.desc[0];  // op | record offset << 4; a.desc[nsteps] is a sentinel
  for (int s = 0; s < a.nsteps; ++s) {
    const int next = a.desc[s + 1];  // scalar load issued a step ahead
    const int op = desc & 15;
    const T* __restrict__ r = rec + (desc >> 4) + grp * record_width(op) * V;
    desc = next;
    if (op == OP_HOUSEHOLDER) {
      if constexpr ((OPS >> OP_HOUSEHOLDER) & 1) step_householder<T, D, U>(x, r);
    } else if (op == OP_JOHNSON) {
      if constexpr ((OPS >> OP_JOHNSON) & 1) step_johnson<T, D, U, LADJ>(x, acc, r);
    } else if (op == OP_JOHNSON_INV) {
      if constexpr ((OPS >> OP_JOHNSON_INV) & 1) step_johnson_inv<T, D, U, LADJ>(x, acc, r);
    } else if (op == OP_SCALESHIFT) {
      if constexpr ((OPS >> OP_SCALESHIFT) & 1) step_scaleshift<T, D, U>(x, r);
    } else if (op == OP_CENTER_STRETCH) {
      if constexpr ((OPS >> OP_CENTER_STRETCH) & 1) step_center_stretch<T, D, U, LADJ>(x, acc, r);
    } else {
      if constexpr ((OPS >> OP_CENTER_CONTRACT) & 1) step_center_contract<T, D, U, LADJ>(x, acc, r);
    }
  }
  store_tile<T, D, U, LM, TAIL, DBG, PAD>(a, ctot, col0, x, acc, old, stage);
}

template <typename T, int D, int U, int LM, int OPS = kOpsAll, bool PAD = false>
struct InterpBody {
  const FlowArgs& a;
  const T* rec;
  T ctot;
  T* stage;
  template <bool TAIL, int DBG>
  __device__ __forceinline__ void tile(int64_t col0, Tile<T, D, U>& x,
                                       const T (&old)[LadjOut<T, D, U>::NLS][LadjOut<T, D, U>::W]) {
    flow_tile<T, D, U, LM, TAIL, DBG, OPS, PAD>(a, rec, ctot, col0, x, old, stage);
  }
};

// OCC: minimum waves per SIMD the register allocation must allow (launch-bounds occupancy hint).
// PAD: the padded fragment path (a.dk = D > a.D, enf_internal.h frag_pad_dim).
// PW (round 5, D <= 2): every wave builds its own records (build_program_wave) in its own LDS slice of
// a.img_off elements, with no block barrier.
template <typename T, int D, int U, int LM, int OCC, int DBG = 0, int OPS = kOpsAll, bool PAD = false, bool PW = false>
__global__ __launch_bounds__(256, OCC) void flow_frag_kernel(FlowArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* stepc = reinterpret_cast<double*>(smem);
  double* ctotp = stepc + kMaxSteps;
  T* stage = reinterpret_cast<T*>(smem + kLdsScalars) + (threadIdx.x >> 6) * kStagePerWave;
  T* rec = reinterpret_cast<T*>(smem + kLdsHeader) + (PW ? (size_t)(threadIdx.x >> 6) * a.img_off : 0);
  (void)ctotp;
  ENF_KARG_CHECK(a);
  if constexpr (DBG == 5) {  // diagnostics: nothing (the launch floor of the grid)
    if (threadIdx.x == 0 && a.N == -1) ((T*)a.Y)[blockIdx.x] = (T)0;
    return;
  }
  if constexpr (DBG == 4) {  // diagnostics: the prologue alone
    const double c = build_program<T, D, Frag<T, D>::V>(a, rec, stepc);
    if (threadIdx.x == 0 && c == 1234.5) ((T*)a.Y)[blockIdx.x] = rec[0];
    return;
  }
  InterpBody<T, D, U, LM, OPS, PAD> body{a, rec, (T)0, stage};
  // the prologue runs after the wave's first tile loads are issued (frag_stream), so the HBM latency
  // of the first tile overlaps the parameter loads and record construction
  frag_stream<T, D, U, LM, DBG >= 4 ? 0 : DBG, PAD>(a, body, [&]() {
    if constexpr (PW) body.ctot = (T)build_program_wave<T, Frag<T, D>::V>(a, rec);
    else body.ctot = (T)build_program<T, D, Frag<T, D>::V>(a, rec, stepc);
  });
}

// ------------------------------------------------------------------------------------------
// generic kernel: any D, any leading dimensions, any alignment. One column per lane; the
// column lives in Y (copied from X first), every step re-reads it from global memory.
// ------------------------------------------------------------------------------------------
// The whole step program on one column y[0 .. D-1] (global memory or an LDS image), in the
// reference's elementwise order; returns the column's ladj in natural-log units (without the
// constant part ctot).
template <typename T>
__device__ __forceinline__ double generic_column(const FlowArgs& a, const T* __restrict__ rec, T* y, int D) {
  double acc = 0.0;  // natural-log units
  for (int s = 0; s < a.nsteps; ++s) {
    const int op = a.steps[s].op;
    const T* r = rec + a.steps[s].off;
    if (op == OP_HOUSEHOLDER) {
      T dot = 0;
      for (int d = 0; d < D; ++d) dot = fma(r[d], y[d], dot);
      for (int d = 0; d < D; ++d) y[d] = fma(-dot, r[d], y[d]);
    } else if (op == OP_SCALESHIFT) {
      for (int d = 0; d < D; ++d) y[d] = fma(y[d], r[2 * d], r[2 * d + 1]);
    } else if (op == OP_JOHNSON) {
      for (int d = 0; d < D; ++d) {
        if constexpr (std::is_same_v<T, float>) {
          const YL r2 = johnson_fwd_f32_slow((y[d] - r[4 * d + 2]) * r[4 * d + 3], r[4 * d], r[4 * d + 1]);
          y[d] = r2.y;
          acc += (double)r2.l * kLn2;
        } else {
          const double z = (y[d] - r[4 * d + 2]) * r[4 * d + 3];
          y[d] = fma(r[4 * d + 1], asinh64(z), r[4 * d]);
          acc -= 0.5 * log1p(z * z);
        }
      }
    } else if (op == OP_JOHNSON_INV) {
      for (int d = 0; d < D; ++d) {
        if constexpr (std::is_same_v<T, float>) {
          const float w = (y[d] - r[4 * d]) * r[4 * d + 1];
          const float sh = sinhf(w);
          y[d] = fmaf(r[4 * d + 3], sh, r[4 * d + 2]);
          acc += 0.5 * log1p((double)sh * sh);
        } else {
          const double w = (y[d] - r[4 * d]) * r[4 * d + 1];
          const double sh = sinh64(w);
          y[d] = fma(r[4 * d + 3], sh, r[4 * d + 2]);
          acc += 0.5 * log1p64_ge0(sh * sh);
        }
      }
    } else if (op == OP_CENTER_STRETCH || op == OP_CENTER_CONTRACT) {
      for (int d = 0; d < D; ++d) {
        const T* rr = r + 8 * d;
        double av, bv, c;
        if constexpr (std::is_same_v<T, float>) {
          av = rr[6]; bv = rr[7]; c = rr[1];
        } else {
          av = rr[0]; bv = rr[1]; c = rr[2];
        }
        const T xv = y[d];
        if (op == OP_CENTER_STRETCH) {
          const T ex = (T)exp(fabs((T)bv * xv));
          const T ome = (T)1 - ex;
          const T inner = ((T)sqrt(ome * ome * (T)exp(2.0 * bv * av) + (T)4 * ex) - ome * (T)exp(bv * av)) / (T)2;
          const T sg = xv > (T)0 ? (T)1 : (xv < (T)0 ? (T)-1 : xv);
          const T yv = sg * (T)log(inner) / (T)bv + (T)c;
          y[d] = yv;
          const double yu = (double)yv - c;
          acc -= log(fabs(1.0 / (1.0 + exp(-bv * (yu - av))) + 1.0 / (1.0 + exp(bv * (yu + av)))));
        } else {
          const double xu = (double)xv - c;
          y[d] = (T)((log(1.0 + exp(bv * (xu - av))) - log(1.0 + exp(-bv * (xu + av)))) / bv);
          acc += log(fabs(1.0 / (1.0 + exp(-bv * (xu - av))) + 1.0 / (1.0 + exp(bv * (xu + av)))));
        }
      }
    }
  }
  return acc;
}

template <typename T, bool LADJ>
__global__ __launch_bounds__(256) void flow_generic_kernel(FlowArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* stepc = reinterpret_cast<double*>(smem);
  double* ctotp = stepc + kMaxSteps;
  T* rec = reinterpret_cast<T*>(smem + kLdsHeader);
  (void)ctotp;
  ENF_KARG_CHECK(a);
  const double ctot = build_program<T, 0, 1>(a, rec, stepc);
  const int D = a.D;
  const T* __restrict__ X = (const T*)a.X;
  T* __restrict__ Y = (T*)a.Y;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a.N;
       j += (int64_t)gridDim.x * blockDim.x) {
    const T* x = X + j * a.ldx;
    T* y = Y + j * a.ldy;
    if (x != y)
      for (int d = 0; d < D; ++d) y[d] = x[d];
    const double acc = generic_column<T>(a, rec, y, D);
    if (LADJ) {
      T* ladj = (T*)a.ladj;
      const T v = (T)(ctot + acc);
      ladj[j] = a.accumulate ? ladj[j] + v : v;
    }
  }
}

// LDS-staged generic kernel (any D whose tile image fits, any leading dimensions and alignment):
// a wave moves a tile of CT columns between HBM and its LDS image with coalesced accesses
// (consecutive lanes on consecutive elements: element-linear over the whole tile when the columns
// are contiguous, column by column otherwise), lane c runs the program on column c of the image
// (row stride DP = D rounded up to odd: conflict-free banks), and the tile goes back the same way.
// magic = ceil(2^32 / D): c = umulhi(i, magic) = i / D exactly for i < CT * D (CT * D <= 2^14).
template <typename T, bool LADJ>
__global__ __launch_bounds__(256) void flow_lds_kernel(FlowArgs a, int ct, int dp, uint32_t magic) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* stepc = reinterpret_cast<double*>(smem);
  double* ctotp = stepc + kMaxSteps;
  T* rec = reinterpret_cast<T*>(smem + kLdsHeader);
  (void)ctotp;
  ENF_KARG_CHECK(a);
  const double ctot = build_program<T, 0, 1>(a, rec, stepc);
  const int D = a.D;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  T* img = reinterpret_cast<T*>(smem + a.img_off) + (size_t)wave * ct * dp;
  const T* __restrict__ X = (const T*)a.X;
  T* __restrict__ Y = (T*)a.Y;
  const int64_t ntiles = (a.N + ct - 1) / ct;
  for (int64_t t = (int64_t)blockIdx.x * 4 + wave; t < ntiles; t += (int64_t)gridDim.x * 4) {
    const int64_t c0 = t * ct;
    const int nc = (int)(a.N - c0 < ct ? a.N - c0 : ct);
    if (a.ldx == D) {
      const T* x = X + c0 * D;
      for (int i = lane; i < nc * D; i += 64) {
        const int c = (int)__umulhi((uint32_t)i, magic);
        img[c * dp + (i - c * D)] = x[i];
      }
    } else {
      for (int c = 0; c < nc; ++c)
        for (int r = lane; r < D; r += 64) img[c * dp + r] = X[(c0 + c) * a.ldx + r];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    double acc = 0.0;
    if (lane < nc) acc = generic_column<T>(a, rec, img + lane * dp, D);
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (a.ldy == D) {
      T* y = Y + c0 * D;
      for (int i = lane; i < nc * D; i += 64) {
        const int c = (int)__umulhi((uint32_t)i, magic);
        y[i] = img[c * dp + (i - c * D)];
      }
    } else {
      for (int c = 0; c < nc; ++c)
        for (int r = lane; r < D; r += 64) Y[(c0 + c) * a.ldy + r] = img[c * dp + r];
    }
    if (LADJ && lane < nc) {
      T* ladj = (T*)a.ladj;
      const T v = (T)(ctot + acc);
      ladj[c0 + lane] = a.accumulate ? ladj[c0 + lane] + v : v;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

// ------------------------------------------------------------------------------------------
// host-side launch
// ------------------------------------------------------------------------------------------
size_t program_lds_bytes(const FlowArgs& a, size_t elem) {
  const bool frag = frag_supported(a, elem);
  size_t n = 0;
  for (int s = 0; s < a.nsteps; ++s) n += record_elems(a.steps[s].op, a.dk ? a.dk : a.D, elem, frag);
  return kLdsHeader + n * elem;
}

// Tuning knobs of the diagnostics build only (enf_internal.h ENF_KNOB): ENF_BLOCKS_PER_CU caps
// resident blocks per CU in the grid size, ENF_FRAG_U / ENF_FRAG_OCC select fp32 D = 32 interpreter
// variants, ENF_DEBUG_MODE the diagnostic kernels (1: synthesized tile instead of loads, 2: also no
// stores), ENF_NO_SPECIALIZE=1 disables the compiled (H o J)^n programs (enf_flow_hj.hip).
#if ENF_DIAG
int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}
#endif

hipError_t frag_grid(const void* kernel, int64_t N, int64_t cols_per_block, size_t lds, const DeviceInfo& dev,
                     int64_t* blocks) {
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, lds);
  if (e != hipSuccess) return e;
  static const int cap_env = ENF_KNOB("ENF_BLOCKS_PER_CU", 0);
  if (cap_env > 0 && per_cu > cap_env) per_cu = cap_env;
  if (per_cu < 1) per_cu = 1;
  int64_t b = (N + cols_per_block - 1) / cols_per_block;
  const int64_t cap = (int64_t)dev.num_cu * per_cu;
  if (b > cap) b = cap;
  *blocks = b < 1 ? 1 : b;
  return hipSuccess;
}

template <typename T, int D, int U, int LM, int OCC = 1, int DBG = 0, int OPS = kOpsAll, bool PAD = false>
static hipError_t launch_frag(const FlowArgs& a, size_t lds, hipStream_t st, const DeviceInfo& dev) {
  using F = Frag<T, D>;
  const void* k = reinterpret_cast<const void*>(&flow_frag_kernel<T, D, U, LM, OCC, DBG, OPS, PAD>);
  int64_t blocks = 0;
  hipError_t e = frag_grid(k, a.N, (int64_t)F::COLS_PER_INSTR * U * 4, lds, dev, &blocks);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((flow_frag_kernel<T, D, U, LM, OCC, DBG, OPS, PAD>), dim3((unsigned)blocks), dim3(256), lds, st,
                     a);
  return hipGetLastError();
}

// D <= 2 with per-wave records (PW): the records' LDS is per wave (img_off = the elements of one copy)
template <typename T, int D, int U, int LM, int OPS = kOpsAll>
static hipError_t launch_frag_pw(const FlowArgs& a, size_t lds, hipStream_t st, const DeviceInfo& dev) {
  using F = Frag<T, D>;
  const size_t elem = sizeof(T);
  const size_t rec_bytes = (lds - kLdsHeader + 15) / 16 * 16;
  FlowArgs b = a;
  b.img_off = (int32_t)(rec_bytes / elem);
#if ENF_BOUNDS
  b.csum = flow_args_csum(b);
#endif
  const size_t ldsw = kLdsHeader + 4 * rec_bytes;
  const void* k = reinterpret_cast<const void*>(&flow_frag_kernel<T, D, U, LM, 1, 0, OPS, false, true>);
  int64_t blocks = 0;
  hipError_t e = frag_grid(k, a.N, (int64_t)F::COLS_PER_INSTR * U * 4, ldsw, dev, &blocks);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((flow_frag_kernel<T, D, U, LM, 1, 0, OPS, false, true>), dim3((unsigned)blocks), dim3(256), ldsw,
                     st, b);
  return hipGetLastError();
}

// the per-wave prologue applies: D <= 2, one lane per (step, row). Measured and NOT taken (round 5, diagnostics
// knob ENF_SMALL_PW=1): at D = 2, N = 1e6, fp64 the kernel times under rocprofv3 were J o C 21.7 vs 20.4 us, K o H o S
// 18.6 vs 17.8, J 14.5 vs 13.3, S 9.9 vs 9.9 with the block prologue (profiles/r05/d2_small_pw_ab.txt): the
// per-lane parameter loads and logs of every wave cost more than the block barrier saves.
static bool pw_eligible(const FlowArgs& a) {
  static const int pw = ENF_KNOB("ENF_SMALL_PW", 0);
  if (!pw || a.dk || a.wy || (a.D != 1 && a.D != 2) || a.nsteps * a.D > 64) return false;
  for (int s = 0; s < a.nsteps; ++s)
    if (a.steps[s].op == OP_DENSE) return false;
  return true;
}

// The padded fragment path (a.dk = the power-of-two layout of a.D rows): every op has neutral
// parameters that map 0 to 0 with ladj 0 (enf_steps.h neutral_values).
constexpr int kOpsPad = kOpsAll;
template <typename T, int LADJ>
static hipError_t dispatch_pad(const FlowArgs& a, size_t lds, hipStream_t st, const DeviceInfo& dev) {
  switch (a.dk) {
    case 8: return launch_frag<T, 8, 4, LADJ, 1, 0, kOpsPad, true>(a, lds, st, dev);
    case 16: return launch_frag<T, 16, 4, LADJ, 1, 0, kOpsPad, true>(a, lds, st, dev);
    case 32: return launch_frag<T, 32, 4, LADJ, 1, 0, kOpsPad, true>(a, lds, st, dev);
    case 64:
      if constexpr (std::is_same_v<T, float>) return launch_frag<T, 64, 4, LADJ, 1, 0, kOpsPad, true>(a, lds, st, dev);
      else return launch_frag<T, 64, 2, LADJ, 1, 0, kOpsPad, true>(a, lds, st, dev);
    case 128:
      if constexpr (std::is_same_v<T, float>) return launch_frag<T, 128, 4, LADJ, 1, 0, kOpsPad, true>(a, lds, st, dev);
      else return launch_frag<T, 128, 2, LADJ, 1, 0, kOpsPad, true>(a, lds, st, dev);
    case 256:
      if constexpr (std::is_same_v<T, float>) return launch_frag<T, 256, 4, LADJ, 1, 0, kOpsPad, true>(a, lds, st, dev);
      break;
    default: break;
  }
  return hipErrorInvalidValue;
}

// the op set of a flow (bit op per step)
static int flow_ops(const FlowArgs& a) {
  int m = 0;
  for (int s = 0; s < a.nsteps; ++s) m |= 1 << a.steps[s].op;
  return m;
}

template <typename T, int LADJ>
static hipError_t dispatch_D(const FlowArgs& a, size_t lds, hipStream_t st, const DeviceInfo& dev) {
  if (a.dk) {
    // the compiled (J o H)^n programs on the padded layout (round 3; D = 24, 36, 100, ... on 32 / 64 / 128)
    static const int nospec = ENF_KNOB("ENF_NO_SPECIALIZE", 0);
    if (!nospec && hj_program_pairs(a) > 0) {
      hipError_t e = std::is_same_v<T, float> ? launch_hj_program(a, LADJ, 0, st, dev)
                                              : launch_hj64_program(a, LADJ, st, dev);
      if (e != hipErrorNotSupported) return e;
    }
    if (!nospec && hji_program_pairs(a) > 0) {
      hipError_t e = std::is_same_v<T, float> ? launch_hji_program(a, LADJ, st, dev)
                                              : launch_hji64_program(a, LADJ, st, dev);
      if (e != hipErrorNotSupported) return e;
    }
    return dispatch_pad<T, LADJ>(a, lds, st, dev);
  }
  if constexpr (std::is_same_v<T, float>) {
    static const int nospec = ENF_KNOB("ENF_NO_SPECIALIZE", 0);
    static const int dbg = ENF_KNOB("ENF_DEBUG_MODE", 0);
    if (!nospec && hj_program_pairs(a) > 0) {
      hipError_t e = launch_hj_program(a, LADJ, dbg, st, dev);
      if (e != hipErrorNotSupported) return e;
    }
    // the compiled inverse program (J^-1, H)^n (round 4)
    if (!nospec && hji_program_pairs(a) > 0) {
      hipError_t e = launch_hji_program(a, LADJ, st, dev);
      if (e != hipErrorNotSupported) return e;
    }
#if ENF_DIAG
    if (a.D == 32) {
      static const int u = ENF_KNOB("ENF_FRAG_U", 4);
      static const int occ = ENF_KNOB("ENF_FRAG_OCC", 1);
      if (dbg == 1) return launch_frag<T, 32, 4, LADJ, 1, 1>(a, lds, st, dev);
      if (dbg == 2) return launch_frag<T, 32, 4, LADJ, 1, 2>(a, lds, st, dev);
      if (u == 2) return launch_frag<T, 32, 2, LADJ>(a, lds, st, dev);
      if (u == 4 && occ == 5) return launch_frag<T, 32, 4, LADJ, 5>(a, lds, st, dev);
    }
#endif
  }
  if constexpr (std::is_same_v<T, double>) {
    // config 2: the compiled J o H program at D = 2 (ENF_NO_D2=1 in the diagnostics build: the interpreter)
    static const int no_d2 = ENF_KNOB("ENF_NO_D2", 0);
    if (!no_d2 && d2_program(a)) return launch_d2_program(a, LADJ, st, dev);
    // the compiled fp64 (J o H)^n program at D = 32 / 64 (ENF_NO_SPECIALIZE=1: the interpreter)
    static const int nospec = ENF_KNOB("ENF_NO_SPECIALIZE", 0);
    if (!nospec && hj_program_pairs(a) > 0) {
      hipError_t e = launch_hj64_program(a, LADJ, st, dev);
      if (e != hipErrorNotSupported) return e;
    }
    // the compiled fp64 inverse program (J^-1, H)^n (round 4)
    if (!nospec && hji_program_pairs(a) > 0) {
      hipError_t e = launch_hji64_program(a, LADJ, st, dev);
      if (e != hipErrorNotSupported) return e;
    }
  }
#if ENF_DIAG
  if (a.D == 2) {  // C2 diagnostics: 1 = synthesized tile, 2 = also no stores, 4 = prologue only
    static const int fdbg = ENF_KNOB("ENF_FRAG_DBG", 0);
    // the product's op set (kOpsHJ, 118 VGPRs); 5 = an empty kernel of the same grid (launch floor)
    if (fdbg == 1) return launch_frag<T, 2, 4, LADJ, 1, 1, kOpsHJ>(a, lds, st, dev);
    if (fdbg == 2) return launch_frag<T, 2, 4, LADJ, 1, 2, kOpsHJ>(a, lds, st, dev);
    if (fdbg == 4) return launch_frag<T, 2, 4, LADJ, 1, 4, kOpsHJ>(a, lds, st, dev);
    if (fdbg == 5) return launch_frag<T, 2, 4, LADJ, 1, 5, kOpsHJ>(a, lds, st, dev);
  }
#endif
  if (pw_eligible(a)) {  // D <= 2: per-wave records, no block barrier (round 5)
    if ((flow_ops(a) & ~kOpsHJ) == 0)
      return a.D == 1 ? launch_frag_pw<T, 1, 4, LADJ, kOpsHJ>(a, lds, st, dev) : launch_frag_pw<T, 2, 4, LADJ, kOpsHJ>(a, lds, st, dev);
    return a.D == 1 ? launch_frag_pw<T, 1, 4, LADJ>(a, lds, st, dev) : launch_frag_pw<T, 2, 4, LADJ>(a, lds, st, dev);
  }
  if ((flow_ops(a) & ~kOpsHJ) == 0) {  // reflections and Johnson layers only (configs 2-5)
#if ENF_DIAG
    static const int hju = ENF_KNOB("ENF_FRAG_HJU", 4);
    if (a.D == 2 && hju == 2) return launch_frag<T, 2, 2, LADJ, 1, 0, kOpsHJ>(a, lds, st, dev);
    if (a.D == 2 && hju == 1) return launch_frag<T, 2, 1, LADJ, 1, 0, kOpsHJ>(a, lds, st, dev);
#endif
    switch (a.D) {
      case 1: return launch_frag<T, 1, 4, LADJ, 1, 0, kOpsHJ>(a, lds, st, dev);
      case 2: return launch_frag<T, 2, 4, LADJ, 1, 0, kOpsHJ>(a, lds, st, dev);
      case 4: return launch_frag<T, 4, 4, LADJ, 1, 0, kOpsHJ>(a, lds, st, dev);
      case 8: return launch_frag<T, 8, 4, LADJ, 1, 0, kOpsHJ>(a, lds, st, dev);
      case 16: return launch_frag<T, 16, 4, LADJ, 1, 0, kOpsHJ>(a, lds, st, dev);
      default: break;
    }
  }
  switch (a.D) {
    case 1: return launch_frag<T, 1, 4, LADJ>(a, lds, st, dev);
    case 2: return launch_frag<T, 2, 4, LADJ>(a, lds, st, dev);
    case 4: return launch_frag<T, 4, 4, LADJ>(a, lds, st, dev);
    case 8: return launch_frag<T, 8, 4, LADJ>(a, lds, st, dev);
    case 16: return launch_frag<T, 16, 4, LADJ>(a, lds, st, dev);
    case 32: return launch_frag<T, 32, 4, LADJ>(a, lds, st, dev);
    case 64:
      if constexpr (std::is_same_v<T, float>) return launch_frag<T, 64, 4, LADJ>(a, lds, st, dev);
      else return launch_frag<T, 64, 2, LADJ>(a, lds, st, dev);
    case 128:
      if constexpr (std::is_same_v<T, float>) return launch_frag<T, 128, 4, LADJ>(a, lds, st, dev);
      else return launch_frag<T, 128, 2, LADJ>(a, lds, st, dev);
    case 256:
      if constexpr (std::is_same_v<T, float>) return launch_frag<T, 256, 4, LADJ>(a, lds, st, dev);
      break;
    default: break;
  }
  return hipErrorInvalidValue;
}

bool frag_supported(const FlowArgs& a, size_t elem) {
  (void)elem;
  return a.frag != 0;  // decided once per call by the host (records are laid out for it)
}

hipError_t launch_flow(const FlowArgs& a, bool f64, hipStream_t st, const DeviceInfo& dev) {
  const size_t elem = f64 ? 8 : 4;
  const size_t lds = program_lds_bytes(a, elem);
  const bool ladj = a.ladj != nullptr;
  if (a.wy) return launch_wy(a, f64, st, dev);
  if (frag_supported(a, elem)) {
    const int lm = !ladj ? 0 : (a.accumulate ? 2 : 1);
    if (f64) return lm == 0 ? dispatch_D<double, 0>(a, lds, st, dev)
                  : lm == 1 ? dispatch_D<double, 1>(a, lds, st, dev) : dispatch_D<double, 2>(a, lds, st, dev);
    return lm == 0 ? dispatch_D<float, 0>(a, lds, st, dev)
         : lm == 1 ? dispatch_D<float, 1>(a, lds, st, dev) : dispatch_D<float, 2>(a, lds, st, dev);
  }
  // LDS-staged generic kernel when a tile of >= 16 columns fits 16 KB per wave (ENF_NO_LDS_GENERIC=1:
  // the one-column-per-lane kernel)
  static const int no_lds = ENF_KNOB("ENF_NO_LDS_GENERIC", 0);
  static const size_t wave_kb = (size_t)ENF_KNOB("ENF_LDS_GENERIC_KB", 16) * 1024;  // image bytes per wave
  const int dp = (a.D | 1);
  int ct = 64;
  while (ct > 8 && (size_t)ct * dp * elem > wave_kb) ct >>= 1;
  if (!no_lds && a.D >= 1 && (size_t)ct * dp * elem <= wave_kb && ct >= 16 && (int64_t)ct * a.D <= (1 << 14)) {
    FlowArgs b = a;
    b.img_off = (int32_t)((lds + 15) / 16 * 16);
#if ENF_BOUNDS
    b.csum = flow_args_csum(b);
#endif
    const size_t ldsb = (size_t)b.img_off + 4 * (size_t)ct * dp * elem;
    const uint32_t magic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)a.D - 1) / (uint64_t)a.D);
    const void* k = f64 ? (ladj ? (const void*)&flow_lds_kernel<double, true> : (const void*)&flow_lds_kernel<double, false>)
                        : (ladj ? (const void*)&flow_lds_kernel<float, true> : (const void*)&flow_lds_kernel<float, false>);
    if (ldsb > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsb);
      if (e != hipSuccess) return e;
    }
    int64_t nb = 0;
    hipError_t e = frag_grid(k, a.N, (int64_t)ct * 4, ldsb, dev, &nb);
    if (e != hipSuccess) return e;
    if (f64) {
      if (ladj) hipLaunchKernelGGL((flow_lds_kernel<double, true>), dim3((unsigned)nb), dim3(256), ldsb, st, b, ct, dp, magic);
      else hipLaunchKernelGGL((flow_lds_kernel<double, false>), dim3((unsigned)nb), dim3(256), ldsb, st, b, ct, dp, magic);
    } else {
      if (ladj) hipLaunchKernelGGL((flow_lds_kernel<float, true>), dim3((unsigned)nb), dim3(256), ldsb, st, b, ct, dp, magic);
      else hipLaunchKernelGGL((flow_lds_kernel<float, false>), dim3((unsigned)nb), dim3(256), ldsb, st, b, ct, dp, magic);
    }
    return hipGetLastError();
  }
  int64_t blocks = (a.N + 255) / 256;
  const int64_t cap = (int64_t)dev.num_cu * 8;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  if (f64) {
    if (ladj) hipLaunchKernelGGL((flow_generic_kernel<double, true>), dim3((unsigned)blocks), dim3(256), lds, st, a);
    else hipLaunchKernelGGL((flow_generic_kernel<double, false>), dim3((unsigned)blocks), dim3(256), lds, st, a);
  } else {
    if (ladj) hipLaunchKernelGGL((flow_generic_kernel<float, true>), dim3((unsigned)blocks), dim3(256), lds, st, a);
    else hipLaunchKernelGGL((flow_generic_kernel<float, false>), dim3((unsigned)blocks), dim3(256), lds, st, a);
  }
  return hipGetLastError();
}

}  // namespace enf
