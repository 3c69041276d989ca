// enf_flow_d2.hip -- compiled program for config 2: JohnsonTrafo ∘ HouseholderTrafo
// at D = 2 in fp64 (src/johnson_trafo.jl:29-32,39-42; src/householder_trafo.jl:8-11, one reflection),
// X read once, Y and the per-sample ladj written once (40 algorithmic bytes per sample).
//
// Why a kernel of its own: at N = 1e6 the interpreter (flow_frag_kernel) spends ~3 us of its ~15 us in a
// block prologue (parameter loads, double log / sqrt / division, the LDS log table, a block barrier)
// that no wave can overlap, and walks its step table per tile (profiles/r02_c2_*: launch floor 2.3 us,
// prologue 5.4, compute-only 12.4, full 14.9). Here every wave builds what it needs itself, with no
// block barrier, while its first tile's loads are in flight:
//  * the parameters are wave-uniform: rows 0 and 1 are computed by lanes 0 and 1 (v_d^2 and
//    log|delta_d| - log|lambda_d|, summed by one lane swap, then sqrt(2/v'v), v_d sqrt(2/v'v), 1/lambda_d)
//    and read back into scalar registers; gamma, delta, xi arrive by scalar loads;
//  * the 33-entry fp64 log table (enf_logtab.h, used by asinh64_tab / logprod64_tab) is copied into
//    the wave's own LDS slice by lanes 0..32 (one wave barrier, no block barrier);
//  * a lane owns whole columns (one 16-byte fragment = one column), U = 2 columns per tile at a stride
//    of 64, so every load / store instruction moves 1 KiB of contiguous HBM and the ladj store 512 B.
// The arithmetic is the interpreter's, operation for operation (enf_steps.h step_householder /
// step_johnson fp64 and build_program's constants, same ocml functions in the prologue), so the
// results are bit-identical to it: dot = vh0 x0 + vh1 x1 (fma), x' = fma(-dot, vh, x),
// z = (x' - xi) * (1/lambda), y = fma(delta, asinh64_tab(z), gamma), q = fma(z, z, 1),
// ladj = fma(1, -log(q0 q1)/2, ctot) (+ the old ladj when accumulating).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>

#include "enf_frag.h"
#include "enf_internal.h"
#include "enf_logtab.h"
#include "enf_math64.h"

namespace enf {

struct D2Args {
  const double* X;
  double* Y;
  double* ladj;
  int64_t N;
  const double* v;    // reflection vector (column of V)
  const double* g;    // Johnson gamma, delta, xi, lambda
  const double* d;
  const double* xi;
  const double* lam;
};

// doubles of one wave's copy of the B-bit log table (enf_logtab.h)
constexpr int d2_tab_doubles(int B) { return 3 * ((1 << B) + 1); }
template <int B>
__device__ __forceinline__ const double* d2_tab_src() {
  static_assert(B == kLogTabBits, "the B = 5 table only (the B = 7 / 8 variants were rejected, round 4)");
  return kLogTab;
}

__device__ __forceinline__ double d2_readlane(double v, int l) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, l), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// DBG (diagnostics build only): 1 = synthesize the tile instead of loading it, 2 = also skip the stores,
// 3 = loads and stores without the Johnson arithmetic (the kernel's memory floor)
template <int U, bool TAIL, int DBG, int NT = 3>
__device__ __forceinline__ void d2_load(const D2Args& a, int64_t col0, int lane, double (&x)[U][2], bool live = true) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    // a tile past the wave's last (live false) is still loaded, so the vmcnt waits stay static, but every
    // lane reads column 0: one cache line instead of the tile
    const int64_t c = live ? col0 + (int64_t)u * 64 + lane : 0;
    if (DBG == 1 || DBG == 2) {
      x[u][0] = (double)(lane + 3 * u) * 0.03125 - 1.0;
      x[u][1] = (double)(lane - 5 * u) * 0.0625 + 0.5;
    } else if (!TAIL) {
      if (ENF_INB(c < a.N, "d2 load X", c, a.N)) {
        const u32x4 v4 = (NT & 1) ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.X + 2 * c))
                                  : *reinterpret_cast<const u32x4*>(a.X + 2 * c);
        __builtin_memcpy(&x[u][0], &v4, 16);
      }
    } else {
      x[u][0] = c < a.N ? a.X[2 * c] : 0.0;
      x[u][1] = c < a.N ? a.X[2 * c + 1] : 0.0;
    }
  }
}

struct D2Prog {
  double vh0, vh1, g0, g1, d0, d1, xi0, xi1, il0, il1, ctot;
};

template <int U, int LM, bool TAIL, int DBG, int TB, int NT = 3>
__device__ __forceinline__ void d2_tile(const D2Args& a, const D2Prog& P, const double* __restrict__ tab, int64_t col0,
                                        int lane, double (&x)[U][2]) {
  double old[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t c = col0 + (int64_t)u * 64 + lane;
    old[u] = (LM == 2 && (!TAIL || c < a.N)) ? a.ladj[c] : 0.0;
  }
  double lad[U], z[U][2];
  bool far = false;  // some |z| >= 2^26, Inf or NaN in this lane
#pragma unroll
  for (int u = 0; u < U; ++u) {
    // HouseholderTrafo: x - vh (vh'x)
    double dot = P.vh0 * x[u][0];
    dot = fma(P.vh1, x[u][1], dot);
    const double x0 = fma(-dot, P.vh0, x[u][0]);
    const double x1 = fma(-dot, P.vh1, x[u][1]);
    // JohnsonTrafo
    z[u][0] = (x0 - P.xi0) * P.il0;
    z[u][1] = (x1 - P.xi1) * P.il1;
    far = far || !asinh64_fin_ok(z[u][0]) || !asinh64_fin_ok(z[u][1]);
  }
  if (DBG == 3) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u][0] = z[u][0];
      x[u][1] = z[u][1];
      lad[u] = z[u][0] * z[u][1];
    }
  } else if (!__any(far)) {
    // the whole wave in |z| < 2^26: the range-free asinh and the plain log of the q product (bit-identical
    // to asinh64_tab / logprod64_tab there; no product of two q < 2^53 overflows)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u][0] = fma(P.d0, asinh64_tab_fin<TB>(z[u][0], tab), P.g0);
      x[u][1] = fma(P.d1, asinh64_tab_fin<TB>(z[u][1], tab), P.g1);
      if (LM > 0) lad[u] = 0.0 - 0.5 * log64_tab_b<TB>(fma(z[u][0], z[u][0], 1.0) * fma(z[u][1], z[u][1], 1.0), 0, tab);
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u][0] = fma(P.d0, asinh64_tab<TB>(z[u][0], tab), P.g0);
      x[u][1] = fma(P.d1, asinh64_tab<TB>(z[u][1], tab), P.g1);
      if (LM > 0) {
        const double q[2] = {fma(z[u][0], z[u][0], 1.0), fma(z[u][1], z[u][1], 1.0)};
        lad[u] = 0.0 - 0.5 * logprod64_tab<2, TB>(q, tab);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t c = col0 + (int64_t)u * 64 + lane;
    if (DBG == 2) {
      if (x[u][0] == 1234.5) a.Y[2 * c] = x[u][1];  // keeps the compute alive, never true in practice
    } else if (!TAIL) {
      if (ENF_INB(c < a.N, "d2 store Y", c, a.N)) {
        u32x4 v4;
        __builtin_memcpy(&v4, &x[u][0], 16);
        if (NT & 2) __builtin_nontemporal_store(v4, reinterpret_cast<u32x4*>(a.Y + 2 * c));
        else *reinterpret_cast<u32x4*>(a.Y + 2 * c) = v4;
      }
    } else if (c < a.N) {
      a.Y[2 * c] = x[u][0];
      a.Y[2 * c + 1] = x[u][1];
    }
    if (LM > 0 && DBG != 2) {
      const double v = fma(1.0, lad[u], P.ctot) + old[u];
      if ((!TAIL && ENF_INB(c < a.N, "d2 ladj", c, a.N)) || (TAIL && c < a.N)) a.ladj[c] = v;
    }
  }
}

// the last r < P tiles of a wave, already loaded in xs[0 .. r-1]: tile K only after tile K - 1 (nested)
template <int K, int P, int U, int LM, int DBG, int TB, int NT>
__device__ __forceinline__ void d2_rem(const D2Args& a, const D2Prog& P_, const double* __restrict__ tab, int r,
                                       int64_t t, int64_t nwaves, int lane, double (&xs)[P][U][2]) {
  if constexpr (K < P - 1) {
    if (K < r) {
      d2_tile<U, LM, false, DBG, TB, NT>(a, P_, tab, t * (64 * U), lane, xs[K]);
      d2_rem<K + 1, P, U, LM, DBG, TB, NT>(a, P_, tab, r, t + nwaves, nwaves, lane, xs);
    }
  }
}

// P: tiles in flight per wave (the current one and P - 1 prefetched): at N = 1e6 a wave has ~4 tiles, so
// with one tile of lookahead only ~2 KiB per wave is in flight, far below what the HBM latency needs.
// PB (diagnostics A/B): the program constants computed once per block by one wave (wave b % 4 of block b, so
// the four SIMDs share the work) and broadcast through LDS after an LDS-only barrier, and one log table per
// block, instead of every wave computing its own. TB: the log table's index bits (enf_logtab.h). NT: bit 0
// nontemporal X loads, bit 1 nontemporal Y stores. LO (diagnostics A/B): 1 = only the first tile's load
// before the prologue, the other P - 1 after it (every wave's first tile ahead of the later ones in the
// memory queues).
template <int U, int LM, int DBG, int P = 2, bool PB = false, int TB = 5, int NT = 3, int LO = 0>
__global__ __launch_bounds__(256, U == 1 ? 8 : 4) void flow_d2_kernel(D2Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  constexpr int kTab = d2_tab_doubles(TB);
  double* tab = reinterpret_cast<double*>(smem) + (PB ? 0 : wave * kTab);
  double* progl = reinterpret_cast<double*>(smem) + kTab;  // PB: the 11 broadcast constants
  constexpr int64_t CT = 64 * U;
  const int64_t ntiles_full = a.N / CT;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + wave;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  double xs[P][U][2];
  // The parameters and the log table are loaded FIRST, then the first P tiles: the vmcnt counter retires
  // loads in issue order, so the prologue waits for its own loads only and computes while the tiles stream
  // in. (Issued after the tiles, as before, the table copy's wait was vmcnt(0): every wave sat until all of
  // its tiles -- the whole 16 MB of X across the chip -- had arrived, and only then started two dependent
  // parameter round trips, so no store could start before the last read: 9.1 of the 11.8 us were the
  // memory phase, profiles/r03_c2_prologue_ab.txt.)
  constexpr int kTabIt = (kTab / 3 + 63) / 64;
  double tv[kTabIt][3];
  const double* src = d2_tab_src<TB>();
#pragma unroll
  for (int it = 0; it < kTabIt; ++it) {
    const int i = lane + 64 * it;
    const int ic = i < kTab / 3 ? i : 0;
    tv[it][0] = src[3 * ic];
    tv[it][1] = src[3 * ic + 1];
    tv[it][2] = src[3 * ic + 2];
  }
  const double v_l = a.v[lane & 1], d_l = a.d[lane & 1], lam_l = a.lam[lane & 1];
  D2Prog P_;
  P_.g0 = a.g[0];
  P_.g1 = a.g[1];
  P_.d0 = a.d[0];
  P_.d1 = a.d[1];
  P_.xi0 = a.xi[0];
  P_.xi1 = a.xi[1];
  __builtin_amdgcn_sched_barrier(0);
  // the wave's table copy and program constants (every wave runs this exactly once: the PB variant's block
  // barrier sees all four waves)
  auto prologue = [&]() {
    // the wave's (PB: the block's) copy of the log table
    if (!PB || wave == 1) {
#pragma unroll
      for (int it = 0; it < kTabIt; ++it) {
        const int i = lane + 64 * it;
        if (i < kTab / 3) {
          tab[3 * i] = tv[it][0];
          tab[3 * i + 1] = tv[it][1];
          tab[3 * i + 2] = tv[it][2];
        }
      }
    }
    if (!PB || wave == (int)(blockIdx.x & 3)) {
    // parameters (build_program / param_values in enf_steps.h, same operations and ocml functions, so the
    // same values). A VALU instruction costs the whole wave whatever its active lanes, so the four logs and
    // the three divisions run as one log and one division over lanes: lanes 0, 1 take log|delta_d| and
    // 1/lambda_d, lanes 2, 3 log|lambda_{d-2}|, lane 2 also 2/v'v.
    double vr = lane < 2 ? v_l : 0.0;
    double pv = vr * vr;
    pv += __shfl_xor(pv, 1);  // lanes 0, 1: v0^2 + v1^2 (build_program's one butterfly stage)
    const double lg = log(fabs(lane < 2 ? d_l : lam_l));  // lanes 0..3
    const double pvb = __shfl(pv, 0);
    const double qt = (lane < 2 ? 1.0 : 2.0) / (lane < 2 ? lam_l : pvb);  // 1/lambda_d; lane 2: 2/v'v
    double pc = lg - __shfl_down(lg, 2);  // lanes 0, 1: log|delta_d| - log|lambda_d|
    pc += __shfl_xor(pc, 1);
    const double hscale = sqrt(d2_readlane(qt, 2));
    const double vh = vr * hscale;
    P_.vh0 = d2_readlane(vh, 0);
    P_.vh1 = d2_readlane(vh, 1);
    P_.il0 = d2_readlane(qt, 0);
    P_.il1 = d2_readlane(qt, 1);
    P_.ctot = (0.0 + 0.0) + d2_readlane(pc, 0);  // the step constants summed in step order (H: 0)
    if (PB && lane == 0) {
      progl[0] = P_.vh0; progl[1] = P_.vh1; progl[2] = P_.il0; progl[3] = P_.il1; progl[4] = P_.ctot;
      progl[5] = P_.g0; progl[6] = P_.g1; progl[7] = P_.d0; progl[8] = P_.d1; progl[9] = P_.xi0; progl[10] = P_.xi1;
    }
    }
    if constexpr (PB) {  // LDS-only barrier: the prefetched tiles stay in flight
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      P_.vh0 = progl[0]; P_.vh1 = progl[1]; P_.il0 = progl[2]; P_.il1 = progl[3]; P_.ctot = progl[4];
      P_.g0 = progl[5]; P_.g1 = progl[6]; P_.d0 = progl[7]; P_.d1 = progl[8]; P_.xi0 = progl[9]; P_.xi1 = progl[10];
    }
    // the table writes are complete before any lane of this wave reads it (LDS is in order per wave)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  };
  const bool full0 = wave_id < ntiles_full;
  if (full0) {
    // the first P tiles, unconditionally (d2_load: a tile past the wave's last reads one line), so the
    // prologue's waits count only its own loads
#pragma unroll
    for (int k = 0; k < (LO == 1 ? 1 : P); ++k) {
      const int64_t tk = wave_id + k * nwaves;
      d2_load<U, false, DBG, NT>(a, tk * CT, lane, xs[k], tk < ntiles_full);
    }
    __builtin_amdgcn_sched_barrier(0);
    prologue();
    if constexpr (LO == 1) {
#pragma unroll
      for (int k = 1; k < P; ++k) {
        const int64_t tk = wave_id + k * nwaves;
        d2_load<U, false, DBG, NT>(a, tk * CT, lane, xs[k], tk < ntiles_full);
      }
    }
    // persistent loop over groups of P tiles, P tiles in flight: compute buffer k, then refill it with the
    // tile P strides ahead. No conditionals inside a group and the remainder nested (d2_rem), so every
    // path into a tile has issued the same loads and stores before it and the vmcnt waits stay static:
    // with the round-2 loop's per-tile `done` exits the compiler merged paths with fewer loads in flight
    // and waited for vmcnt(0) at the top of every group.
    const int64_t nt_w = (ntiles_full - 1 - wave_id) / nwaves + 1;  // this wave's tiles, >= 1
    int64_t t = wave_id;
    for (int64_t g = nt_w / P; g > 0; --g) {
#pragma unroll
      for (int k = 0; k < P; ++k) {
        d2_tile<U, LM, false, DBG, TB, NT>(a, P_, tab, t * CT, lane, xs[k]);
        const int64_t tn = t + P * nwaves;
        d2_load<U, false, DBG, NT>(a, tn * CT, lane, xs[k], tn < ntiles_full);
        t += nwaves;
      }
    }
    d2_rem<0, P, U, LM, DBG, TB, NT>(a, P_, tab, (int)(nt_w % P), t, nwaves, lane, xs);
  } else {
    prologue();
  }
  if (ntiles_full * CT < a.N && wave_id == ntiles_full % nwaves) {
    const int64_t c0 = ntiles_full * CT;
    d2_load<U, true, 0>(a, c0, lane, xs[0]);
    d2_tile<U, LM, true, 0, TB>(a, P_, tab, c0, lane, xs[0]);
  }
}

// Eligible: fp64, D = 2, fragment layout (contiguous, 16-byte aligned columns), exactly one single-column
// reflection followed by one Johnson layer.
bool d2_program(const FlowArgs& a) {
  return a.frag && a.D == 2 && a.nsteps == 2 && a.steps[0].op == OP_HOUSEHOLDER && a.steps[1].op == OP_JOHNSON;
}

template <int U, int LM, int DBG, int P = 2, bool PB = false, int TB = 5, int NT = 3, int LO = 0>
static hipError_t launch_d2_u(const D2Args& h, hipStream_t st, const DeviceInfo& dev) {
  const size_t lds = 4 * d2_tab_doubles(TB) * sizeof(double) + 16 * sizeof(double);
  const void* k = reinterpret_cast<const void*>(&flow_d2_kernel<U, LM, DBG, P, PB, TB, NT, LO>);
  int64_t blocks = 0;
  hipError_t e = frag_grid(k, h.N, (int64_t)64 * U * 4, lds, dev, &blocks);
  if (e != hipSuccess) return e;
  // three blocks per CU (3 waves per SIMD, ~2.5 tiles per wave at N = 1e6): every wave pays the prologue,
  // so fewer, longer waves beat full occupancy. Round 2 (prologue after the tiles) measured 2 blocks best
  // (11.2 vs 11.9 us; 1 block per CU: 12.6 us, profiles/r02_c2_d2_ab.txt); with the round-3 prologue
  // issued ahead of the tiles, 3 blocks: 10.63 / 10.65 vs 11.30 / 11.45 us warm for 2, 10.93 vs 10.89 cold;
  // 4 / 5 blocks 11.4 / 11.4-11.9 (profiles/r03_c2_bpc_sweep.txt). ENF_BLOCKS_PER_CU overrides in the
  // diagnostics build.
  static const int bpc_env = ENF_KNOB("ENF_BLOCKS_PER_CU", 0);
  const int64_t cap = (int64_t)dev.num_cu * 3;
  if (bpc_env == 0 && blocks > cap) blocks = cap;
  hipLaunchKernelGGL((flow_d2_kernel<U, LM, DBG, P, PB, TB, NT, LO>), dim3((unsigned)blocks), dim3(256), lds, st, h);
  return hipGetLastError();
}

template <int LM>
static hipError_t launch_d2_lm(const D2Args& h, hipStream_t st, const DeviceInfo& dev) {
#if ENF_DIAG
  // ENF_D2_U: columns per lane per tile (2 default; 1: 49 VGPRs, 8 waves per SIMD); ENF_D2_DBG 1 / 2:
  // synthesized tile / also no stores
  static const int u = ENF_KNOB("ENF_D2_U", 2);
  static const int dbg = ENF_KNOB("ENF_D2_DBG", 0);
  // ENF_D2_P: tiles in flight per wave
  static const int pf = ENF_KNOB("ENF_D2_P", 4);
  static const int pb = ENF_KNOB("ENF_D2_PB", 0);
  constexpr int tb = 5;  // log table index bits (B = 7 / 8: rejected in round 4, sources removed in round 6)
  // ENF_D2_LO=1: the first tile before the prologue, the rest after it
  static const int lo = ENF_KNOB("ENF_D2_LO", 0);
  if (lo == 1 && dbg == 0 && u == 2 && pb == 0 && tb == 5) {
    if (pf == 4) return launch_d2_u<2, LM, 0, 4, false, 5, 3, 1>(h, st, dev);
    if (pf == 3) return launch_d2_u<2, LM, 0, 3, false, 5, 3, 1>(h, st, dev);
  }
  // ENF_D2_NT: bit 0 nontemporal X loads, bit 1 nontemporal Y stores (3 default)
  static const int nt = ENF_KNOB("ENF_D2_NT", 3);
  if ((dbg == 0 || dbg == 3) && u == 2 && pb == 0 && pf == 4 && nt != 3) {
    if (dbg == 0) {
      if (nt == 0) return launch_d2_u<2, LM, 0, 4, false, 5, 0>(h, st, dev);
      if (nt == 1) return launch_d2_u<2, LM, 0, 4, false, 5, 1>(h, st, dev);
      return launch_d2_u<2, LM, 0, 4, false, 5, 2>(h, st, dev);
    }
    if (nt == 0) return launch_d2_u<2, LM, 3, 4, false, 5, 0>(h, st, dev);
    if (nt == 1) return launch_d2_u<2, LM, 3, 4, false, 5, 1>(h, st, dev);
    return launch_d2_u<2, LM, 3, 4, false, 5, 2>(h, st, dev);
  }
  if (dbg == 3) return launch_d2_u<2, LM, 3, 4>(h, st, dev);
  if (dbg == 0 && u == 2 && pb == 1 && pf == 4) return launch_d2_u<2, LM, 0, 4, true>(h, st, dev);
  if (dbg == 0 && u == 2 && pb == 1 && pf == 2) return launch_d2_u<2, LM, 0, 2, true>(h, st, dev);
  if (dbg == 2 && pb == 1) return launch_d2_u<2, LM, 2, 4, true>(h, st, dev);
  if (dbg == 0 && u == 2 && pf == 3) return launch_d2_u<2, LM, 0, 3>(h, st, dev);
  if (dbg == 0 && u == 2 && pf == 2) return launch_d2_u<2, LM, 0, 2>(h, st, dev);
  if (dbg == 0 && u == 1 && pf == 4) return launch_d2_u<1, LM, 0, 4>(h, st, dev);
  if (dbg == 1) return launch_d2_u<2, LM, 1>(h, st, dev);
  if (dbg == 2) return launch_d2_u<2, LM, 2>(h, st, dev);
  if (u == 1) return launch_d2_u<1, LM, 0>(h, st, dev);
#endif
  // U = 2, 4 tiles in flight per wave (85 VGPRs; P = 4 vs 2: 11.70 vs 12.00 us on one box,
  // profiles/r03_c2_variants.txt); U = 4 interleaves 8 asinh chains and spilled at 128 VGPRs (round 2)
  return launch_d2_u<2, LM, 0, 4>(h, st, dev);
}

hipError_t launch_d2_program(const FlowArgs& a, int lm, hipStream_t st, const DeviceInfo& dev) {
  D2Args h;
  std::memset(&h, 0, sizeof h);
  h.X = (const double*)a.X;
  h.Y = (double*)a.Y;
  h.ladj = (double*)a.ladj;
  h.N = a.N;
  const Step& sh = a.steps[0];
  const LayerDesc& J = a.layers[a.steps[1].layer];
  h.v = (const double*)a.layers[sh.layer].p[0] + (int64_t)sh.col * 2;
  h.g = (const double*)J.p[0];
  h.d = (const double*)J.p[1];
  h.xi = (const double*)J.p[2];
  h.lam = (const double*)J.p[3];
  if (lm == 0) return launch_d2_lm<0>(h, st, dev);
  if (lm == 1) return launch_d2_lm<1>(h, st, dev);
  return launch_d2_lm<2>(h, st, dev);
}

}  // namespace enf
