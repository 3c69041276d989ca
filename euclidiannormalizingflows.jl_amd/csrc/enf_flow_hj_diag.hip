// enf_flow_hj_diag.hip -- diagnostics build only (libenf_diag.so, tools/): the A/B variants of the compiled
// (J o H)^n program that were measured and rejected, selected by ENF_* knobs (enf_internal.h ENF_KNOB):
//   ENF_HJ_SPEC=1     the wave-specialised kernel flow_hjs_kernel (transcendentals on waves of their own)
//   ENF_HJ_ASINH=0/2/3 the asinh form (round 1's absolute-error form / the one-med3 clamp / the older merge)
//   ENF_DEBUG_MODE    1 = synthesized tile, 2 = no stores either, 8 = nontemporal loads, 9 = plain stores
// diag_dispatch_hj returns hipErrorNotSupported when no knob applies (the product kernel then runs).
#include "enf_hj.h"

namespace enf {

// ---------------------------------------------------------------------------------------------------
// Wave-specialised form of the same program (round 3): the transcendentals on waves of their own.
//
// On gfx950 a v_sqrt / v_log interleaved with a wave's own FMAs costs ~5.5 ns of SIMD time instead of the
// ~3.7 ns it costs in a run of transcendentals (tools/microbench21: 224 FMAs + 32 transcendentals per wave,
// 416 ns per wave-iteration vs 240 + 118 alone), while transcendentals issued by OTHER waves of the SIMD
// largely overlap a wave's FMA stream (tools/microbench22: two FMA waves + two transcendental waves per SIMD
// 1.27 ms vs 1.67 ms for the same work mixed in every wave). So a block of 16 waves splits each pair:
//  * F waves (0-7, two per SIMD) own the tiles: dot, reflection and z of pair p; later the small-|z| form,
//    the merge and y = gamma + delta' L of pair p (the shipped kernel's operations, in its order);
//  * T waves (8-15, two per SIMD; T wave 8 + f serves F wave f) take z through LDS and return
//    t = log2(|z| + sqrt(1 + z^2)); they also keep the ladj (the -1/2 log2 of the q product of a lane's 8
//    rows, one log2 per 8 rows, as before) and store it, and stage the next tiles' X through LDS.
// Every F wave keeps two tiles in flight (slots A and B, one step apart), so that while the T wave works on
// one slot's transcendentals the F wave works on the other slot. Steps are paced by one block barrier; a
// step moves 16 values per lane each way. Identical arithmetic to flow_hj_kernel (AS = 1), so identical
// results; the exact-range redo of a tile whose q product overflows is run by its F wave.
// MEASURED AND REJECTED (diagnostics build only, ENF_HJ_SPEC=1): bit-identical outputs but 0.97 vs 0.78 ms at
// D = 32 and 0.99 vs 0.80 ms at D = 64 (profiles/r03_hjs_spec_ab.jsonl) -- one block barrier per step puts all
// F waves of a SIMD in the same phase, so the LDS round trips and the dot's DPP chain of each step are exposed
// instead of hidden behind the other waves' work; the synthetic form of the same pacing
// (tools/microbench23: 975 ns per step against 888 for the mixed stream) showed the same.
constexpr int kHjSpecDefault = 0;         // product default of ENF_HJ_SPEC (dispatch_hj)
constexpr int kHjsF = 8;                  // F waves per block; T waves kHjsF .. 2 kHjsF - 1
constexpr int kHjsSlot = 64 * 16;         // floats of one slot: 16 values per lane
constexpr size_t kHjsStage = (size_t)2 * kHjsF * kStagePerWave * sizeof(float);
constexpr size_t kHjsFlags = 16 * sizeof(int);  // overflow flag per F wave and slot
constexpr size_t kHjsExch = (size_t)kHjsF * 2 * kHjsSlot * sizeof(float);  // z / t exchange
constexpr size_t kHjsXArea = kHjsExch;                                      // next tiles' X
static size_t hjs_lds_bytes(int D, int n) {
  return kHjScratch + kHjsStage + kHjsFlags + kHjsExch + kHjsXArea + (size_t)(n + 1) * kHjW * D * sizeof(float);
}

// LDS slot of one lane: 16 values in 4 16-byte vectors at a stride of 1 KiB (conflict-free b128 access)
template <int R, int U>
__device__ __forceinline__ void slot_write(float* __restrict__ slot, int lane, const float (&v)[U][R]) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int h = 0; h < R / 4; ++h) {
      u32x4 w;
      __builtin_memcpy(&w, &v[u][4 * h], 16);
      *reinterpret_cast<u32x4*>(slot + (u * (R / 4) + h) * 256 + 4 * lane) = w;
    }
}
template <int R, int U>
__device__ __forceinline__ void slot_read(const float* __restrict__ slot, int lane, float (&v)[U][R]) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int h = 0; h < R / 4; ++h) {
      const u32x4 w = *reinterpret_cast<const u32x4*>(slot + (u * (R / 4) + h) * 256 + 4 * lane);
      __builtin_memcpy(&v[u][4 * h], &w, 16);
    }
}

// F: y of pair p - 1 from the T wave's t (x holds that pair's z on entry), record r = record p
template <int R, int U>
__device__ __forceinline__ void hjs_merge(float (&x)[U][R], const float (&t)[U][R], const HJParams<R>& prm,
                                          uint32_t csign) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < R; ++e) {
      const float q = fmaf(x[u][e], x[u][e], 1.0f);
      const uint32_t m = asinh2_mask(q, csign);
      const float L = asinh2_pick(asinh2_small(x[u][e], q), t[u][e], m);
      x[u][e] = fmaf(L, prm.m(HJ_DP, e), prm.m(HJ_GP, e));
    }
}

// Y of a finished tile (F wave); the ladj is the T wave's
template <int D, int R, int U>
__device__ __forceinline__ void hjs_store_y(const HJArgs& a, int64_t col0, const float (&x)[U][R]) {
  using L = HJLay<D, R, U>;
  const int lane = threadIdx.x & 63;
  float* __restrict__ Y = (float*)a.Y;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t c = L::col(col0, u, lane);
#pragma unroll
    for (int h = 0; h < L::NF; ++h) {
      u32x4 v4;
      __builtin_memcpy(&v4, &x[u][4 * h], 16);
      if (ENF_INB(c < a.N, "hjs store Y", c, a.N))
        __builtin_nontemporal_store(v4, reinterpret_cast<u32x4*>(Y + c * D + L::row(h, lane)));
    }
  }
}

template <int D, int LM>
__global__ __launch_bounds__(1024, 1) void flow_hjs_kernel(HJArgs a) {
  constexpr int R = 8, U = 2;
  using L = HJLay<D, R, U>;
  constexpr int G = L::G;
  const int n = a.n;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* scr = reinterpret_cast<double*>(smem);
  float* ctotp = reinterpret_cast<float*>(scr + 2 * kHjMaxPairs);
  unsigned char* p0 = smem + kHjScratch;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  float* stage = reinterpret_cast<float*>(p0) + wave * kStagePerWave;
  int* flags = reinterpret_cast<int*>(p0 + kHjsStage);
  float* exch = reinterpret_cast<float*>(p0 + kHjsStage + kHjsFlags);
  float* xarea = exch + kHjsF * 2 * kHjsSlot;
  float* rec = xarea + kHjsF * 2 * kHjsSlot;
  const bool isF = wave < kHjsF;
  const int f = isF ? wave : wave - kHjsF;
  float* ex[2] = {exch + (2 * f) * kHjsSlot, exch + (2 * f + 1) * kHjsSlot};
  float* xa[2] = {xarea + (2 * f) * kHjsSlot, xarea + (2 * f + 1) * kHjsSlot};

  constexpr int64_t CT = L::TC;
  const int64_t ntiles = a.N / CT;
  const int64_t stride = (int64_t)gridDim.x * kHjsF;
  const int64_t g = (int64_t)blockIdx.x * kHjsF + f;  // this F wave's (or its partner's) tile stream
  const int64_t K = g < ntiles ? (ntiles - 1 - g) / stride + 1 : 0;
  const int64_t g0 = (int64_t)blockIdx.x * kHjsF;
  const int64_t Kmax = g0 < ntiles ? (ntiles - 1 - g0) / stride + 1 : 0;
  auto tile_col = [&](int64_t k) { return (g + k * stride) * CT; };

  // T waves: the first tile of each slot, loaded before the prologue
  float xt[2][U][R];
  if (!isF) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (s < K) hj_load<D, R, U, false, 0>(a, tile_col(s), xt[s]);
  }
  build_hj_program<D, R, 1>(a, n, rec, scr, ctotp);  // ends with a block barrier
  const float ctot = *ctotp;
  const float* recl = rec + (lane % G) * kHjW * R;
  if (!isF) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (s < K) slot_write<R, U>(xa[s], lane, xt[s]);
    if (lane < 2) flags[2 * f + lane] = 0;
  }
  __syncthreads();

  // steps: slot A (X = 0) holds tiles 0, 2, 4, ... of the stream and gets F steps 0, 2, 4, ...; slot B tiles
  // 1, 3, ... and steps 1, 3, ...; a tile takes n F steps (pair p's z phase, merged with pair p - 1's y),
  // its last y comes with the first step of the slot's next tile. T processes at step s the slot F touched
  // at step s - 1.
  const int64_t nA = (Kmax + 1) / 2, nB = Kmax / 2;
  const int64_t S = Kmax == 0 ? 0 : ((2 * n * nA > 2 * n * nB + 1) ? 2 * n * nA : 2 * n * nB + 1) + 1;
  const uint32_t csign = sign_mask_vgpr();
  float x[2][U][R];        // F: the two slots' tiles (z after a z phase, y after a merge)
  float acc[2][U] = {};    // T: ladj partials of the two slots' tiles
  float mx[2] = {0.f, 0.f};  // T: largest q product of the slot's tile
  HJParams<R> prm;

  auto f_step = [&](auto XC, int64_t s) {
    constexpr int X = decltype(XC)::value;
    if (s < X) return;
    const int64_t q = (s - X) >> 1;
    const int64_t j = q / n;
    const int p = (int)(q - j * n);
    const int64_t k = 2 * j + X;
    if (p == 0 && j > 0 && k - 2 < K) {
      // the slot's previous tile: its last y (record n), or the exact-range redo from X
      const int64_t c0 = tile_col(k - 2);
      if (flags[2 * f + X] == 0) {
        float t[U][R];
        slot_read<R, U>(ex[X], lane, t);
        prm.template load<0, HJ_IL>(recl + n * kHjW * D);
        hjs_merge<R, U>(x[X], t, prm, csign);
        hjs_store_y<D, R, U>(a, c0, x[X]);
      } else {
        float old[L::NLS];
        hj_load<D, R, U, false, 0>(a, c0, x[X]);
        hj_load_old<D, R, U, LM>(a, c0, old, false);
        float accx[U];
#pragma unroll
        for (int u = 0; u < U; ++u) accx[u] = 0.f;
        const float* r = recl;
        HJParams<R> pe;
        pe.template load<0, HJ_IL>(r);
        for (int pp = 0; pp < n; ++pp) hj_pair_exact<D, R, U, LM != 0, 1>(x[X], accx, r, pe);
        hj_store<D, R, U, LM, false, 0>(a, ctot, c0, x[X], accx, old, stage);
      }
    }
    if (k >= K) return;
    const float* rp = recl + p * kHjW * D;
    prm.template load<0, HJ_IL>(rp);
    if (p == 0) {
      slot_read<R, U>(xa[X], lane, x[X]);
    } else {
      float t[U][R];
      slot_read<R, U>(ex[X], lane, t);
      hjs_merge<R, U>(x[X], t, prm, csign);
    }
    hj_pair_z<D, R, U>(x[X], rp, prm);
    slot_write<R, U>(ex[X], lane, x[X]);
  };

  auto t_step = [&](auto YC, int64_t s) {
    constexpr int Y = decltype(YC)::value;
    if (s < Y + 1) return;
    const int64_t q = (s - 1 - Y) >> 1;
    const int64_t j = q / n;
    const int p = (int)(q - j * n);
    const int64_t k = 2 * j + Y;
    if (k >= K) return;
    if (p == 0 && k + 2 < K) hj_load<D, R, U, false, 0>(a, tile_col(k + 2), xt[Y]);  // the slot's next tile
    float z[U][R], t[U][R];
    slot_read<R, U>(ex[Y], lane, z);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float qv[R];
#pragma unroll
      for (int e = 0; e < R; ++e) qv[e] = fmaf(z[u][e], z[u][e], 1.0f);
      sqrt8(t[u], qv);
      const float pr = prod_tree<R>(qv);
#pragma unroll
      for (int e = 0; e < R; ++e) t[u][e] = fabsf(z[u][e]) + t[u][e];
      log2_8_inplace(t[u]);
      if (LM > 0) acc[Y][u] = fmaf(-0.5f, hw_log2(pr), acc[Y][u]);
      mx[Y] = fmaxf(mx[Y], pr);
    }
    slot_write<R, U>(ex[Y], lane, t);
    if (p == n - 1) {
      // tile done: the F wave redoes it in the exact form when some q product overflowed (+Inf / NaN)
      const bool ovf = __any(!(mx[Y] <= FLT_MAX));
      if (lane == 0) flags[2 * f + Y] = ovf ? 1 : 0;
      if (LM > 0 && !ovf) {
        const int64_t c0 = tile_col(k);
        float old[L::NLS];
        hj_load_old<D, R, U, LM>(a, c0, old, false);
        float* __restrict__ ladj = (float*)a.ladj;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const float tot = group_sum<G>(acc[Y][u]);
          if ((lane % G) == 0) stage[u * L::CPS + lane / G] = tot;
        }
#pragma unroll
        for (int kk = 0; kk < L::NLS; ++kk) {
          const int c = kk * 64 + (L::TC >= 64 ? lane : lane % L::TC);
          const float v = fmaf((float)kLn2, stage[c], ctot) + old[kk];
          if (ENF_INB(c0 + c < a.N, "hjs ladj", c0 + c, a.N)) ladj[c0 + c] = v;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc[Y][u] = 0.f;
      mx[Y] = 0.f;
      if (k + 2 < K) slot_write<R, U>(xa[Y], lane, xt[Y]);  // waits for the load issued at p == 0
    }
  };

  // one loop per role (wave-uniform branch; both execute the same S barriers), so that neither keeps the
  // other's registers live
  if (isF) {
    for (int64_t s = 0; s < S; s += 2) {
      f_step(std::integral_constant<int, 0>{}, s);
      __syncthreads();
      if (s + 1 < S) {
        f_step(std::integral_constant<int, 1>{}, s + 1);
        __syncthreads();
      }
    }
  } else {
    for (int64_t s = 0; s < S; s += 2) {
      t_step(std::integral_constant<int, 1>{}, s);
      __syncthreads();
      if (s + 1 < S) {
        t_step(std::integral_constant<int, 0>{}, s + 1);
        __syncthreads();
      }
    }
  }
  // the ragged last tile: one F wave, whole program in its own registers (flow_hj_kernel's tail path)
  if (isF && ntiles * CT < a.N && g == ntiles % stride) {
    HJBody<D, R, U, LM, 1, 0> body{a, recl, ctot, stage, n};
    const int64_t c0 = ntiles * CT;
    float xt0[U][R], old[L::NLS];
    hj_load<D, R, U, true, 0>(a, c0, xt0);
    hj_load_old<D, R, U, LM>(a, c0, old, true);
    body.template tile<true, 0>(c0, xt0, old);
  }
}

// one block of 16 waves per CU
template <int D, int LM>
static hipError_t launch_hjs(const HJArgs& h, hipStream_t st, const DeviceInfo& dev) {
  const size_t lds = hjs_lds_bytes(D, h.n);
  const void* k = reinterpret_cast<const void*>(&flow_hjs_kernel<D, LM>);
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  int64_t blocks = dev.num_cu;
  const int64_t need = (h.N + (int64_t)HJLay<D, 8, 2>::TC * kHjsF - 1) / ((int64_t)HJLay<D, 8, 2>::TC * kHjsF);
  if (blocks > need) blocks = need > 0 ? need : 1;
  hipLaunchKernelGGL((flow_hjs_kernel<D, LM>), dim3((unsigned)blocks), dim3(1024), lds, st, h);
  return hipGetLastError();
}

// R = 8 rows per lane, U = 2 slabs (16 values per lane). Diagnostics build only (ENF_DIAG):
// ENF_DEBUG_MODE 1/2 (synthesized tile / no stores), ENF_HJ_ASINH = 0/2 (round 1's asinh form / the
// one-med3 clamp asinh2_med3 in place of the four-op merge: 9% faster, rejected for its coherent bias,
// DESIGN.md §3).
template <int DBG, int LM>
static hipError_t launch_hj_as(int as, const HJArgs& a, hipStream_t st, const DeviceInfo& dev) {
  if (as == 0) return launch_hj<32, 8, 2, LM, 4, DBG, 0>(a, st, dev);
  if (as == 2) return launch_hj<32, 8, 2, LM, 4, DBG, 2>(a, st, dev);
  if (as == 3) return launch_hj<32, 8, 2, LM, 4, DBG, 3>(a, st, dev);
  return launch_hj<32, 8, 2, LM, 4, DBG, 1>(a, st, dev);
}

// ---------------------------------------------------------------------------------------------------
// Mailbox form (round 4): the transcendentals on waves of their own WITHOUT a block
// barrier per step. A block of 8 waves: F waves 0-3 and T waves 4-7, F wave f paired with T wave f + 4 (the
// same SIMD when waves are placed round-robin), two blocks per CU (2 F + 2 T waves per SIMD).
//  * F owns the tiles' arithmetic: per pair the merge of the previous pair's asinh (the small-|z| form, the
//    mask, the pick -- the product's operations), y = gamma + delta' L, the reflection and z; Y stores.
//  * T takes z through its LDS mailbox and returns t = log2(|z| + sqrt(1 + z^2)) in place; it keeps the
//    ladj (-1/2 log2 of the q product of a lane's 8 rows) and stores it; it loads X from HBM and hands each
//    new tile to F through a second mailbox buffer.
// Each F wave keeps two tiles in flight (slots A and B): while T works on one slot F works on the other.
// Pacing is by per-slot sequence flags in LDS (written by one lane after the data, s_waitcnt lgkmcnt(0)
// between; polled with s_sleep), never a block barrier. Every wait is bounded (kMbSpinMax polls): a wave that
// runs out sets err and moves on, so the grid always drains (wrong results, never a hang).
// Same arithmetic as flow_hj_kernel (AS = 1), so the same results; a tile whose q product overflows is
// flagged by T with its last t and redone by F in the exact-range form (Y and ladj).
constexpr int kMbF = 4;                                      // F waves per block (T waves kMbF .. 2 kMbF - 1)
constexpr int kMbSlot = 64 * 16;                             // floats of one mailbox buffer: 16 values per lane
constexpr size_t kMbPair = (size_t)2 * 2 * kMbSlot * sizeof(float);  // per F/T pair: 2 slots x {zt, xb}
constexpr size_t kMbStage = (size_t)2 * kMbF * kStagePerWave * sizeof(float);
constexpr size_t kMbFlags = 0;  // (the flags are a static __shared__ array: per pair zf[2], tf[2], xf[2], err, pad)
constexpr int kMbSpinMax = 1 << 16;  // ~4M clocks of s_sleep 1 per wait: a broken schedule drains in seconds
static size_t hjm_lds_bytes(int D, int n) {
  return kHjScratch + kMbStage + kMbFlags + kMbF * kMbPair + (size_t)(n + 1) * kHjW * D * sizeof(float);
}

// mailbox flags: words of a static __shared__ array, read and written as relaxed workgroup-scope atomics (each
// access is a ds_read_b32 / ds_write_b32 that the compiler neither caches nor drops)
typedef int mb_flag;

template <int NOWAIT>
__device__ __forceinline__ void mb_publish(mb_flag* f, int v, int lane) {
  // the mailbox data before its flag: DS operations of a wave complete in order, and the wait makes sure
  if constexpr (!NOWAIT) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else asm volatile("" ::: "memory");
  if (lane == 0) __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ int mb_load(mb_flag* f) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// returns the flag value once (v >> sh) >= want (wave-uniform), or after kMbSpinMax polls with *err set
template <int SLEEP>
__device__ __forceinline__ int mb_wait(mb_flag* f, int want, int sh, mb_flag* err, int lane) {
  int v = mb_load(f);
  for (int i = 0; (v >> sh) < want; ++i) {
    if (i >= (SLEEP ? kMbSpinMax : 64 * kMbSpinMax)) {
      if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      break;
    }
    if constexpr (SLEEP) __builtin_amdgcn_s_sleep(1);
    v = mb_load(f);
  }
  asm volatile("" ::: "memory");
  return v;
}

template <int D, int LM, int NOWAIT, int SLEEP = 1>
__global__ __launch_bounds__(512, 4) void flow_hjm_kernel(HJArgs a, int* errp) {
  constexpr int R = 8, U = 2;
  using L = HJLay<D, R, U>;
  constexpr int G = L::G;
  const int n = a.n;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* scr = reinterpret_cast<double*>(smem);
  float* ctotp = reinterpret_cast<float*>(scr + 2 * kHjMaxPairs);
  unsigned char* p0 = smem + kHjScratch;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  float* stage = reinterpret_cast<float*>(p0) + wave * kStagePerWave;
  const bool isF = wave < kMbF;
  const int f = isF ? wave : wave - kMbF;
  __shared__ int mb_flags[kMbF * 8];
  mb_flag* flags = mb_flags + f * 8;
  mb_flag* zf = flags;      // [2] F -> T: z of step s in zt[S]
  mb_flag* tf = flags + 2;  // [2] T -> F: 2 s + ovf, t of step s in zt[S]
  mb_flag* xf = flags + 4;  // [2] T -> F: tile k of the slot in xb[S]
  mb_flag* err = flags + 6;
  float* mb = reinterpret_cast<float*>(p0 + kMbStage + kMbFlags + (size_t)f * kMbPair);
  // (no arrays of pointers or runtime slot indices below: they would put the tiles in scratch memory)
  auto zt = [&](int S) { return mb + S * kMbSlot; };
  auto xb = [&](int S) { return mb + (2 + S) * kMbSlot; };
  float* rec = reinterpret_cast<float*>(p0 + kMbStage + kMbFlags + (size_t)kMbF * kMbPair);

  constexpr int64_t CT = L::TC;
  const int64_t ntiles = a.N / CT;
  const int64_t P = (int64_t)gridDim.x * kMbF;
  const int64_t g = (int64_t)blockIdx.x * kMbF + f;
  const int64_t K = g < ntiles ? (ntiles - 1 - g) / P + 1 : 0;  // full tiles of this pair
  const int64_t KA = (K + 1) / 2, KB = K / 2;                   // tiles of slot A / B
  auto KS = [&](int S) { return S ? KB : KA; };
  auto tile_col = [&](int S, int64_t k) { return (g + (2 * k + S) * P) * CT; };

  float xt[2][U][R];  // T: the next tile of each slot (registers until its mailbox buffer is free)
  if (!isF) {
    if (KA > 0) hj_load<D, R, U, false, 0>(a, tile_col(0, 0), xt[0]);
    if (KB > 0) hj_load<D, R, U, false, 0>(a, tile_col(1, 0), xt[1]);
  }
  build_hj_program<D, R, 1>(a, n, rec, scr, ctotp);  // ends with a block barrier
  const float ctot = *ctotp;
  const float* recl = rec + (lane % G) * kHjW * R;
  if (!isF) {
    if (KA > 0) slot_write<R, U>(xb(0), lane, xt[0]);
    if (KB > 0) slot_write<R, U>(xb(1), lane, xt[1]);
    if (lane < 7) flags[lane] = lane >= 4 ? 0 : -1;  // zf, tf = -1; xf = 0 (tile 0 of each slot is in xb); err 0
    if (KA > 1) hj_load<D, R, U, false, 0>(a, tile_col(0, 1), xt[0]);
    if (KB > 1) hj_load<D, R, U, false, 0>(a, tile_col(1, 1), xt[1]);
  }
  __syncthreads();

  const int64_t stA = KA * n, stB = KB * n;
  const int64_t smax = stA > stB ? stA : stB;
  const uint32_t csign = sign_mask_vgpr();
  if (isF) {
    float x[2][U][R];  // z of the slot's current pair after its phase
    HJParams<R> prm;
    // the end of tile k - 1 of slot S (t of its last pair in zt[S]): y of the last pair, Y (or the exact redo)
    auto finish = [&](auto SC, int64_t k, int tv) {
      constexpr int S = decltype(SC)::value;
      const int64_t c0 = tile_col(S, k);
      if ((tv & 1) == 0) {
        float t[U][R];
        slot_read<R, U>(zt(S), lane, t);
        prm.template load<0, HJ_IL>(recl + n * kHjW * D);
        hjs_merge<R, U>(x[S], t, prm, csign);
        hjs_store_y<D, R, U>(a, c0, x[S]);
      } else {
        float old[L::NLS], accx[U];
        hj_load<D, R, U, false, 0>(a, c0, x[S]);
        hj_load_old<D, R, U, LM>(a, c0, old, false);
#pragma unroll
        for (int u = 0; u < U; ++u) accx[u] = 0.f;
        const float* r = recl;
        HJParams<R> pe;
        pe.template load<0, HJ_IL>(r);
        for (int pp = 0; pp < n; ++pp) hj_pair_exact<D, R, U, LM != 0, 1>(x[S], accx, r, pe);
        hj_store<D, R, U, LM, false, 0>(a, ctot, c0, x[S], accx, old, stage);
      }
    };
    auto phase = [&](auto SC, int64_t s) {
      constexpr int S = decltype(SC)::value;
      const int64_t k = s / n;
      const int p = (int)(s - k * n);
      const float* rp = recl + p * kHjW * D;
      if (p == 0) {
        if (k > 0) finish(SC, k - 1, mb_wait<SLEEP>(tf + S, (int)s - 1, 1, err, lane));
        (void)mb_wait<SLEEP>(xf + S, (int)k, 0, err, lane);
        slot_read<R, U>(xb(S), lane, x[S]);
        prm.template load<0, HJ_IL>(rp);  // (vh of pair 0: hj_pair_z reads the other slots)
      } else {
        (void)mb_wait<SLEEP>(tf + S, (int)s - 1, 1, err, lane);
        float t[U][R];
        slot_read<R, U>(zt(S), lane, t);
        prm.template load<0, HJ_IL>(rp);
        hjs_merge<R, U>(x[S], t, prm, csign);
      }
      hj_pair_z<D, R, U>(x[S], rp, prm);
      slot_write<R, U>(zt(S), lane, x[S]);
      mb_publish<NOWAIT>(zf + S, (int)s, lane);
    };
    for (int64_t s = 0; s < smax; ++s) {
      if (s < stA) phase(std::integral_constant<int, 0>{}, s);
      if (s < stB) phase(std::integral_constant<int, 1>{}, s);
    }
    if (KA > 0) finish(std::integral_constant<int, 0>{}, KA - 1, mb_wait<SLEEP>(tf, (int)stA - 1, 1, err, lane));
    if (KB > 0) finish(std::integral_constant<int, 1>{}, KB - 1, mb_wait<SLEEP>(tf + 1, (int)stB - 1, 1, err, lane));
  } else {
    float acc[2][U], mx[2];
#pragma unroll
    for (int S = 0; S < 2; ++S) {
      mx[S] = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) acc[S][u] = 0.f;
    }
    auto phase = [&](auto SC, int64_t s) {
      constexpr int S = decltype(SC)::value;
      const int64_t k = s / n;
      const int p = (int)(s - k * n);
      (void)mb_wait<SLEEP>(zf + S, (int)s, 0, err, lane);
      float z[U][R], t[U][R];
      slot_read<R, U>(zt(S), lane, z);
      if (p == 0 && k + 1 < KS(S)) {
        // F has read xb[S] for tile k (before writing z): hand over tile k + 1, load tile k + 2
        slot_write<R, U>(xb(S), lane, xt[S]);
        mb_publish<NOWAIT>(xf + S, (int)k + 1, lane);
        if (k + 2 < KS(S)) hj_load<D, R, U, false, 0>(a, tile_col(S, k + 2), xt[S]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float q[R];
#pragma unroll
        for (int e = 0; e < R; ++e) q[e] = fmaf(z[u][e], z[u][e], 1.0f);
        __builtin_amdgcn_s_setprio(3);
        sqrt8(t[u], q);
        __builtin_amdgcn_s_setprio(0);
        const float pr = prod_tree<R>(q);
#pragma unroll
        for (int e = 0; e < R; ++e) t[u][e] = fabsf(z[u][e]) + t[u][e];
        __builtin_amdgcn_s_setprio(3);
        log2_8_inplace(t[u]);
        __builtin_amdgcn_s_setprio(0);
        if (LM > 0) acc[S][u] = fmaf(-0.5f, hw_log2(pr), acc[S][u]);
        mx[S] = fmaxf(mx[S], pr);
      }
      slot_write<R, U>(zt(S), lane, t);
      int ovf = 0;
      if (p == n - 1) ovf = __any(!(mx[S] <= FLT_MAX)) ? 1 : 0;
      mb_publish<NOWAIT>(tf + S, 2 * (int)s + ovf, lane);
      if (p == n - 1) {
        if (LM > 0 && !ovf) {
          const int64_t c0 = tile_col(S, k);
          float old[L::NLS];
          hj_load_old<D, R, U, LM>(a, c0, old, false);
          float* __restrict__ ladj = (float*)a.ladj;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const float tot = group_sum<G>(acc[S][u]);
            if ((lane % G) == 0) stage[u * L::CPS + lane / G] = tot;
          }
#pragma unroll
          for (int kk = 0; kk < L::NLS; ++kk) {
            const int c = kk * 64 + (L::TC >= 64 ? lane : lane % L::TC);
            const float v = fmaf((float)kLn2, stage[c], ctot) + old[kk];
            if (ENF_INB(c0 + c < a.N, "hjm ladj", c0 + c, a.N)) ladj[c0 + c] = v;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc[S][u] = 0.f;
        mx[S] = 0.f;
      }
    };
    for (int64_t s = 0; s < smax; ++s) {
      if (s < stA) phase(std::integral_constant<int, 0>{}, s);
      if (s < stB) phase(std::integral_constant<int, 1>{}, s);
    }
  }
  // the ragged last tile: one F wave, the whole program in its own registers (flow_hj_kernel's tail path)
  if (isF && ntiles * CT < a.N && g == ntiles % P) {
    HJBody<D, R, U, LM, 1> body{a, recl, ctot, stage, n};
    const int64_t c0 = ntiles * CT;
    float xt0[U][R], old[L::NLS];
    hj_load<D, R, U, true, 0>(a, c0, xt0);
    hj_load_old<D, R, U, LM>(a, c0, old, true);
    body.template tile<true, 0>(c0, xt0, old);
  }
  if (mb_load(err) && lane == 0) atomicOr(errp, 1);
}

static int* g_mb_err = nullptr;  // device error word of the mailbox kernel (diagnostics: read by tools)

template <int D, int LM, int NOWAIT, int SLEEP = 1>
static hipError_t launch_hjm(const HJArgs& h, hipStream_t st, const DeviceInfo& dev) {
  if (!g_mb_err) {
    hipError_t e = hipMalloc(&g_mb_err, sizeof(int));
    if (e != hipSuccess) return e;
    e = hipMemset(g_mb_err, 0, sizeof(int));
    if (e != hipSuccess) return e;
  }
  const size_t lds = hjm_lds_bytes(D, h.n);
  const void* k = reinterpret_cast<const void*>(&flow_hjm_kernel<D, LM, NOWAIT, SLEEP>);
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  int per_cu = 0;
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 512, lds);
  if (e != hipSuccess) return e;
  if (per_cu < 1) per_cu = 1;
  static const int bpc = ENF_KNOB("ENF_HJ_MBOX_BPC", 2);
  if (per_cu > bpc) per_cu = bpc;
  int64_t blocks = (int64_t)dev.num_cu * per_cu;
  const int64_t need = (h.N + (int64_t)HJLay<D, 8, 2>::TC * kMbF - 1) / ((int64_t)HJLay<D, 8, 2>::TC * kMbF);
  if (blocks > need) blocks = need > 0 ? need : 1;
  hipLaunchKernelGGL((flow_hjm_kernel<D, LM, NOWAIT, SLEEP>), dim3((unsigned)blocks), dim3(512), lds, st, h, g_mb_err);
  return hipGetLastError();
}

template <int LM>
static hipError_t launch_hjm_d(int D, int nowait, const HJArgs& h, hipStream_t st, const DeviceInfo& dev) {
  if (D == 32 && nowait == 2) return launch_hjm<32, LM, 1, 0>(h, st, dev);  // busy polling, no s_sleep
  if (D == 32) return nowait ? launch_hjm<32, LM, 1>(h, st, dev) : launch_hjm<32, LM, 0>(h, st, dev);
  return nowait ? launch_hjm<64, LM, 1>(h, st, dev) : launch_hjm<64, LM, 0>(h, st, dev);
}

// the mailbox kernel's error word (1: some wave ran out of polls): read and cleared by tools (diagnostics)
extern "C" int enf_diag_mailbox_error(void) {
  if (!g_mb_err) return 0;
  int v = 0;
  if (hipMemcpy(&v, g_mb_err, sizeof v, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  (void)hipMemset(g_mb_err, 0, sizeof(int));
  return v;
}

hipError_t diag_dispatch_hj(const HJArgs& a, int D, int lm, int dbg, hipStream_t st, const DeviceInfo& dev) {
  if (a.dreal != D) return hipErrorNotSupported;  // (padded layout: product kernel only)
  static const int spec = ENF_KNOB("ENF_HJ_SPEC", kHjSpecDefault);
  if (spec && dbg == 0 && (D == 32 || D == 64)) {
    if (lm == 0) return D == 32 ? launch_hjs<32, 0>(a, st, dev) : launch_hjs<64, 0>(a, st, dev);
    if (lm == 1) return D == 32 ? launch_hjs<32, 1>(a, st, dev) : launch_hjs<64, 1>(a, st, dev);
    return D == 32 ? launch_hjs<32, 2>(a, st, dev) : launch_hjs<64, 2>(a, st, dev);
  }
  // ENF_HJ_MBOX: 1 = the mailbox kernel flow_hjm_kernel, 2 = the same without the lgkmcnt wait before a flag,
  // 3 = that and busy polling (no s_sleep)
  static const int mbox = ENF_KNOB("ENF_HJ_MBOX", 0);
  if (mbox && dbg == 0 && (D == 32 || D == 64)) {
    const int v = mbox == 3 ? 2 : mbox == 2 ? 1 : 0;
    if (lm == 0) return launch_hjm_d<0>(D, v, a, st, dev);
    if (lm == 1) return launch_hjm_d<1>(D, v, a, st, dev);
    return launch_hjm_d<2>(D, v, a, st, dev);
  }
  // ENF_HJ_R16 (round 4, last session): the D = 64 program with 16 rows per lane and one column per lane tile
  // (4 lanes per column: two DPP stages per dot instead of three, one ladj log2 per 16 rows) against the product's
  // 8 rows x 2 columns
  static const int r16 = ENF_KNOB("ENF_HJ_R16", 0);
  if (r16 && dbg == 0 && D == 64 && lm == 1) return launch_hj<64, 16, 1, 1, 4>(a, st, dev);
  if (D != 32 || lm != 1) return hipErrorNotSupported;
  static const int as = ENF_KNOB("ENF_HJ_ASINH", 1);
  if (dbg == 0 && as == 1) return hipErrorNotSupported;
  if (dbg == 1) return launch_hj_as<1, 1>(as, a, st, dev);
  if (dbg == 2) return launch_hj_as<2, 1>(as, a, st, dev);
  if (dbg == 8) return launch_hj_as<8, 1>(as, a, st, dev);
  if (dbg == 9) return launch_hj_as<9, 1>(as, a, st, dev);
  return launch_hj_as<0, 1>(as, a, st, dev);
}

}  // namespace enf
