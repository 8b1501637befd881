// drcvar_halfspace.hip — fused safe-halfspace kernel for MI355X (gfx950, CDNA4) + its C ABI.
//
// One workgroup evaluates one unit = one (obstacle, horizon step): N fp64 samples xi_i in R^2.
// Everything the reference does per unit in core/halfspaces.py:70-194 and core/risk_metrics.py:
// 84-338 happens in ONE pass over HBM (16 B per sample, read once, 16-B/lane coalesced loads):
//
//   1. load the samples into registers (P per thread); one block reduction gives the sums for the
//      mean AND the (pivot-shifted) second moments                        [barrier 1]
//   2. h = (mu - ego)/|mu - ego| ([1,0] if < 1e-10)            core/geometry.py:35-53
//      mean halfspace from the origin                           core/halfspaces.py:84-94
//   3. d_i = h . xi_i                                           core/risk_metrics.py:145,233
//   4. exact (m+1)-th order statistic tau of d, m = floor(alpha*N), sort-free: histogram of d in
//      LDS over [mean_d - 5 sd_d, mean_d + 5 sd_d] (clamped, so every map is monotone in d)
//                                                                         [barrier 2]
//      every wave scans the histogram -> target bucket; when it holds <= kCap samples (the normal
//      case) they are compacted per wave in a fixed order                 [barrier 3]
//      and wave 0 ranks them directly.  Otherwise the bucket is refined (exact min/max, re-histogram;
//      value-linear, then order-preserving integer keys) until <= kCap remain.  Because each map is
//      monotone, a candidate set is always a contiguous run of the sorted order: exact with ties.
//   5. L = tau + sum_{d<tau} (d - tau) / (alpha N)               lower-tail mean = -CVaR_alpha(-d)
//      (= (sum of the m smallest + (alpha N - m) tau) / (alpha N)); the tail sum is accumulated
//      relative to mean_d during the compaction pass, so no further reduction is needed.
//   6. g_cvar = r - delta - L, g* = r - delta + eps/alpha - L, g~ = g* - r, r = R_c |h|
//      (closed-form optimum of the LPs at core/risk_metrics.py:105-125 and :198-213;
//       lambda* = 1/alpha because lambda only enters the budget row and its bound, :110,:122)
//
// Wave reductions use DPP row permutations + readlane (no LDS round trips).  Every reduction and
// the candidate order are fixed, so results are bitwise reproducible run to run.
// No MFMA: ~10 flops per 16-B sample — the kernel is bounded by HBM.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "drcvar_exchange.h"
#include "drcvar_halfspace.h"

namespace {

constexpr int kWave = 64;
constexpr int kCap = 128;          // candidates ranked directly (per-wave region size in LDS)
constexpr int kMaxValueIters = 3;  // value-linear refinements before switching to integer keys
constexpr double kSentinel = 100.0;
// sample load forms (kernel template)
constexpr int kLoadPair = 0, kLoadVec = 1, kLoadNt = 2;
constexpr int64_t kNtBytes = 256ll << 20;  // launches reading more than the MALL use kLoadNt
typedef double dbl2 __attribute__((ext_vector_type(2)));

#ifdef DRCVAR_STAMPS
// diagnostic build only: per-unit shader-clock stamps at phase boundaries (wave 0)
#ifdef DRCVAR_STAMPS_WAVES  // + per-wave stamps (slots 8 + 4j + wave) around the load phase
constexpr int kStampUnits = 16384, kStamps = 16;
#else
constexpr int kStampUnits = 16384, kStamps = 8;
#endif
__device__ unsigned long long g_stamps[kStampUnits * kStamps];
#define DRCVAR_STAMP(k)                                                                       \
  do {                                                                                        \
    const unsigned su_ = blockIdx.y * gridDim.x + blockIdx.x;                                 \
    if (threadIdx.x == 0 && su_ < kStampUnits)                                                \
      g_stamps[su_ * kStamps + (k)] = DRCVAR_STAMP_CLOCK();                                   \
  } while (0)
#ifdef DRCVAR_STAMPS_REALTIME  // 100 MHz clock shared by every XCD: spreads across workgroups
#define DRCVAR_STAMP_CLOCK() __builtin_amdgcn_s_memrealtime()
#else  // shader clock of the workgroup's XCD: phase lengths in cycles
#define DRCVAR_STAMP_CLOCK() __builtin_amdgcn_s_memtime()
#endif
#else
#define DRCVAR_STAMP(k) \
  do {                  \
  } while (0)
#endif
#if defined(DRCVAR_STAMPS) && defined(DRCVAR_STAMPS_WAVES)
#define DRCVAR_STAMP_WAVE(j)                                                                  \
  do {                                                                                        \
    const unsigned su_ = blockIdx.y * gridDim.x + blockIdx.x;                                 \
    if ((threadIdx.x & 63) == 0 && threadIdx.x < 256 && su_ < kStampUnits)                    \
      g_stamps[su_ * kStamps + 8 + 4 * (j) + (threadIdx.x >> 6)] = DRCVAR_STAMP_CLOCK();      \
  } while (0)
#else
#define DRCVAR_STAMP_WAVE(j) \
  do {                       \
  } while (0)
#endif

// Launch-uniform scalars, precomputed on the host so the per-unit critical path carries as few
// fp64 divisions as possible.
struct Params {
  double rc;              // robot_radius + obstacle_radius
  double alpha;
  double delta;
  double epsilon;
  double eps_over_alpha;  // lambda* epsilon (risk_metrics.py:110,122)
  double inv_n;           // 1 / N
  double inv_n0;          // 1 / size of the window's subsample (pilot: min(N, 64); row 0: min(N, threads))
  double k;               // alpha N
  double inv_k;           // 1 / (alpha N)
  double z_alpha;         // standard-normal alpha-quantile: centre of the fast-path window
  double window_sd;       // half-width of the fast-path window, in sd of d
  double z_lo;            // z_alpha - window_sd: low edge of the window, in sd of d
  double hist_scale;      // bins / (2 window_sd): bins per sd of d (set per launch plan)
  uint32_t rank;          // min(floor(alpha N), N - 1): 0-based rank of tau
  int unbounded;          // alpha N > N: both LPs unbounded (tau -> -inf), solver-failure sentinel
  double degenerate_sq;   // smallest x with sqrt(x) >= 1e-10: |v| < 1e-10  <=>  v.v < degenerate_sq
};

// 1/sqrt(x) to ~1 ulp: hardware seed + one Newton step (the exact sqrt + divide sequence is far
// longer and sits on the critical path of every unit)
__device__ __forceinline__ double rsqrt_nr(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  return y * fma(-0.5 * x * y, y, 1.5);
}

// ---------------------------------------------------------------------------------------------
// wave primitives: DPP row permutations (each an involution, so every lane of a row ends with the
// bitwise-identical value), then the four row results combined through readlane in fixed order
// ---------------------------------------------------------------------------------------------
// (mov_dpp, not update_dpp with an old value of 0: every lane of these permutations has a source,
// so the old value is never used, and materialising it cost two v_mov plus a DPP hazard wait per
// stage of every reduction on the chain)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}
constexpr int kDppQuadXor1 = 0xB1;    // quad_perm [1,0,3,2]
constexpr int kDppQuadXor2 = 0x4E;    // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141; // row_half_mirror
constexpr int kDppMirror = 0x140;     // row_mirror

struct OpAdd {
  __device__ static double f(double a, double b) { return a + b; }
};
struct OpMin {
  __device__ static double f(double a, double b) { return fmin(a, b); }
};
struct OpMax {
  __device__ static double f(double a, double b) { return fmax(a, b); }
};

// gfx950 lane swaps: permlane16_swap exchanges odd rows of its first operand with even rows of
// its second, permlane32_swap the upper half of the first with the lower half of the second.
// With both operands = v, element [0] holds rows (0,0,2,2) / halves (lo,lo) and element [1] rows
// (1,1,3,3) / halves (hi,hi), so Op([0], [1]) combines row pairs / halves in every lane at once.
// a wave-uniform value moved to SGPRs (keeps uniform scalars out of the VGPR budget)
__device__ __forceinline__ double uniform_f64(double v) {
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ float uniform_f32(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

template <class Op>
__device__ __forceinline__ double swap_combine16(double v) {
  const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
  return Op::f(__hiloint2double(hi[0], lo[0]), __hiloint2double(hi[1], lo[1]));
}
template <class Op>
__device__ __forceinline__ double swap_combine32(double v) {
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
  return Op::f(__hiloint2double(hi[0], lo[0]), __hiloint2double(hi[1], lo[1]));
}

// Result is uniform across the wave (bitwise: every lane evaluates the same tree,
// ((r0 + r1) + (r2 + r3)) over the row results).  Requires all 64 lanes active.
// Measured (scripts/micro/reduce.hip): ~190 cycles latency, ~150 cycles per extra independent value.
template <class Op>
__device__ __forceinline__ double wave_reduce(double v) {
  v = Op::f(v, dpp_f64<kDppQuadXor1>(v));
  v = Op::f(v, dpp_f64<kDppQuadXor2>(v));
  v = Op::f(v, dpp_f64<kDppHalfMirror>(v));
  v = Op::f(v, dpp_f64<kDppMirror>(v));
  return uniform_f64(swap_combine32<Op>(swap_combine16<Op>(v)));
}

// fp32 sum over the wave, same tree (the DPP moves fold into v_add_f32_dpp): ~60 cycles per value.
__device__ __forceinline__ float wave_sum_f32(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kDppQuadXor1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kDppQuadXor2, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kDppHalfMirror, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kDppMirror, 0xF, 0xF, false));
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  v = __int_as_float(a[0]) + __int_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return uniform_f32(__int_as_float(b[0]) + __int_as_float(b[1]));
}

// Sum of NW per-wave partials p[0..NW) read by every thread (broadcast LDS reads), fixed
// pairwise tree — cheaper than a second wave reduction for the small NW of the launch plans.
template <int NW, class T>
__device__ __forceinline__ T sum_partials(const T* p) {
  T v[NW];
#pragma unroll
  for (int w = 0; w < NW; ++w) v[w] = p[w];
#pragma unroll
  for (int stride = 1; stride < NW; stride *= 2)
#pragma unroll
    for (int w = 0; w + stride < NW; w += 2 * stride) v[w] = v[w] + v[w + stride];
  if constexpr (sizeof(T) == 8) {
    return uniform_f64(v[0]);
  } else {
    return uniform_f32(v[0]);
  }
}

template <class Op>
__device__ __forceinline__ double identity_of();
template <>
__device__ __forceinline__ double identity_of<OpAdd>() { return 0.0; }
template <>
__device__ __forceinline__ double identity_of<OpMin>() { return INFINITY; }
template <>
__device__ __forceinline__ double identity_of<OpMax>() { return -INFINITY; }

// Workgroup reduction of K values.  `slot` is LDS scratch of K*NW doubles owned by the call site
// (never reused by another call without a barrier in between).  The per-wave partials are
// combined by a second wave reduction (lane w holds wave w's partial), so the order is fixed.
template <class Op, int NW, int K>
__device__ __forceinline__ void block_reduce(double (&v)[K], double* slot) {
#pragma unroll
  for (int q = 0; q < K; ++q) v[q] = wave_reduce<Op>(v[q]);
  if constexpr (NW > 1) {
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x / kWave;
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < K; ++q) slot[q * NW + w] = v[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < K; ++q) {
      const double part = lane < NW ? slot[q * NW + lane] : identity_of<Op>();
      v[q] = wave_reduce<Op>(part);
    }
  }
}

// KD fp64 and KF fp32 wave sums at once: the same trees as wave_reduce / wave_sum_f32 (so the
// results are bitwise those of the one-value forms), written stage by stage across the values so
// that the independent chains fill each other's DPP hazard slots (one value at a time, the
// compiler emitted the seven chains back to back: ~750 cycles on the critical path of barrier 1).
template <int CTRL>
__device__ __forceinline__ double mov_dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ float mov_dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL, int KD, int KF>
__device__ __forceinline__ void sum_stage(double* v, float* f) {
  double td[KD > 0 ? KD : 1];
  float tf[KF > 0 ? KF : 1];
#pragma unroll
  for (int q = 0; q < KD; ++q) td[q] = mov_dpp_f64<CTRL>(v[q]);
#pragma unroll
  for (int q = 0; q < KF; ++q) tf[q] = mov_dpp_f32<CTRL>(f[q]);
#pragma unroll
  for (int q = 0; q < KD; ++q) v[q] = v[q] + td[q];
#pragma unroll
  for (int q = 0; q < KF; ++q) f[q] = f[q] + tf[q];
}
// (v, f: KD doubles and KF floats in registers — either count may be 0)
template <int KD, int KF>
__device__ __forceinline__ void wave_sum_multi(double* v, float* f) {
  sum_stage<kDppQuadXor1, KD, KF>(v, f);
  sum_stage<kDppQuadXor2, KD, KF>(v, f);
  sum_stage<kDppHalfMirror, KD, KF>(v, f);
  sum_stage<kDppMirror, KD, KF>(v, f);
#pragma unroll
  for (int q = 0; q < KD; ++q) v[q] = swap_combine16<OpAdd>(v[q]);
#pragma unroll
  for (int q = 0; q < KF; ++q) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_int(f[q]), __float_as_int(f[q]), false, false);
    f[q] = __int_as_float(a[0]) + __int_as_float(a[1]);
  }
#pragma unroll
  for (int q = 0; q < KD; ++q) v[q] = swap_combine32<OpAdd>(v[q]);
#pragma unroll
  for (int q = 0; q < KF; ++q) {
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_int(f[q]), __float_as_int(f[q]), false, false);
    f[q] = __int_as_float(b[0]) + __int_as_float(b[1]);
  }
#pragma unroll
  for (int q = 0; q < KD; ++q) v[q] = uniform_f64(v[q]);
#pragma unroll
  for (int q = 0; q < KF; ++q) f[q] = uniform_f32(f[q]);
}

// Workgroup sums of the load phase: KD fp64 values (the mean sums) and KF fp32 values (the
// pivot-shifted second moments, which only position the histogram window).  One barrier.
// `pilot` (optional): the 64-sample pilot published before the barrier — this lane's sample is
// read in the same batch of LDS reads as the partials (read at its first use, after the direction,
// it was a second LDS round trip on the chain to the window pass).
template <int NW, int KD, int KF, bool PILOT = false>
__device__ __forceinline__ void block_sum_moments(double* v, float* f, double* slot_d, float* slot_f,
                                                  const double2* pilot = nullptr,
                                                  double2* pilot_v = nullptr) {
  wave_sum_multi<KD, KF>(v, f);
  DRCVAR_STAMP_WAVE(1);  // diagnostic build: this wave's reduction done, before the barrier
  const int lane = threadIdx.x & (kWave - 1);
  if constexpr (NW > 1) {
    const int w = threadIdx.x / kWave;
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < KD; ++q) slot_d[q * NW + w] = v[q];
#pragma unroll
      for (int q = 0; q < KF; ++q) slot_f[q * NW + w] = f[q];
    }
    __syncthreads();
    if constexpr (PILOT) *pilot_v = pilot[lane];
#pragma unroll
    for (int q = 0; q < KD; ++q) v[q] = sum_partials<NW>(slot_d + q * NW);
#pragma unroll
    for (int q = 0; q < KF; ++q) f[q] = sum_partials<NW>(slot_f + q * NW);
  } else {
    if constexpr (PILOT) *pilot_v = pilot[lane];  // (one wave: each lane reads back its own store)
  }
  if constexpr (PILOT) asm volatile("" ::"v"(pilot_v->x), "v"(pilot_v->y));
}

// order-preserving map double -> uint64 (total order on non-NaN values)
__device__ __forceinline__ uint64_t f64_key(double d) {
  const uint64_t u = static_cast<uint64_t>(__double_as_longlong(d));
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

// Monotone (non-decreasing) map of the candidate interval [lo, hi] onto NB histogram bins.
template <int LOG_NB>
struct BucketMap {
  static constexpr int NB = 1 << LOG_NB;
  bool value_mode;
  double lo, scale;
  uint64_t klo;
  int shift;

  // exact range [lo_, hi_] of the candidates, lo_ < hi_: bucket(lo_) = 0 < bucket(hi_)
  __device__ __forceinline__ void init_range(double lo_, double hi_, int iter) {
    lo = lo_;
    const double range = hi_ - lo_;
    scale = static_cast<double>(NB) / range;
    value_mode = iter < kMaxValueIters && range > 0.0 && scale < 1e300 && range * scale >= 1.0;
    klo = f64_key(lo_);
    const uint64_t diff = f64_key(hi_) - klo;  // >= 1 when hi > lo
    const int bits = 64 - __builtin_clzll(diff | 1ull);
    shift = bits > LOG_NB ? bits - LOG_NB : 0;
  }
  __device__ __forceinline__ int operator()(double d) const {
    if (value_mode) {
      const double t = fmin(fmax((d - lo) * scale, 0.0), static_cast<double>(NB - 1));
      return static_cast<int>(t);
    }
    return static_cast<int>((f64_key(d) - klo) >> shift);  // key mode: lo <= d <= hi only
  }
};

struct ScanResult {
  int bin;
  uint32_t below, cnt;
  bool found;  // false when the histogram holds fewer than rr + 1 samples
};

// Histogram storage: lane l of a scanning wave owns bins [l*B, (l+1)*B), B = NB/64.  One padding
// word after every B bins makes the owner reads conflict-free (lane stride B+1 words, B+1 odd).
template <int NB>
__device__ __forceinline__ int hist_slot(int bin) {  // bin >= 0
  constexpr unsigned B = NB / kWave;
  const unsigned b = static_cast<unsigned>(bin);
  return static_cast<int>(b + b / B);
}
template <int NB>
constexpr int hist_words() {
  return NB + kWave;
}

// Inclusive prefix sum over the 64 lanes: DPP row shifts within each row of 16, then the row
// totals (lanes 15, 31, 47) added through readlane — no LDS round trips.
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x, int lane) {
  constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;
  int v = static_cast<int>(x);
  v += __builtin_amdgcn_update_dpp(0, v, kRowShr1, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0, v, kRowShr2, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0, v, kRowShr4, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0, v, kRowShr8, 0xF, 0xF, true);
  const int r0 = __builtin_amdgcn_readlane(v, 15);
  const int r1 = __builtin_amdgcn_readlane(v, 31);
  const int r2 = __builtin_amdgcn_readlane(v, 47);
  const int row = lane >> 4;
  v += (row >= 1 ? r0 : 0) + (row >= 2 ? r1 : 0) + (row >= 3 ? r2 : 0);
  return static_cast<uint32_t>(v);
}

// Any wave: the bin holding the sample of rank rr (0-based) and the counts below / inside it.
// Result is uniform across the wave.
template <int NB>
__device__ __forceinline__ void load_bins(const uint32_t* hist, int lane, uint32_t (&h)[NB / kWave]) {
  constexpr int B = NB / kWave;
  const uint32_t* mine = hist + lane * (B + 1);
#pragma unroll
  for (int q = 0; q < B; ++q) h[q] = mine[q];
}

// Same, with this lane's bins already loaded (load_bins) — lets the caller issue the histogram
// reads together with its other post-barrier LDS reads.
template <int NB>
__device__ __forceinline__ ScanResult scan_loaded_bins(const uint32_t (&h)[NB / kWave], uint32_t rr,
                                                      int lane) {
  constexpr int B = NB / kWave;  // contiguous bins per lane
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < B; ++q) s += h[q];
  const uint32_t incl = wave_inclusive_scan(s, lane);
  const unsigned long long hit = __ballot(incl > rr);
  if (hit == 0ull) return ScanResult{0, 0u, 0u, false};
  const int owner = __ffsll(static_cast<long long>(hit)) - 1;  // uniform
  // in the owner lane: first bin whose running count passes rr (branch-free over the B bins)
  uint32_t cum = incl - s;
  int bin = lane * B + B - 1;
  uint32_t below = 0, cnt = 0;
  bool done = false;
#pragma unroll
  for (int q = 0; q < B; ++q) {
    const bool take = !done && cum + h[q] > rr;
    bin = take ? lane * B + q : bin;
    below = take ? cum : below;
    cnt = take ? h[q] : cnt;
    done = done || take;
    cum += h[q];
  }
  return ScanResult{__builtin_amdgcn_readlane(bin, owner),
                    static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(below), owner)),
                    static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(cnt), owner)),
                    true};
}

template <int NB>
__device__ __forceinline__ ScanResult scan_bins(const uint32_t* hist, uint32_t rr, int lane) {
  uint32_t h[NB / kWave];
  load_bins<NB>(hist, lane, h);
  return scan_loaded_bins<NB>(h, rr, lane);
}

__device__ __forceinline__ bool in_range(double d, double lo, double hi) {
  return lo <= d && d <= hi;  // false for the NaN padding of idle slots
}

// MeanSafeHalfspace (core/halfspaces.py:84-94): direction from the ORIGIN, offset
// -(h.mu - R_c |h|), with compute_separating_vector's [1, 0] fallback
__device__ __forceinline__ void mean_halfspace(double mux, double muy, double rc, double* m0,
                                               double* m1, double* g) {
  const double nm = sqrt(mux * mux + muy * muy);
  const bool degenerate = nm < 1e-10;
  *m0 = degenerate ? 1.0 : mux / nm;
  *m1 = degenerate ? 0.0 : muy / nm;
  *g = -((*m0 * mux + *m1 * muy) - rc * sqrt(*m0 * *m0 + *m1 * *m1));
}

// columns 0..2 of the record (the mean halfspace), by one lane
__device__ __forceinline__ void write_mean_halfspace(double* rec, double mux, double muy,
                                                     double rc, int lane) {
  double m0, m1, g_mean;
  mean_halfspace(mux, muy, rc, &m0, &m1, &g_mean);
  if (lane == 0) {
    reinterpret_cast<double2*>(rec)[0] = make_double2(m0, m1);
    rec[DRCVAR_COL_G_MEAN] = g_mean;
  }
}

__device__ __forceinline__ void store_record(double* rec, double m0, double m1, double gm,
                                             double h0, double h1, double gc, double gs,
                                             double gt) {
  reinterpret_cast<double2*>(rec)[0] = make_double2(m0, m1);
  reinterpret_cast<double2*>(rec)[1] = make_double2(gm, h0);
  reinterpret_cast<double2*>(rec)[2] = make_double2(h1, gc);
  reinterpret_cast<double2*>(rec)[3] = make_double2(gs, gt);
}

// The peer-push exchange (drcvar_safe_halfspaces_f64_peer, include/drcvar_exchange.h): every
// rank's launch writes each record straight into the exchange region of every rank of the node
// (its own and, over xGMI, the peers' — regions mapped into this process by IPC), at the record's
// global row, in the buffer of this step's parity; drcvar_peer_signal_wait then publishes and
// awaits the generation.  The regions are uncached device memory, and the stores are system-scope
// (write-through) so that no L2 holds a record a peer's later read could miss.
struct PeerArgs {
  double* region[DRCVAR_MAX_PEERS];    // rank j's region (parity 0 rows, parity 1 rows, flags)
  int64_t rows;                        // records per parity buffer (n_ranks * per)
  int64_t row_base;                    // global row of this launch's unit 0
  const unsigned long long* gen;       // this rank's completed-step counter (device)
  int32_t n_ranks;
};

__device__ __forceinline__ void store_sys(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One record to every rank's region: lane j < n_ranks writes rank j's copy (values uniform across
// the wave).  Parity = (completed steps + 1) & 1: the buffer this step fills.
__device__ __forceinline__ void peer_store_record(const PeerArgs& pa, unsigned long long gen,
                                                  int64_t u, int lane, double m0, double m1,
                                                  double gm, double h0, double h1, double gc,
                                                  double gs, double gt) {
  if (lane < pa.n_ranks) {
    const int64_t parity = static_cast<int64_t>((gen + 1ull) & 1ull);
    double* r = pa.region[lane] + (parity * pa.rows + pa.row_base + u) * DRCVAR_OUT_WIDTH;
    store_sys(r + 0, m0);
    store_sys(r + 1, m1);
    store_sys(r + 2, gm);
    store_sys(r + 3, h0);
    store_sys(r + 4, h1);
    store_sys(r + 5, gc);
    store_sys(r + 6, gs);
    store_sys(r + 7, gt);
  }
  // every record store acknowledged (system scope: performed in the destination's memory) before
  // the wave ends, so the publish launch behind this one finds them all in place
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// d_i = h . xi_i — one expression, used both for the register-resident samples and for re-reads,
// so both paths see bitwise-identical values (core/risk_metrics.py:145,233: h @ samples.T)
__device__ __forceinline__ double project(double h0, double h1, double x, double y) {
  return fma(h0, x, h1 * y);
}

template <bool VEC>
__device__ __forceinline__ double project_at(const double* base, int i, int64_t s_samp, double h0,
                                             double h1) {
  const int64_t off = static_cast<int64_t>(i) * s_samp;
  if constexpr (VEC) {
    const double2 v = *reinterpret_cast<const double2*>(base + off);
    return project(h0, h1, v.x, v.y);
  } else {
    return project(h0, h1, base[off], base[off + 1]);
  }
}

// Value-linear position in the fast-path window: t(d) = d * scale + off (one fma, rounded once,
// so monotone non-decreasing in d for any scale > 0).  Below the window: t < 0; inside: 0 <= t <
// NB (bin = trunc(t) <= NB - 1); above it (and the +inf padding): t >= NB.
struct LinearMap {
  double scale, off;
  __device__ __forceinline__ double operator()(double d) const { return fma(d, scale, off); }
};

// LDS accesses of one wave complete in order; this keeps the compiler from moving them across a
// wave-local hand-off (no barrier needed within a wave)
__device__ __forceinline__ void wave_lds_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// Per-wave ordered compaction step: append the candidates of one row to this wave's LDS region.
__device__ __forceinline__ void append_candidate(double* region, uint32_t& wbase, bool is_cand,
                                                 double v, unsigned long long lt_mask) {
  const unsigned long long ballot = __ballot(is_cand);
  if (is_cand) region[wbase + __popcll(ballot & lt_mask)] = v;
  wbase += static_cast<uint32_t>(__popcll(ballot));
}

// Lane w < NW: the candidate count of wave w (0 elsewhere) — the ranking's input, read by the
// caller so that it can be issued together with other LDS reads.
template <int NW>
__device__ __forceinline__ uint32_t wave_counts(const uint32_t* wcount, int lane) {
  return lane < NW ? wcount[lane] : 0u;
}
// Makes a loaded value available at this point (an empty asm that consumes it): keeps the compiler
// from sinking independent LDS loads past a branch or a wait, so they share one round trip.
__device__ __forceinline__ void lds_values_ready(uint32_t v) { asm volatile("" ::"v"(v)); }

// Wave 0 (all lanes active): tau = the candidate of rank rr among the c <= kCap candidates held in
// per-wave regions cand[w * kCap + i], i < wcount[w] (global order: wave, then position — fixed).
// Candidates are pulled into registers (g = lane, lane + 64) and compared through readlane, so
// the O(c^2) ranking never waits on LDS.  Also returns s_cand = sum over candidates below tau of
// (cand - tau), accumulated in candidate order.  Q = candidate registers per lane: 1 when
// c <= 64 (the usual case), 2 up to kCap.
template <int NW, int Q>
__device__ __forceinline__ double rank_candidates_q(const double* cand, uint32_t cw, uint32_t c,
                                                    uint32_t rr, int lane, double* s_cand) {
  int slot[2] = {-1, -1};
  uint32_t acc = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const uint32_t nw = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(cw), w));
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const uint32_t g = lane + q * kWave;
      if (g >= acc && g < acc + nw) slot[q] = w * kCap + static_cast<int>(g - acc);
    }
    acc += nw;
  }
  double mine[2] = {NAN, NAN};  // candidates g = lane, lane + 64
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (slot[q] >= 0) mine[q] = cand[slot[q]];
  // per candidate v (lane-parallel): #{z < v}, #{z == v} and sum_{z < v} (z - v); the lane of
  // tau then holds s_cand itself, so no reduction follows the ranking
  uint32_t less[2] = {0u, 0u}, eq[2] = {0u, 0u};
  double sl[2] = {0.0, 0.0};
  const uint32_t c0 = c < kWave ? c : kWave;
  for (uint32_t i = 0; i < c0; ++i) {  // uniform trip count
    const double z = readlane_f64(mine[0], static_cast<int>(i));
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const bool lt = z < mine[q];
      less[q] += lt ? 1u : 0u;
      eq[q] += (z == mine[q]) ? 1u : 0u;
      sl[q] += lt ? z - mine[q] : 0.0;
    }
  }
  for (uint32_t i = kWave; Q == 2 && i < c; ++i) {
    const double z = readlane_f64(mine[1], static_cast<int>(i - kWave));
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const bool lt = z < mine[q];
      less[q] += lt ? 1u : 0u;
      eq[q] += (z == mine[q]) ? 1u : 0u;
      sl[q] += lt ? z - mine[q] : 0.0;
    }
  }
  bool found = false;
  double found_v = 0.0, found_s = 0.0;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    if (lane + q * kWave < c && less[q] <= rr && rr < less[q] + eq[q]) {
      found = true;
      found_v = mine[q];
      found_s = sl[q];
    }
  }
  const unsigned long long fb = __ballot(found);
  const int src = __ffsll(static_cast<long long>(fb)) - 1;
  *s_cand = readlane_f64(found_s, src);
  return readlane_f64(found_v, src);
}
template <int NW>
__device__ __forceinline__ double rank_candidates(const double* cand, uint32_t cw, uint32_t c,
                                                  uint32_t rr, int lane, double* s_cand) {
  return c <= static_cast<uint32_t>(kWave) ? rank_candidates_q<NW, 1>(cand, cw, c, rr, lane, s_cand)
                                           : rank_candidates_q<NW, 2>(cand, cw, c, rr, lane, s_cand);
}

// Exact selection for the units the register fast path does not finish (degenerate moments, or a
// first-pass bucket with more than kCap samples).  It re-reads the unit's samples (L2/MALL-hot)
// instead of keeping register state live: exact min/max, then histogram refinement (value-linear,
// then order-preserving integer keys) until <= kCap candidates remain or the run collapses to one
// value.  Result (valid in wave 0): tau and dsum = sum_{d<tau} (d - tau).
// proj(i): the projection h . xi_i of sample i (re-read from memory).
template <int BLOCK, int LOG_NB, class Proj>
__device__ __forceinline__ void select_from_memory(const Proj& proj, int n, double mu_d,
                                                uint32_t rank, uint32_t* hist, double* cand,
                                                uint32_t* wcount, double* red_rng,
                                                double* red_tail, double* tau_out,
                                                double* dsum_out) {
  constexpr int NW = BLOCK / kWave;
  constexpr int NB = 1 << LOG_NB;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = tid / kWave;
  __syncthreads();  // the fast path's readers of hist / red_* are done

  double vmin[1] = {INFINITY}, vmax[1] = {-INFINITY};
  for (int i = tid; i < n; i += BLOCK) {
    const double v = proj(i);
    vmin[0] = fmin(vmin[0], v);
    vmax[0] = fmax(vmax[0], v);
  }
  block_reduce<OpMin, NW, 1>(vmin, red_rng);
  block_reduce<OpMax, NW, 1>(vmax, red_rng + NW);
  double lo = vmin[0], hi = vmax[0];
  if (lo == hi) {  // every sample projects to one value (the noise-free step 0): no tail below it
    *tau_out = lo;
    *dsum_out = 0.0;
    return;        // uniform; no second pass over the samples
  }
  uint32_t rr = rank, c = static_cast<uint32_t>(n);
  bool have_bin = false, tau_known = false;
  double tau = lo;
  int bin = 0;
  BucketMap<LOG_NB> map;
  for (int iter = 0; !tau_known; ++iter) {
    map.init_range(lo, hi, iter);
    for (int b = tid; b < hist_words<NB>(); b += BLOCK) hist[b] = 0u;
    __syncthreads();
    for (int i = tid; i < n; i += BLOCK) {
      const double v = proj(i);
      if (in_range(v, lo, hi)) atomicAdd(&hist[hist_slot<NB>(map(v))], 1u);
    }
    __syncthreads();
    const ScanResult sr = scan_bins<NB>(hist, rr, lane);
    bin = sr.bin;
    rr -= sr.below;
    c = sr.cnt;
    have_bin = true;
    if (c <= kCap) break;
    double rmin[1] = {INFINITY}, rmax[1] = {-INFINITY};
    for (int i = tid; i < n; i += BLOCK) {
      const double v = proj(i);
      if (in_range(v, lo, hi) && map(v) == bin) {
        rmin[0] = fmin(rmin[0], v);
        rmax[0] = fmax(rmax[0], v);
      }
    }
    __syncthreads();  // all waves have scanned hist before it is cleared again
    block_reduce<OpMin, NW, 1>(rmin, red_rng);
    block_reduce<OpMax, NW, 1>(rmax, red_rng + NW);
    lo = rmin[0];
    hi = rmax[0];
    have_bin = false;
    if (lo == hi) {
      tau_known = true;
      tau = lo;
    }
  }

  double sq = 0.0;
  uint32_t wbase = 0;
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  for (int i0 = 0; i0 < n; i0 += BLOCK) {  // uniform trip count: ballots see whole waves
    const int i = i0 + tid;
    const double v = i < n ? proj(i) : NAN;
    const bool inr = in_range(v, lo, hi);
    const int bj = (have_bin && inr) ? map(v) : 0;
    const bool below = v < lo || (have_bin && inr && bj < bin);
    if (below) sq += v - mu_d;
    append_candidate(cand + wave * kCap, wbase, !tau_known && inr && (!have_bin || bj == bin), v,
                     lt_mask);
  }
  sq = wave_reduce<OpAdd>(sq);
  if (lane == 0) {
    red_tail[wave] = sq;
    wcount[wave] = wbase;
  }
  __syncthreads();
  if (wave != 0) return;
  const double s_below = sum_partials<NW>(red_tail);
  double s_cand = 0.0;
  if (!tau_known) tau = rank_candidates<NW>(cand, wave_counts<NW>(wcount, lane), c, rr, lane, &s_cand);
  const double n_below = static_cast<double>(rank - rr);
  *tau_out = tau;
  *dsum_out = (s_below - n_below * (tau - mu_d)) + s_cand;
}

// compute_separating_vector(ego, mu) (core/geometry.py:35-53): (mu - ego) / |mu - ego|, [1, 0]
// below 1e-10 (rsqrt + one Newton step).  Branch-free: an overflowing norm (n2 = inf) selects
// 1/inf = 0, as diff / norm gives 0 (finite diff) or NaN (infinite diff); a NaN n2 stays NaN.
__device__ __forceinline__ void separating_direction(double mux, double muy, double e0, double e1,
                                                     double deg_sq, double* h0, double* h1) {
  const double dx = mux - e0, dy = muy - e1;
  const double n2 = dx * dx + dy * dy;
  const double inv = n2 == INFINITY ? 0.0 : rsqrt_nr(n2);
  const bool degenerate = n2 < deg_sq;
  *h0 = degenerate ? 1.0 : dx * inv;
  *h1 = degenerate ? 0.0 : dy * inv;
}

// |h| for R_c |h| (risk_metrics.py:293, :234).  h is a unit vector up to rounding on the
// separating-direction path, where sqrt(1 + e) = 1 + e/2 - e^2/8 (+ O(e^3)) replaces the long
// fp64 sqrt sequence (e = |h|^2 - 1 is exact there; the result is within 1 ulp of the correctly
// rounded sqrt — it can differ only where 1 + e/2 is a rounding tie); any other h takes sqrt.
__device__ __forceinline__ double norm_h(double h0, double h1) {
  const double n2 = h0 * h0 + h1 * h1;
  const double e = n2 - 1.0;
  if (fabs(e) < 0x1p-40) return 1.0 + fma(-0.125 * e, e, 0.5 * e);  // uniform branch
  return sqrt(n2);
}

// Per-unit status word (DRCVAR_UNIT_*): which of the reference's solver-failure branches the unit
// took (core/risk_metrics.py:173-177,261-265: the LP status; :298-303,334-338: the sentinels) —
// reported by the kernel itself, so no caller has to infer it from the sentinel's value.
__device__ __forceinline__ int32_t failure_status(bool nonfinite, const Params& prm) {
  return (nonfinite ? DRCVAR_UNIT_NONFINITE : 0) | (prm.unbounded ? DRCVAR_UNIT_UNBOUNDED : 0) |
         (prm.epsilon < 0.0 ? DRCVAR_UNIT_DR_UNBOUNDED : 0);
}

// Offsets from the lower-tail statistics (wave 0, lane 0 writes).  L = tau + dsum / k.
// (The peer form below computes the same values in every lane of wave 0, from lane 0's tau and
// dsum, and writes the whole record — the mean halfspace too — to every rank.)
// r = R_c |h| (risk_metrics.py:293, :234), computed by the caller as soon as h is known.
template <int NW>
__device__ __forceinline__ void finish_offsets(double* rec, const Params& prm, double r, double h0,
                                               double h1, double tau, double dsum, double mux,
                                               double muy, int lane) {
  if (lane == 0) {
    const double L = tau + dsum * prm.inv_k;  // lower-tail mean
    const double g_cvar = r - prm.delta - L;
    double g_star = kSentinel, g_tilde = kSentinel - r;
    if (prm.epsilon >= 0.0) {  // else: DR LP unbounded (lambda -> inf), solver-failure sentinel
      g_star = r - prm.delta + prm.eps_over_alpha - L;
      g_tilde = g_star - r;
    }
    if constexpr (NW == 1) {
      double m0, m1, g_mean;
      mean_halfspace(mux, muy, prm.rc, &m0, &m1, &g_mean);
      store_record(rec, m0, m1, g_mean, h0, h1, g_cvar, g_star, g_tilde);
    } else {  // columns 0..2 are written by wave 1
      reinterpret_cast<double*>(rec)[DRCVAR_COL_H0] = h0;
      reinterpret_cast<double2*>(rec)[2] = make_double2(h1, g_cvar);
      reinterpret_cast<double2*>(rec)[3] = make_double2(g_star, g_tilde);
    }
  }
}

__device__ __forceinline__ void finish_offsets_peer(const PeerArgs& pa, unsigned long long gen,
                                                    int64_t u, const Params& prm, double r,
                                                    double h0, double h1, double tau, double dsum,
                                                    double mux, double muy, int lane) {
  tau = readlane_f64(tau, 0);
  dsum = readlane_f64(dsum, 0);
  const double L = tau + dsum * prm.inv_k;
  const double g_cvar = r - prm.delta - L;
  double g_star = kSentinel, g_tilde = kSentinel - r;
  if (prm.epsilon >= 0.0) {
    g_star = r - prm.delta + prm.eps_over_alpha - L;
    g_tilde = g_star - r;
  }
  double m0, m1, g_mean;
  mean_halfspace(mux, muy, prm.rc, &m0, &m1, &g_mean);
  peer_store_record(pa, gen, u, lane, m0, m1, g_mean, h0, h1, g_cvar, g_star, g_tilde);
}


// ---------------------------------------------------------------------------------------------
// the fused kernel
//   BLOCK    threads per unit (one workgroup per unit)
//   P        samples held per thread (N <= BLOCK * P)
//   LOG_NB   log2 of histogram bins
//   LOAD     kLoadPair: two 8-B loads per sample; kLoadVec: every (x, y) pair is 16-B aligned ->
//            one 16-B load per sample; kLoadNt: the same, nontemporal (launches larger than the
//            256 MB Infinity Cache, whose samples are streamed exactly once)
//   GIVEN_H  `dir` holds h per unit (cvar_halfspace / dr_cvar_halfspace) instead of ego per step
// ---------------------------------------------------------------------------------------------
//   PEER     the peer-push exchange form: records go to every rank's exchange region (PeerArgs)
//            instead of `out`
template <int BLOCK, int P, int LOG_NB, int LOAD, bool GIVEN_H, bool PEER>
__global__ void __launch_bounds__(BLOCK)
safe_halfspace_kernel(const double* __restrict__ samples, int64_t n_steps, int n,
                      int64_t s_obs, int64_t s_step, int64_t s_samp,
                      const double* __restrict__ dir, int64_t dir_s_obs, int64_t dir_s_step,
                      Params prm, double* __restrict__ out, int32_t* __restrict__ status,
                      PeerArgs peer) {
  constexpr int NW = BLOCK / kWave;
  constexpr int NB = 1 << LOG_NB;
  __shared__ uint32_t hist[hist_words<NB>()];
  __shared__ double cand[NW * kCap];
  __shared__ double lane_tail[P <= 8 ? BLOCK : 1];
  __shared__ uint32_t wcount[NW];
  __shared__ uint32_t wbelow_sh[NW];
  // Small plans (the latency-bound ones) place the histogram window from a 64-sample pilot after
  // barrier 1 — the variance of the projections themselves, one two-value wave reduction —
  // instead of reducing five row-0 second moments across the workgroup before it: per-wave stamps
  // (-DDRCVAR_STAMPS_WAVES) showed the seven-value reduction at ~1 000 cycles of one wave's issue
  // on the chain to barrier 1.  Large plans (bandwidth-bound) keep the row-0 moments, whose larger
  // subsample gives their narrower windows (0.25 sd at N = 10 000) more margin.
  constexpr bool kPilot = P <= 8;
  __shared__ double2 pilot[kPilot ? kWave : 1];
  __shared__ double red_mom[2 * NW];
  __shared__ float red_mom0[5 * NW];
  __shared__ double red_rng[2 * NW];
  __shared__ double red_tail[NW];

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = tid / kWave;
  // grid (n_steps, n_obstacles): no integer division ahead of the sample loads (the host splits
  // launches of more than 65535 obstacles)
  const int64_t o = blockIdx.y, t = blockIdx.x;
  const int64_t u = o * n_steps + t;
  const double* base = samples + o * s_obs + t * s_step;
  double* rec = out + u * DRCVAR_OUT_WIDTH;

  DRCVAR_STAMP(0);

  // ---- 1. load + moments ----------------------------------------------------------------
  // Branch-free: idle slots of the last row re-load sample n-1 and contribute zeros.  Offsets:
  // one 64-bit product for the thread's first sample, then a uniform step per row (the clamp is a
  // select, not a product per sample: the per-sample quarter-rate multiplies sat before the
  // loads were issued).
  double x[P], y[P];
  const int64_t off0 = static_cast<int64_t>(tid) * s_samp;
  const int64_t row_step = static_cast<int64_t>(BLOCK) * s_samp;
  const int64_t off_last = static_cast<int64_t>(n - 1) * s_samp;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int i = tid + j * BLOCK;
    const int64_t off = i < n ? off0 + j * row_step : off_last;
    if constexpr (LOAD == kLoadNt) {  // streamed once: keep it out of L2 / MALL
      const dbl2 v = __builtin_nontemporal_load(reinterpret_cast<const dbl2*>(base + off));
      x[j] = v.x;
      y[j] = v.y;
    } else if constexpr (LOAD == kLoadVec) {
      const double2 v = *reinterpret_cast<const double2*>(base + off);
      x[j] = v.x;
      y[j] = v.y;
    } else {
      x[j] = base[off];
      y[j] = base[off + 1];
    }
  }
  // The unit's direction input and the early scalars are fetched while the 16-B sample loads
  // are in flight (otherwise the compiler sinks these scalar loads to their first use, after
  // barrier 1, and their latency lands on the critical path).
  // The pivot of the row-0 moments (the unit's first sample, a uniform scalar load) is issued in
  // the same batch: loaded after the wait for the direction input, it put a second scalar-memory
  // round trip in series on the way to the first moment sums.
  const double* dp = dir + o * dir_s_obs + t * dir_s_step;
  const double e0 = dp[0], e1 = dp[1];
  double px = 0.0, py = 0.0;  // row-0 moments' pivot: the unit's first sample
  if constexpr (!kPilot) {
    px = base[0];
    py = base[1];
  }
  const double inv_n = prm.inv_n, inv_n0 = prm.inv_n0, deg_sq = prm.degenerate_sq;
  const double z_lo = prm.z_lo, hist_scale = prm.hist_scale;
  // inv_k too: first used by the offsets, it was fetched only after the histogram scan, and the
  // candidate pass waited for that scalar load (its lgkm wait also covers the kernarg fetch)
  const double inv_k = prm.inv_k;
  asm volatile("" ::"s"(e0), "s"(e1), "s"(px), "s"(py), "s"(inv_n), "s"(inv_n0), "s"(deg_sq),
               "s"(z_lo), "s"(hist_scale), "s"(inv_k), "s"(status));
  unsigned long long gen = 0;  // the peer form's completed-step counter (parity of the buffer)
  if constexpr (PEER) gen = *peer.gen;
  // the histogram is cleared while the sample loads are in flight (barrier 1 orders it before
  // the first atomic)
#pragma unroll
  for (int b = tid; b < hist_words<NB>(); b += BLOCK) hist[b] = 0u;
  // Sums for the mean over every sample (plain sums, as np.mean, in fp64); second moments over
  // row 0 only (the first BLOCK samples), shifted by the unit's first sample and summed in fp32 —
  // they merely position the fast-path window, so a subsample at low precision is enough: an
  // inaccurate window can only cost speed (the exact fallback), never exactness.
  double mom[2] = {0.0, 0.0};               // Sx Sy
  float mom0[5] = {0.f, 0.f, 0.f, 0.f, 0.f};  // row 0, pivot-shifted: Sa Sb Saa Sbb Sab
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const bool valid = tid + j * BLOCK < n;
    const double a = valid ? x[j] : 0.0, b = valid ? y[j] : 0.0;
    mom[0] += a;
    mom[1] += b;
    if (!kPilot && j == 0) {
      const float fa = valid ? static_cast<float>(x[0] - px) : 0.f;
      const float fb = valid ? static_cast<float>(y[0] - py) : 0.f;
      mom0[0] = fa;
      mom0[1] = fb;
      mom0[2] = fa * fa;
      mom0[3] = fb * fb;
      mom0[4] = fa * fb;
    }
  }
  if (kPilot && wave == 0) pilot[lane] = make_double2(x[0], y[0]);  // samples 0..63 (lane < n)
  DRCVAR_STAMP(1);
  DRCVAR_STAMP_WAVE(0);  // diagnostic build: this wave's samples summed (its loads done)
  double2 pv = make_double2(0.0, 0.0);  // this lane's pilot sample (small plans)
  if constexpr (kPilot)
    block_sum_moments<NW, 2, 0, true>(mom, mom0, red_mom, red_mom0, pilot, &pv);  // [barrier 1]
  else
    block_sum_moments<NW, 2, 5>(mom, mom0, red_mom, red_mom0);           // [barrier 1]
  DRCVAR_STAMP(2);
  const double mux = mom[0] * inv_n, muy = mom[1] * inv_n;
  // any non-finite sample makes a sum non-finite (so do sums that overflow): solver failure
  const bool bad = !(std::isfinite(mom[0]) && std::isfinite(mom[1]));

  // ---- 2. direction ----------------------------------------------------------------------
  double h0, h1;
  if constexpr (GIVEN_H) {
    h0 = e0;
    h1 = e1;
  } else {
    separating_direction(mux, muy, e0, e1, deg_sq, &h0, &h1);
  }
  if (bad || prm.unbounded) {  // solver failure, risk_metrics.py:298-303,334-338
    if constexpr (PEER) {
      if (wave == 0) {
        const double r = prm.rc * norm_h(h0, h1);  // R_c |h|
        double m0, m1, g_mean;
        mean_halfspace(mux, muy, prm.rc, &m0, &m1, &g_mean);
        peer_store_record(peer, gen, u, lane, m0, m1, g_mean, h0, h1, kSentinel, kSentinel,
                          kSentinel - r);
        if (status && lane == 0) status[u] = failure_status(bad, prm);
      }
      return;
    }
    if (tid == 0) {
      const double r = prm.rc * norm_h(h0, h1);  // R_c |h|
      double m0, m1, g_mean;
      mean_halfspace(mux, muy, prm.rc, &m0, &m1, &g_mean);
      store_record(rec, m0, m1, g_mean, h0, h1, kSentinel, kSentinel, kSentinel - r);
      if (status) status[u] = failure_status(bad, prm);
    }
    return;  // uniform across the workgroup
  }

  // ---- 3. projections; window histogram around the estimated quantile ------------------------
  double d[P];
#pragma unroll
  for (int j = 0; j < P; ++j)  // +inf padding: never below, inside or a candidate
    d[j] = (tid + j * BLOCK < n) ? project(h0, h1, x[j], y[j]) : INFINITY;
  const double mu_d = h0 * mux + h1 * muy;
  double var_d;
  if constexpr (kPilot) {  // variance of the pilot's projections about the exact mean, in fp32
    float fm[2];
    fm[0] = lane < n ? static_cast<float>(project(h0, h1, pv.x, pv.y) - mu_d) : 0.f;
    fm[1] = fm[0] * fm[0];
    wave_sum_multi<0, 2>(nullptr, fm);
    const double m1 = fm[0] * inv_n0;
    var_d = fm[1] * inv_n0 - m1 * m1;
  } else {
    const double ma0 = mom0[0] * inv_n0, mb0 = mom0[1] * inv_n0;  // row-0 covariance
    const double cxx = mom0[2] * inv_n0 - ma0 * ma0, cyy = mom0[3] * inv_n0 - mb0 * mb0;
    const double cxy = mom0[4] * inv_n0 - ma0 * mb0;
    var_d = h0 * h0 * cxx + 2.0 * h0 * h1 * cxy + h1 * h1 * cyy;
  }
  // window [wlo, wlo + 2 window_sd sd_d), wlo = mean_d + (z_alpha - window_sd) sd_d; only
  // samples inside it are histogrammed (LDS atomics), samples below it are counted with ballots.
  // Any positive scale keeps the map monotone, so the approximate reciprocal sqrt is exact enough.
  const double inv_sd = rsqrt_nr(var_d);
  const double sd_d = var_d * inv_sd;
  const double wlo = fma(z_lo, sd_d, mu_d);
  const double scale = prm.hist_scale * inv_sd;
  const LinearMap map{scale, -wlo * scale};
  const uint32_t rank = prm.rank;
  bool fast = var_d > 0.0 && std::isfinite(map.scale) && std::isfinite(map.off) && map.scale > 0.0;
  constexpr double kNB = static_cast<double>(NB);
  uint32_t rr = rank, c = 0;
  int bin = 0;
  // per-sample bucket codes, two 16-bit codes per register: the bin inside the window, 0xFFFF
  // outside it (the sum of samples below the window is taken in this pass)
  constexpr int PC = (P + 1) / 2;
  uint32_t code[PC];
  double sq = 0.0;  // sum over samples below the target bucket of (d - mu_d)
  if (fast) {
    uint32_t wbelow = 0;  // samples of this wave below the window (wave-uniform)
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const double v = d[j];
      const double tv = map(v);
      const bool low = tv < 0.0;
      wbelow += static_cast<uint32_t>(__popcll(__ballot(low)));
      sq += low ? v - mu_d : 0.0;
      const bool inw = !low && tv < kNB;
      const int b = inw ? static_cast<int>(tv) : 0;  // 0 <= b <= NB - 1 inside the window
      if (inw) atomicAdd(&hist[hist_slot<NB>(b)], 1u);
      const uint32_t cj = inw ? static_cast<uint32_t>(b) : 0xFFFFu;
      if (j % 2 == 0) code[j / 2] = cj;
      else code[j / 2] |= cj << 16;
    }
    if (lane == 0) wbelow_sh[wave] = wbelow;
    DRCVAR_STAMP(3);
    __syncthreads();                                                      // [barrier 2]
    uint32_t hb[NB / kWave];  // this lane's bins, read together with the per-wave counts
    load_bins<NB>(hist, lane, hb);
    uint32_t below = 0;  // all samples below the window
#pragma unroll
    for (int w = 0; w < NW; ++w) below += wbelow_sh[w];
    // the bins are wanted only when the target lies in the window (a branch on `below`): without
    // this the compiler issued their loads inside the branch, a second LDS round trip after the
    // wait for the counts
#pragma unroll
    for (int b = 0; b < NB / kWave; ++b) lds_values_ready(hb[b]);
    if (rank >= below) {
      const ScanResult sr = scan_loaded_bins<NB>(hb, rank - below, lane);  // every wave, same result
      bin = sr.bin;
      rr = rank - below - sr.below;
      c = sr.cnt;
      fast = sr.found && c <= kCap;
    } else {
      fast = false;  // tau lies below the window (far from Gaussian): exact fallback
    }
    DRCVAR_STAMP(4);
  }

  // ---- 4. candidates of the target bucket + tail sum below them -----------------------------
  double tau, dsum;  // dsum = sum_{d<tau} (d - tau)
  double rch;        // R_c |h| (risk_metrics.py:293, :234), wave 0
  if (fast) [[likely]] {
    uint32_t wbase = 0;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    const uint32_t ubin = static_cast<uint32_t>(bin);
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const uint32_t cj = (code[j / 2] >> (16 * (j % 2))) & 0xFFFFu;
      sq += cj < ubin ? d[j] - mu_d : 0.0;
      append_candidate(cand + wave * kCap, wbase, cj == ubin, d[j], lt_mask);
    }
    if constexpr (kPilot) {
      // small plans: this lane's tail partial goes to LDS unreduced; wave 0 reduces the four waves'
      // partials once after barrier 3, beside the ranking's LDS reads, instead of every wave
      // reducing its own ahead of the barrier
      lane_tail[tid] = sq;
      if (lane == 0) wcount[wave] = wbase;
    } else {
      sq = wave_reduce<OpAdd>(sq);
      if (lane == 0) {
        red_tail[wave] = sq;
        wcount[wave] = wbase;
      }
    }
    DRCVAR_STAMP(5);
    __syncthreads();                                                      // [barrier 3]
    DRCVAR_STAMP(6);
    if (wave != 0) {
      if (!PEER && wave == 1) write_mean_halfspace(rec, mux, muy, prm.rc, lane);
      return;
    }
    // the per-wave candidate counts are read in the same batch as the tail partials (the ranking
    // needs them for its candidate addresses; read inside it, they were a second LDS round trip)
    const uint32_t cw = wave_counts<NW>(wcount, lane);
    double s_below;
    if constexpr (kPilot) {
      double tl[NW];
#pragma unroll
      for (int w = 0; w < NW; ++w) tl[w] = lane_tail[w * kWave + lane];
      lds_values_ready(cw);
      double t = tl[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) t += tl[w];
      s_below = wave_reduce<OpAdd>(t);
    } else {
      s_below = sum_partials<NW>(red_tail);
      lds_values_ready(cw);
    }
    rch = prm.rc * norm_h(h0, h1);  // R_c |h|: off the histogram's critical path
    double s_cand;
    tau = rank_candidates<NW>(cand, cw, c, rr, lane, &s_cand);
    dsum = (s_below - static_cast<double>(rank - rr) * (tau - mu_d)) + s_cand;
  } else [[unlikely]] {
    // No spread in the moments: the noise-free step 0 of every obstacle (simulation/obstacles.py:63)
    // has all samples equal — settled from the registers by one min/max reduction (tau = the
    // common value, no tail below it) instead of the re-reading fallback, which costs two passes
    // over memory and four barriers and made these units the slowest of a launch.
    // Small plans only: on the 20-sample plan the extra live range costs the second workgroup
    // per CU (127 -> 130 VGPRs), and a C5 launch is bandwidth-bound, not set by its slowest unit.
    bool settled = false;
    if (P <= 8 && !(var_d > 0.0)) {  // uniform
      double lo[1] = {INFINITY}, hi[1] = {-INFINITY};
#pragma unroll
      for (int j = 0; j < P; ++j) {
        if (tid + j * BLOCK < n) {
          lo[0] = fmin(lo[0], d[j]);
          hi[0] = fmax(hi[0], d[j]);
        }
      }
      block_reduce<OpMin, NW, 1>(lo, red_rng);
      block_reduce<OpMax, NW, 1>(hi, red_rng + NW);
      if (lo[0] == hi[0]) {  // uniform (the reductions end with identical values in every lane)
        tau = lo[0];
        dsum = 0.0;
        settled = true;
      }
    }
    if (!settled) {
      const auto proj = [&](int i) { return project_at<LOAD != kLoadPair>(base, i, s_samp, h0, h1); };
      select_from_memory<BLOCK, LOG_NB>(proj, n, mu_d, rank, hist, cand, wcount, red_rng, red_tail,
                                        &tau, &dsum);
    }
    if (wave != 0) {
      if (!PEER && wave == 1) write_mean_halfspace(rec, mux, muy, prm.rc, lane);
      return;
    }
    rch = prm.rc * norm_h(h0, h1);
  }

  // ---- 5. offsets (wave 0) -------------------------------------------------------------------
  if constexpr (PEER)
    finish_offsets_peer(peer, gen, u, prm, rch, h0, h1, tau, dsum, mux, muy, lane);
  else
    finish_offsets<NW>(rec, prm, rch, h0, h1, tau, dsum, mux, muy, lane);
  if (status && lane == 0) status[u] = failure_status(false, prm);
  DRCVAR_STAMP(7);
}


// ---------------------------------------------------------------------------------------------
// streaming variant for N > DRCVAR_MAX_SAMPLES: nothing is held in registers — the mean is a
// strided pass over the unit's samples and the order statistic comes from select_from_memory's
// exact histogram refinement over re-reads (min/max pass, ~1 histogram pass per factor 10^3 of
// N, a candidate pass).  Any N up to 2^31 - 1; ~4 reads of the unit instead of 1.
// ---------------------------------------------------------------------------------------------
constexpr int kStreamBlock = 1024;
constexpr int kStreamLogNB = 10;

template <bool VEC, bool GIVEN_H>
__global__ void __launch_bounds__(kStreamBlock)
safe_halfspace_stream_kernel(const double* __restrict__ samples, int64_t n_steps, int n,
                             int64_t s_obs, int64_t s_step, int64_t s_samp,
                             const double* __restrict__ dir, int64_t dir_s_obs,
                             int64_t dir_s_step, Params prm, double* __restrict__ out,
                             int32_t* __restrict__ status) {
  constexpr int BLOCK = kStreamBlock;
  constexpr int NW = BLOCK / kWave;
  constexpr int NB = 1 << kStreamLogNB;
  __shared__ uint32_t hist[hist_words<NB>()];
  __shared__ double cand[NW * kCap];
  __shared__ uint32_t wcount[NW];
  __shared__ double red_mom[2 * NW];
  __shared__ double red_rng[2 * NW];
  __shared__ double red_tail[NW];
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = tid / kWave;
  const int64_t u = blockIdx.x;
  const int64_t o = u / n_steps;
  const int64_t t = u - o * n_steps;
  const double* base = samples + o * s_obs + t * s_step;
  double* rec = out + u * DRCVAR_OUT_WIDTH;
  double mom[2] = {0.0, 0.0};
  for (int i = tid; i < n; i += BLOCK) {
    const double* pt = base + static_cast<int64_t>(i) * s_samp;
    if constexpr (VEC) {
      const double2 v = *reinterpret_cast<const double2*>(pt);
      mom[0] += v.x;
      mom[1] += v.y;
    } else {
      mom[0] += pt[0];
      mom[1] += pt[1];
    }
  }
  block_reduce<OpAdd, NW, 2>(mom, red_mom);
  const double mux = mom[0] * prm.inv_n, muy = mom[1] * prm.inv_n;
  const bool bad = !(std::isfinite(mom[0]) && std::isfinite(mom[1]));
  const double* dp = dir + o * dir_s_obs + t * dir_s_step;
  double h0, h1;
  if constexpr (GIVEN_H) {
    h0 = dp[0];
    h1 = dp[1];
  } else {
    separating_direction(mux, muy, dp[0], dp[1], prm.degenerate_sq, &h0, &h1);
  }
  const double rch = prm.rc * norm_h(h0, h1);  // R_c |h|
  if (bad || prm.unbounded) {
    if (tid == 0) {
      const double r = rch;
      double m0, m1, g_mean;
      mean_halfspace(mux, muy, prm.rc, &m0, &m1, &g_mean);
      store_record(rec, m0, m1, g_mean, h0, h1, kSentinel, kSentinel, kSentinel - r);
      if (status) status[u] = failure_status(bad, prm);
    }
    return;
  }
  const double mu_d = h0 * mux + h1 * muy;
  double tau, dsum;
  const auto proj = [&](int i) { return project_at<VEC>(base, i, s_samp, h0, h1); };
  select_from_memory<BLOCK, kStreamLogNB>(proj, n, mu_d, prm.rank, hist,
                                               cand, wcount, red_rng, red_tail, &tau, &dsum);
  if (wave != 0) {
    if (wave == 1) write_mean_halfspace(rec, mux, muy, prm.rc, lane);
    return;
  }
  finish_offsets<NW>(rec, prm, rch, h0, h1, tau, dsum, mux, muy, lane);
  if (status && lane == 0) status[u] = failure_status(false, prm);
}

// ---------------------------------------------------------------------------------------------
// launch plans
// ---------------------------------------------------------------------------------------------
struct Plan {
  int block, per, log_nb;
  bool automatic;  // part of the default chain (smallest automatic plan with block*per >= N)
};
constexpr Plan kPlans[] = {
    {64, 2, 7, true},       // N <=   128
    {128, 4, 8, true},      // N <=   512
    {256, 4, 9, true},      // N <=  1024
    {256, 8, 10, true},     // N <=  2048
    {256, 16, 10, true},    // N <=  4096
    {256, 20, 10, true},    // N <=  5120   (C4 N = 5000: 27.3 us vs 38.9 us on 512 x 16)
    {512, 16, 10, true},    // N <=  8192   (2 workgroups per CU)
    {512, 20, 10, true},    // N <= 10240   (2 workgroups per CU)
    {1024, 12, 10, true},   // N <= 12288
    {1024, 16, 10, true},   // N <= 16384
    // alternative geometries, selectable through drcvar_safe_halfspaces_f64_ex (tuning)
    {64, 16, 9, false},
    {128, 8, 9, false},
    {512, 2, 9, false},
    {1024, 10, 10, false},
};
constexpr int kNumPlans = sizeof(kPlans) / sizeof(kPlans[0]);

int pick_plan(int64_t n, int threads, int per) {
  for (int p = 0; p < kNumPlans; ++p) {
    const Plan& pl = kPlans[p];
    if (n > static_cast<int64_t>(pl.block) * pl.per) continue;
    if (threads == 0 && per == 0) {
      if (pl.automatic) return p;
    } else if (pl.block == threads && pl.per == per) {
      return p;
    }
  }
  return -1;
}

struct Launch {
  const double* samples;
  int64_t units, n_steps, n, s_obs, s_step, s_samp;
  const double* dir;
  int64_t dir_s_obs, dir_s_step;
  Params prm;
  double* out;
  int32_t* status;  // [units] or null
  hipStream_t stream;
  PeerArgs peer;    // the peer form only
};

// grid (n_steps, obstacles), at most kMaxGridY obstacles per launch (the y-dimension limit):
// larger batches are split into obstacle chunks on the host
constexpr int64_t kMaxGridY = 65535;

template <int BLOCK, int P, int LOG_NB, int LOAD, bool GIVEN_H, bool PEER>
int launch_form(const Launch& L) {
  const int64_t n_obs = L.units / L.n_steps;
  const size_t dyn = 0;
  for (int64_t o0 = 0; o0 < n_obs; o0 += kMaxGridY) {
    const int64_t chunk = n_obs - o0 < kMaxGridY ? n_obs - o0 : kMaxGridY;
    PeerArgs pa = L.peer;
    pa.row_base += o0 * L.n_steps;
    hipLaunchKernelGGL((safe_halfspace_kernel<BLOCK, P, LOG_NB, LOAD, GIVEN_H, PEER>),
                       dim3(static_cast<unsigned>(L.n_steps), static_cast<unsigned>(chunk)),
                       dim3(BLOCK), dyn, L.stream, L.samples + o0 * L.s_obs, L.n_steps,
                       static_cast<int>(L.n), L.s_obs, L.s_step, L.s_samp,
                       L.dir + o0 * L.dir_s_obs, L.dir_s_obs, L.dir_s_step, L.prm,
                       L.out + o0 * L.n_steps * DRCVAR_OUT_WIDTH,
                       L.status ? L.status + o0 * L.n_steps : nullptr, pa);
  }
  return DRCVAR_OK;
}

template <int BLOCK, int P, int LOG_NB, bool GIVEN_H, bool PEER>
int launch_plan(Launch L, bool vec) {
  const int64_t sub = P <= 8 ? kWave : BLOCK;  // the window's subsample: pilot or row 0 (kernel)
  L.prm.inv_n0 = 1.0 / static_cast<double>(L.n < sub ? L.n : sub);
  L.prm.hist_scale = static_cast<double>(1 << LOG_NB) / (2.0 * L.prm.window_sd);
  // measured on C5 (2.05 GB): nontemporal 16-B loads 0.746 of HBM peak vs 0.715; on C3 (3.2 MB,
  // cache-resident across steps) they cost 3 %, so only launches larger than the MALL use them
  const bool nt = vec && L.units * L.n * 16 > kNtBytes;
  if (nt) return launch_form<BLOCK, P, LOG_NB, kLoadNt, GIVEN_H, PEER>(L);
  if (vec) return launch_form<BLOCK, P, LOG_NB, kLoadVec, GIVEN_H, PEER>(L);
  if constexpr (PEER) return DRCVAR_ERR_UNSUPPORTED;  // the peer form reads packed 16-B samples
  else return launch_form<BLOCK, P, LOG_NB, kLoadPair, GIVEN_H, false>(L);
}

template <bool GIVEN_H>
void launch_stream(const Launch& L, bool vec) {
  const dim3 grid(static_cast<unsigned>(L.units)), block(kStreamBlock);
  if (vec) {
    hipLaunchKernelGGL((safe_halfspace_stream_kernel<true, GIVEN_H>), grid, block, 0, L.stream,
                       L.samples, L.n_steps, static_cast<int>(L.n), L.s_obs, L.s_step, L.s_samp,
                       L.dir, L.dir_s_obs, L.dir_s_step, L.prm, L.out, L.status);
  } else {
    hipLaunchKernelGGL((safe_halfspace_stream_kernel<false, GIVEN_H>), grid, block, 0, L.stream,
                       L.samples, L.n_steps, static_cast<int>(L.n), L.s_obs, L.s_step, L.s_samp,
                       L.dir, L.dir_s_obs, L.dir_s_step, L.prm, L.out, L.status);
  }
}

template <bool GIVEN_H, bool PEER = false>
int dispatch(const Launch& L, int threads, int per) {
  if (L.units == 0) return DRCVAR_OK;
  const bool vec = (reinterpret_cast<uintptr_t>(L.samples) % 16 == 0) && (L.s_obs % 2 == 0) &&
                   (L.s_step % 2 == 0) && (L.s_samp % 2 == 0);
  if (L.n > DRCVAR_MAX_SAMPLES) {  // beyond the register plans: the streaming kernel
    if (PEER || threads != 0 || per != 0) return DRCVAR_ERR_UNSUPPORTED;
    if (L.n > DRCVAR_MAX_SAMPLES_STREAM) return DRCVAR_ERR_UNSUPPORTED;
    (void)hipGetLastError();
    launch_stream<GIVEN_H>(L, vec);
    return hipGetLastError() == hipSuccess ? DRCVAR_OK : DRCVAR_ERR_LAUNCH;
  }
  const int p = pick_plan(L.n, threads, per);
  if (p < 0) return DRCVAR_ERR_UNSUPPORTED;
  (void)hipGetLastError();  // clear stale errors from unrelated work
  int rc = DRCVAR_OK;
  switch (p) {
    case 0: rc = launch_plan<64, 2, 7, GIVEN_H, PEER>(L, vec); break;
    case 1: rc = launch_plan<128, 4, 8, GIVEN_H, PEER>(L, vec); break;
    case 2: rc = launch_plan<256, 4, 9, GIVEN_H, PEER>(L, vec); break;
    case 3: rc = launch_plan<256, 8, 10, GIVEN_H, PEER>(L, vec); break;
    case 4: rc = launch_plan<256, 16, 10, GIVEN_H, PEER>(L, vec); break;
    case 5: rc = launch_plan<256, 20, 10, GIVEN_H, PEER>(L, vec); break;
    case 6: rc = launch_plan<512, 16, 10, GIVEN_H, PEER>(L, vec); break;
    case 7: rc = launch_plan<512, 20, 10, GIVEN_H, PEER>(L, vec); break;
    case 8: rc = launch_plan<1024, 12, 10, GIVEN_H, PEER>(L, vec); break;
    case 9: rc = launch_plan<1024, 16, 10, GIVEN_H, PEER>(L, vec); break;
    default:
      if constexpr (PEER) {
        return DRCVAR_ERR_UNSUPPORTED;  // tuning geometries: not in the peer form
      } else {
        switch (p) {
          case 10: rc = launch_plan<64, 16, 9, GIVEN_H, false>(L, vec); break;
          case 11: rc = launch_plan<128, 8, 9, GIVEN_H, false>(L, vec); break;
          case 12: rc = launch_plan<512, 2, 9, GIVEN_H, false>(L, vec); break;
          default: rc = launch_plan<1024, 10, 10, GIVEN_H, false>(L, vec); break;
        }
      }
  }
  if (rc != DRCVAR_OK) return rc;
  return hipGetLastError() == hipSuccess ? DRCVAR_OK : DRCVAR_ERR_LAUNCH;
}

// Standard-normal quantile (P. J. Acklam's rational approximation, |rel err| < 1.2e-9) — only
// positions the fast-path window, so its accuracy never affects results.
double normal_quantile(double p) {
  static const double a[] = {-3.969683028665376e+01, 2.209460984245205e+02, -2.759285104469687e+02,
                             1.383577518672690e+02, -3.066479806614716e+01, 2.506628277459239e+00};
  static const double b[] = {-5.447609879822406e+01, 1.615858368580409e+02, -1.556989798598866e+02,
                             6.680131188771972e+01, -1.328068155288572e+01};
  static const double c[] = {-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e+00,
                             -2.549732539343734e+00, 4.374664141464968e+00, 2.938163982698783e+00};
  static const double d[] = {7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e+00,
                             3.754408661907416e+00};
  p = std::fmin(std::fmax(p, 1e-12), 1.0 - 1e-12);
  const double plow = 0.02425;
  if (p < plow) {
    const double q = std::sqrt(-2.0 * std::log(p));
    return (((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
           ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1.0);
  }
  if (p > 1.0 - plow) return -normal_quantile(1.0 - p);
  const double q = p - 0.5, r = q * q;
  return (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * q /
         (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1.0);
}

Params make_params(double rr, double ro, double alpha, double delta, double eps, int64_t n) {
  Params p;
  p.rc = rr + ro;
  p.alpha = alpha;
  p.delta = delta;
  p.epsilon = eps;
  p.eps_over_alpha = eps / alpha;
  const double dn = static_cast<double>(n);
  p.inv_n = 1.0 / dn;
  p.k = alpha * dn;                      // exactly as the reference forms alpha * n_samples
  p.inv_k = 1.0 / p.k;
  p.unbounded = !(p.k <= dn);
  const int64_t m = static_cast<int64_t>(std::floor(p.k));
  p.rank = static_cast<uint32_t>(p.unbounded ? 0 : (m < n - 1 ? m : n - 1));
  // window: the Gaussian alpha-quantile +- max(0.25 sd, 12 standard errors of the sample quantile)
  const double a = std::fmin(std::fmax(alpha, 1e-12), 1.0 - 1e-12);
  p.z_alpha = normal_quantile(a);
  const double phi = std::exp(-0.5 * p.z_alpha * p.z_alpha) * 0.3989422804014327;
  const double se = std::sqrt(a * (1.0 - a) / dn) / phi;
  p.window_sd = std::fmax(0.25, 12.0 * se);
  p.z_lo = p.z_alpha - p.window_sd;
  double t = 1e-20;  // smallest t with sqrt(t) >= 1e-10 (sqrt is correctly rounded and monotone)
  while (std::sqrt(t) >= 1e-10) t = std::nextafter(t, 0.0);
  while (std::sqrt(t) < 1e-10) t = std::nextafter(t, 1.0);
  p.degenerate_sq = t;
  return p;
}

bool params_ok(double rr, double ro, double alpha, double delta, double eps) {
  return std::isfinite(rr) && std::isfinite(ro) && std::isfinite(alpha) && alpha > 0.0 &&
         std::isfinite(delta) && std::isfinite(eps);
}

int safe_halfspaces(const double* samples, int64_t n_obstacles, int64_t n_steps,
                    int64_t n_samples, int64_t stride_obstacle, int64_t stride_step,
                    int64_t stride_sample, const double* ego_ref_pos, int64_t ego_stride_step,
                    double robot_radius, double obstacle_radius, double alpha, double delta,
                    double epsilon, double* out, int32_t* status, void* stream, int threads,
                    int per, const drcvar_peer_set* peers = nullptr, int64_t row_base = 0) {
  if (n_obstacles < 0 || n_steps < 0 || n_samples < 1) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (!params_ok(robot_radius, obstacle_radius, alpha, delta, epsilon))
    return DRCVAR_ERR_INVALID_ARGUMENT;
  const int64_t units = n_obstacles * n_steps;
  if (units == 0) return DRCVAR_OK;
  if (!samples || !ego_ref_pos || (!out && !peers) || units > 0x7fffffff)
    return DRCVAR_ERR_INVALID_ARGUMENT;
  Launch L{samples, units, n_steps, n_samples, stride_obstacle, stride_step, stride_sample,
           ego_ref_pos, 0, ego_stride_step,
           make_params(robot_radius, obstacle_radius, alpha, delta, epsilon, n_samples), out,
           status, static_cast<hipStream_t>(stream)};
  if (peers) {
    const drcvar_peer_set& ps = *peers;
    if (ps.n_ranks < 1 || ps.n_ranks > DRCVAR_MAX_PEERS || ps.rank < 0 || ps.rank >= ps.n_ranks ||
        !ps.state || ps.rows < 0 || row_base < 0 || row_base + units > ps.rows)
      return DRCVAR_ERR_INVALID_ARGUMENT;
    for (int j = 0; j < ps.n_ranks; ++j)
      if (!ps.region[j]) return DRCVAR_ERR_INVALID_ARGUMENT;
    for (int j = 0; j < DRCVAR_MAX_PEERS; ++j) L.peer.region[j] = j < ps.n_ranks ? ps.region[j] : nullptr;
    L.peer.rows = ps.rows;
    L.peer.row_base = row_base;
    L.peer.gen = ps.state;
    L.peer.n_ranks = ps.n_ranks;
    return dispatch<false, true>(L, 0, 0);
  }
  return dispatch<false>(L, threads, per);
}

}  // namespace

extern "C" {

#ifdef DRCVAR_STAMPS
// diagnostic build only (not part of the ABI header): copy the phase stamps to the host
int drcvar_diag_stamps(unsigned long long* host, int n_units) {
  const int n = n_units < kStampUnits ? n_units : kStampUnits;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * n * kStamps,
                             0, hipMemcpyDeviceToHost) == hipSuccess ? n : -1;
}
#endif

int drcvar_abi_version(void) { return DRCVAR_ABI_VERSION; }

const char* drcvar_strerror(int code) {
  switch (code) {
    case DRCVAR_OK: return "ok";
    case DRCVAR_ERR_INVALID_ARGUMENT: return "invalid argument";
    case DRCVAR_ERR_UNSUPPORTED: return "n_samples beyond DRCVAR_MAX_SAMPLES_STREAM or no such launch geometry";
    case DRCVAR_ERR_LAUNCH: return "HIP kernel launch failed";
    default: return "unknown error";
  }
}

int drcvar_launch_plan(int64_t n_samples, int32_t* threads_per_unit, int32_t* samples_per_thread,
                       int32_t* bins) {
  if (n_samples < 1) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (n_samples > DRCVAR_MAX_SAMPLES) {  // streaming kernel: nothing per thread held on chip
    if (n_samples > DRCVAR_MAX_SAMPLES_STREAM) return DRCVAR_ERR_UNSUPPORTED;
    if (threads_per_unit) *threads_per_unit = kStreamBlock;
    if (samples_per_thread) *samples_per_thread = 0;
    if (bins) *bins = 1 << kStreamLogNB;
    return DRCVAR_OK;
  }
  const int p = pick_plan(n_samples, 0, 0);
  if (p < 0) return DRCVAR_ERR_UNSUPPORTED;
  if (threads_per_unit) *threads_per_unit = kPlans[p].block;
  if (samples_per_thread) *samples_per_thread = kPlans[p].per;
  if (bins) *bins = 1 << kPlans[p].log_nb;
  return DRCVAR_OK;
}

int drcvar_safe_halfspaces_f64(const double* samples, int64_t n_obstacles, int64_t n_steps,
                               int64_t n_samples, int64_t stride_obstacle, int64_t stride_step,
                               int64_t stride_sample, const double* ego_ref_pos,
                               int64_t ego_stride_step, double robot_radius,
                               double obstacle_radius, double alpha, double delta, double epsilon,
                               double* out, void* stream) {
  return safe_halfspaces(samples, n_obstacles, n_steps, n_samples, stride_obstacle, stride_step,
                         stride_sample, ego_ref_pos, ego_stride_step, robot_radius,
                         obstacle_radius, alpha, delta, epsilon, out, nullptr, stream, 0, 0);
}

int drcvar_safe_halfspaces_f64_ex(const double* samples, int64_t n_obstacles, int64_t n_steps,
                                  int64_t n_samples, int64_t stride_obstacle, int64_t stride_step,
                                  int64_t stride_sample, const double* ego_ref_pos,
                                  int64_t ego_stride_step, double robot_radius,
                                  double obstacle_radius, double alpha, double delta,
                                  double epsilon, double* out, void* stream,
                                  int32_t threads_per_unit, int32_t samples_per_thread) {
  if ((threads_per_unit == 0) != (samples_per_thread == 0)) return DRCVAR_ERR_INVALID_ARGUMENT;
  return safe_halfspaces(samples, n_obstacles, n_steps, n_samples, stride_obstacle, stride_step,
                         stride_sample, ego_ref_pos, ego_stride_step, robot_radius,
                         obstacle_radius, alpha, delta, epsilon, out, nullptr, stream,
                         threads_per_unit, samples_per_thread);
}

int drcvar_safe_halfspaces_f64_v2(const double* samples, int64_t n_obstacles, int64_t n_steps,
                                  int64_t n_samples, int64_t stride_obstacle, int64_t stride_step,
                                  int64_t stride_sample, const double* ego_ref_pos,
                                  int64_t ego_stride_step, double robot_radius,
                                  double obstacle_radius, double alpha, double delta,
                                  double epsilon, double* out, int32_t* status, void* stream,
                                  int32_t threads_per_unit, int32_t samples_per_thread) {
  if ((threads_per_unit == 0) != (samples_per_thread == 0)) return DRCVAR_ERR_INVALID_ARGUMENT;
  return safe_halfspaces(samples, n_obstacles, n_steps, n_samples, stride_obstacle, stride_step,
                         stride_sample, ego_ref_pos, ego_stride_step, robot_radius,
                         obstacle_radius, alpha, delta, epsilon, out, status, stream,
                         threads_per_unit, samples_per_thread);
}

int drcvar_safe_halfspaces_f64_peer(const double* samples, int64_t n_obstacles, int64_t n_steps,
                                    int64_t n_samples, int64_t stride_obstacle, int64_t stride_step,
                                    int64_t stride_sample, const double* ego_ref_pos,
                                    int64_t ego_stride_step, double robot_radius,
                                    double obstacle_radius, double alpha, double delta,
                                    double epsilon, const drcvar_peer_set* peers, int64_t row_base,
                                    int32_t* status, void* stream) {
  if (!peers) return DRCVAR_ERR_INVALID_ARGUMENT;
  return safe_halfspaces(samples, n_obstacles, n_steps, n_samples, stride_obstacle, stride_step,
                         stride_sample, ego_ref_pos, ego_stride_step, robot_radius,
                         obstacle_radius, alpha, delta, epsilon, nullptr, status, stream, 0, 0,
                         peers, row_base);
}

int drcvar_offsets_given_h_f64_v2(const double* samples, int64_t n_units, int64_t n_samples,
                                  int64_t stride_unit, int64_t stride_sample, const double* h,
                                  int64_t h_stride_unit, double robot_radius,
                                  double obstacle_radius, double alpha, double delta,
                                  double epsilon, double* out, int32_t* status, void* stream) {
  if (n_units < 0 || n_samples < 1) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (!params_ok(robot_radius, obstacle_radius, alpha, delta, epsilon))
    return DRCVAR_ERR_INVALID_ARGUMENT;
  if (n_units == 0) return DRCVAR_OK;
  if (!samples || !h || !out || n_units > 0x7fffffff) return DRCVAR_ERR_INVALID_ARGUMENT;
  // units along the grid's x dimension: one "obstacle" of n_units steps
  Launch L{samples, n_units, n_units, n_samples, 0, stride_unit, stride_sample,
           h, 0, h_stride_unit,
           make_params(robot_radius, obstacle_radius, alpha, delta, epsilon, n_samples), out,
           status, static_cast<hipStream_t>(stream)};
  return dispatch<true>(L, 0, 0);
}

int drcvar_offsets_given_h_f64(const double* samples, int64_t n_units, int64_t n_samples,
                               int64_t stride_unit, int64_t stride_sample, const double* h,
                               int64_t h_stride_unit, double robot_radius, double obstacle_radius,
                               double alpha, double delta, double epsilon, double* out,
                               void* stream) {
  return drcvar_offsets_given_h_f64_v2(samples, n_units, n_samples, stride_unit, stride_sample, h,
                                       h_stride_unit, robot_radius, obstacle_radius, alpha, delta,
                                       epsilon, out, nullptr, stream);
}

}  // extern "C"
