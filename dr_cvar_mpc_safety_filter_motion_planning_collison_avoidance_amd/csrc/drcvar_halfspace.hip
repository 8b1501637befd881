// drcvar_halfspace.hip — fused safe-halfspace kernel for MI355X (gfx950, CDNA4) + its C ABI.
//
// One workgroup evaluates one unit = one (obstacle, horizon step): N fp64 samples xi_i in R^2.
// Everything the reference does per unit in core/halfspaces.py:70-194 and core/risk_metrics.py:
// 84-338 happens in ONE pass over HBM (16 B per sample, read once, coalesced 16-B/lane loads):
//
//   1. load the samples into registers (P per thread), block-reduce their sum   -> mean mu
//   2. h = (mu - ego)/|mu - ego| ([1,0] if < 1e-10)            core/geometry.py:35-53
//      mean halfspace from the origin                           core/halfspaces.py:84-94
//   3. d_i = h . xi_i, block min/max                            core/risk_metrics.py:145,233
//   4. exact (m+1)-th order statistic tau of d, m = floor(alpha*N), sort-free:
//        value-linear histogram of d in LDS (NB bins, LDS atomics) -> scan -> target bucket;
//        refine (exact min/max of that bucket, then re-histogram; falls back to order-preserving
//        integer keys when the value range degenerates) until <= kCap candidates remain;
//        rank the candidates directly.  Every bucket map is monotone in d, so a candidate set is
//        always a contiguous run of the sorted order and the result is exact with ties.
//   5. L = tau + sum_{d<tau} (d - tau) / (alpha N)             lower-tail mean = -CVaR_alpha(-d)
//      (= (sum of the m smallest + (alpha N - m) tau) / (alpha N); deterministic block reduction)
//   6. g_cvar = r - delta - L, g* = r - delta + eps/alpha - L, g~ = g* - r, r = R_c |h|
//      (closed-form optimum of the LPs at core/risk_metrics.py:105-125 and :198-213;
//       lambda* = 1/alpha because lambda only enters the budget row and its bound, :110,:122)
//
// No MFMA: ~6 flops per 16 B sample — the kernel is bounded by HBM.
// All reductions have a fixed order, so results are bitwise reproducible run to run.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "drcvar_halfspace.h"

namespace {

constexpr int kWave = 64;
constexpr int kCap = 128;          // candidate count ranked directly
constexpr int kMaxValueIters = 3;  // value-linear passes before switching to integer keys
constexpr double kSentinel = 100.0;

struct Params {
  double rc;  // robot_radius + obstacle_radius
  double alpha;
  double delta;
  double epsilon;
};

// ---------------------------------------------------------------------------------------------
// wave / workgroup reductions (butterfly: every lane ends with the bitwise-identical value)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, kWave));
  return v;
}

// Sum of three values over the workgroup; `slot` is LDS scratch of 3*NW doubles owned by this
// call site (callers never reuse a slot without two barriers in between).
template <int NW>
__device__ __forceinline__ void block_sum3(double& a, double& b, double& c, double* slot) {
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum(c);
  if constexpr (NW > 1) {
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) {
      slot[w] = a;
      slot[NW + w] = b;
      slot[2 * NW + w] = c;
    }
    __syncthreads();
    a = slot[0];
    b = slot[NW];
    c = slot[2 * NW];
#pragma unroll
    for (int i = 1; i < NW; ++i) {
      a += slot[i];
      b += slot[NW + i];
      c += slot[2 * NW + i];
    }
  }
}

template <int NW>
__device__ __forceinline__ void block_minmax(double& mn, double& mx, double* slot) {
  mn = wave_min(mn);
  mx = wave_max(mx);
  if constexpr (NW > 1) {
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) {
      slot[w] = mn;
      slot[NW + w] = mx;
    }
    __syncthreads();
    mn = slot[0];
    mx = slot[NW];
#pragma unroll
    for (int i = 1; i < NW; ++i) {
      mn = fmin(mn, slot[i]);
      mx = fmax(mx, slot[NW + i]);
    }
  }
}

// order-preserving map double -> uint64 (total order on non-NaN values)
__device__ __forceinline__ uint64_t f64_key(double d) {
  const uint64_t u = static_cast<uint64_t>(__double_as_longlong(d));
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

// Monotone bucket map of the current candidate interval [lo, hi] onto NB bins.
template <int LOG_NB>
struct BucketMap {
  static constexpr int NB = 1 << LOG_NB;
  bool value_mode;
  double lo, scale;
  uint64_t klo;
  int shift;

  __device__ __forceinline__ void init(double lo_, double hi_, int iter) {
    lo = lo_;
    const double range = hi_ - lo_;
    scale = static_cast<double>(NB) / range;
    // value-linear while the range is well-conditioned: bucket(lo) = 0 and bucket(hi) >= 1
    value_mode = iter < kMaxValueIters && range > 0.0 && scale < 1e300 && range * scale >= 1.0;
    klo = f64_key(lo_);
    const uint64_t diff = f64_key(hi_) - klo;  // >= 1 when hi > lo
    const int bits = 64 - __builtin_clzll(diff | 1ull);
    shift = bits > LOG_NB ? bits - LOG_NB : 0;
  }
  // precondition: lo <= d <= hi
  __device__ __forceinline__ int operator()(double d) const {
    if (value_mode) {
      const int b = static_cast<int>((d - lo) * scale);
      return b < NB - 1 ? b : NB - 1;
    }
    return static_cast<int>((f64_key(d) - klo) >> shift);
  }
};

// Wave 0: find the bin holding the candidate of rank rr (0-based) of the histogram.
template <int NB>
__device__ __forceinline__ void scan_bins(const uint32_t* hist, uint32_t rr, int lane,
                                          int* out_bin, uint32_t* out_below, uint32_t* out_cnt) {
  constexpr int B = NB / kWave;  // contiguous bins per lane
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < B; ++q) s += hist[lane * B + q];
  uint32_t incl = s;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const uint32_t v = __shfl_up(incl, off, kWave);
    if (lane >= off) incl += v;
  }
  const unsigned long long hit = __ballot(incl > rr);
  const int owner = __ffsll(static_cast<long long>(hit)) - 1;
  if (lane == owner) {
    uint32_t cum = incl - s;
    for (int q = 0; q < B; ++q) {
      const uint32_t h = hist[lane * B + q];
      if (cum + h > rr) {
        *out_bin = lane * B + q;
        *out_below = cum;
        *out_cnt = h;
        break;
      }
      cum += h;
    }
  }
}

__device__ __forceinline__ bool in_range(double d, double lo, double hi) {
  return lo <= d && d <= hi;  // false for the NaN padding of idle slots
}

// ---------------------------------------------------------------------------------------------
// the fused kernel
//   BLOCK    threads per unit (one workgroup per unit)
//   P        samples held per thread (N <= BLOCK * P)
//   LOG_NB   log2 of histogram bins
//   VEC      every (x, y) pair is 16-B aligned -> one 16-B load per sample
//   GIVEN_H  `dir` holds h per unit (cvar_halfspace / dr_cvar_halfspace) instead of ego per step
// ---------------------------------------------------------------------------------------------
template <int BLOCK, int P, int LOG_NB, bool VEC, bool GIVEN_H>
__global__ void __launch_bounds__(BLOCK)
safe_halfspace_kernel(const double* __restrict__ samples, int64_t n_steps, int64_t n,
                      int64_t s_obs, int64_t s_step, int64_t s_samp,
                      const double* __restrict__ dir, int64_t dir_s_obs, int64_t dir_s_step,
                      Params prm, double* __restrict__ out) {
  constexpr int NW = BLOCK / kWave;
  constexpr int NB = 1 << LOG_NB;
  __shared__ uint32_t hist[NB];
  __shared__ double cand[kCap];
  __shared__ double red_sum[3 * NW];
  __shared__ double red_rng[2 * NW];
  __shared__ double red_ref[2 * NW];
  __shared__ double red_tail[3 * NW];
  __shared__ int sh_bin;
  __shared__ uint32_t sh_below, sh_cnt, sh_ncand;
  __shared__ double sh_tau;

  const int tid = threadIdx.x;
  const int64_t u = blockIdx.x;
  const int64_t o = u / n_steps;
  const int64_t t = u - o * n_steps;
  const double* base = samples + o * s_obs + t * s_step;
  if (tid == 0) sh_ncand = 0;

  // ---- 1. load + sum ---------------------------------------------------------------------
  double x[P], y[P];
  double sx = 0.0, sy = 0.0, bad = 0.0;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int64_t i = tid + static_cast<int64_t>(j) * BLOCK;
    if (i < n) {
      if constexpr (VEC) {
        const double2 v = *reinterpret_cast<const double2*>(base + i * s_samp);
        x[j] = v.x;
        y[j] = v.y;
      } else {
        x[j] = base[i * s_samp];
        y[j] = base[i * s_samp + 1];
      }
      sx += x[j];
      sy += y[j];
      bad += (std::isfinite(x[j]) && std::isfinite(y[j])) ? 0.0 : 1.0;
    } else {
      x[j] = 0.0;
      y[j] = 0.0;
    }
  }
  block_sum3<NW>(sx, sy, bad, red_sum);
  const double dn = static_cast<double>(n);
  const double mux = sx / dn, muy = sy / dn;

  // ---- 2. directions ---------------------------------------------------------------------
  const double* dp = dir + o * dir_s_obs + t * dir_s_step;
  double h0, h1;
  if constexpr (GIVEN_H) {
    h0 = dp[0];
    h1 = dp[1];
  } else {
    const double dx = mux - dp[0], dy = muy - dp[1];
    const double nrm = sqrt(dx * dx + dy * dy);
    h0 = 1.0;
    h1 = 0.0;
    if (!(nrm < 1e-10)) {
      h0 = dx / nrm;
      h1 = dy / nrm;
    }
  }
  const double r = prm.rc * sqrt(h0 * h0 + h1 * h1);
  double* rec = out + u * DRCVAR_OUT_WIDTH;
  if (tid == 0) {
    const double nm = sqrt(mux * mux + muy * muy);
    double m0 = 1.0, m1 = 0.0;
    if (!(nm < 1e-10)) {
      m0 = mux / nm;
      m1 = muy / nm;
    }
    rec[DRCVAR_COL_MEAN_H0] = m0;
    rec[DRCVAR_COL_MEAN_H1] = m1;
    rec[DRCVAR_COL_G_MEAN] = -((m0 * mux + m1 * muy) - prm.rc * sqrt(m0 * m0 + m1 * m1));
    rec[DRCVAR_COL_H0] = h0;
    rec[DRCVAR_COL_H1] = h1;
  }
  const double k = prm.alpha * dn;
  if (bad != 0.0 || !(k <= dn)) {  // solver-failure convention, risk_metrics.py:298-303,334-338
    if (tid == 0) {
      rec[DRCVAR_COL_G_CVAR] = kSentinel;
      rec[DRCVAR_COL_G_DR_STAR] = kSentinel;
      rec[DRCVAR_COL_G_DR_TILDE] = kSentinel - r;
    }
    return;  // uniform across the workgroup
  }

  // ---- 3. projections --------------------------------------------------------------------
  double d[P];
  double dmin = INFINITY, dmax = -INFINITY;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int64_t i = tid + static_cast<int64_t>(j) * BLOCK;
    d[j] = (i < n) ? h0 * x[j] + h1 * y[j] : NAN;
    if (i < n) {
      dmin = fmin(dmin, d[j]);
      dmax = fmax(dmax, d[j]);
    }
  }
  block_minmax<NW>(dmin, dmax, red_rng);

  // ---- 4. exact order statistic ----------------------------------------------------------
  const int64_t m = static_cast<int64_t>(floor(k));
  const uint32_t rank = static_cast<uint32_t>(m < n - 1 ? m : n - 1);
  double tau;
  if (dmin == dmax) {
    tau = dmin;
  } else {
    double lo = dmin, hi = dmax;
    uint32_t rr = rank;                      // rank inside the candidate set
    uint32_t c = static_cast<uint32_t>(n);  // candidate count
    bool have_bin = false;                   // candidates = bucket `bin` of `map` within [lo, hi]
    int bin = 0;
    BucketMap<LOG_NB> map;
    for (int iter = 0; c > kCap; ++iter) {
      if (have_bin) {  // shrink [lo, hi] to the exact range of the target bucket
        double mn = INFINITY, mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < P; ++j) {
          if (in_range(d[j], lo, hi) && map(d[j]) == bin) {
            mn = fmin(mn, d[j]);
            mx = fmax(mx, d[j]);
          }
        }
        block_minmax<NW>(mn, mx, red_ref);
        lo = mn;
        hi = mx;
        have_bin = false;
        if (lo == hi) break;
      }
      map.init(lo, hi, iter);
      for (int b = tid; b < NB; b += BLOCK) hist[b] = 0u;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < P; ++j) {
        if (in_range(d[j], lo, hi)) atomicAdd(&hist[map(d[j])], 1u);
      }
      __syncthreads();
      if (tid < kWave) scan_bins<NB>(hist, rr, tid, &sh_bin, &sh_below, &sh_cnt);
      __syncthreads();
      bin = sh_bin;
      rr -= sh_below;
      c = sh_cnt;
      have_bin = true;
    }
    if (!have_bin && lo == hi) {
      tau = lo;
    } else {
      // compact the <= kCap candidates into LDS and rank them directly
#pragma unroll
      for (int j = 0; j < P; ++j) {
        if (in_range(d[j], lo, hi) && (!have_bin || map(d[j]) == bin)) {
          cand[atomicAdd(&sh_ncand, 1u)] = d[j];
        }
      }
      __syncthreads();
      for (uint32_t a = tid; a < c; a += BLOCK) {
        const double v = cand[a];
        uint32_t less = 0, eq = 0;
        for (uint32_t b = 0; b < c; ++b) {
          const double w = cand[b];
          less += (w < v) ? 1u : 0u;
          eq += (w == v) ? 1u : 0u;
        }
        if (less <= rr && rr < less + eq) sh_tau = v;  // ties write the same value
      }
      __syncthreads();
      tau = sh_tau;
    }
  }

  // ---- 5. lower-tail sum, relative to tau -------------------------------------------------
  // S_m = sum_{d<tau} d + (m - #{d<tau}) tau  and  L = (S_m + (k - m) tau) / k  simplify to
  // L = tau + D / k  with  D = sum_{d<tau} (d - tau) <= 0: the differences are small, so the sum
  // carries far less rounding than the plain tail sum when |d| >> spread.
  double dsum = 0.0, unused0 = 0.0, unused1 = 0.0;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    if (d[j] < tau) dsum += d[j] - tau;
  }
  block_sum3<NW>(dsum, unused0, unused1, red_tail);

  // ---- 6. offsets -------------------------------------------------------------------------
  if (tid == 0) {
    const double L = tau + dsum / k;
    rec[DRCVAR_COL_G_CVAR] = r - prm.delta - L;
    if (prm.epsilon >= 0.0) {
      const double g_star = r - prm.delta + prm.epsilon / prm.alpha - L;
      rec[DRCVAR_COL_G_DR_STAR] = g_star;
      rec[DRCVAR_COL_G_DR_TILDE] = g_star - r;
    } else {  // DR LP unbounded (lambda -> inf): solver-failure sentinel
      rec[DRCVAR_COL_G_DR_STAR] = kSentinel;
      rec[DRCVAR_COL_G_DR_TILDE] = kSentinel - r;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// launch plans: smallest plan whose BLOCK * P covers N
// ---------------------------------------------------------------------------------------------
struct Plan {
  int block, per, log_nb;
};
constexpr Plan kPlans[] = {
    {64, 2, 7},      // N <=   128
    {128, 4, 8},     // N <=   512
    {256, 4, 9},     // N <=  1024
    {256, 8, 10},    // N <=  2048
    {256, 16, 11},   // N <=  4096
    {512, 16, 12},   // N <=  8192
    {1024, 10, 12},  // N <= 10240
    {1024, 12, 12},  // N <= 12288
    {1024, 16, 12},  // N <= 16384
};
constexpr int kNumPlans = sizeof(kPlans) / sizeof(kPlans[0]);

int pick_plan(int64_t n) {
  for (int p = 0; p < kNumPlans; ++p)
    if (n <= static_cast<int64_t>(kPlans[p].block) * kPlans[p].per) return p;
  return -1;
}

struct Launch {
  const double* samples;
  int64_t units, n_steps, n, s_obs, s_step, s_samp;
  const double* dir;
  int64_t dir_s_obs, dir_s_step;
  Params prm;
  double* out;
  hipStream_t stream;
};

template <int BLOCK, int P, int LOG_NB, bool GIVEN_H>
void launch_plan(const Launch& L, bool vec) {
  const dim3 grid(static_cast<unsigned>(L.units)), block(BLOCK);
  if (vec) {
    hipLaunchKernelGGL((safe_halfspace_kernel<BLOCK, P, LOG_NB, true, GIVEN_H>), grid, block, 0,
                       L.stream, L.samples, L.n_steps, L.n, L.s_obs, L.s_step, L.s_samp, L.dir,
                       L.dir_s_obs, L.dir_s_step, L.prm, L.out);
  } else {
    hipLaunchKernelGGL((safe_halfspace_kernel<BLOCK, P, LOG_NB, false, GIVEN_H>), grid, block, 0,
                       L.stream, L.samples, L.n_steps, L.n, L.s_obs, L.s_step, L.s_samp, L.dir,
                       L.dir_s_obs, L.dir_s_step, L.prm, L.out);
  }
}

template <bool GIVEN_H>
int dispatch(const Launch& L) {
  if (L.units == 0) return DRCVAR_OK;
  const int p = pick_plan(L.n);
  if (p < 0) return DRCVAR_ERR_UNSUPPORTED;
  const bool vec = (reinterpret_cast<uintptr_t>(L.samples) % 16 == 0) && (L.s_obs % 2 == 0) &&
                   (L.s_step % 2 == 0) && (L.s_samp % 2 == 0);
  (void)hipGetLastError();  // clear stale errors from unrelated work
  switch (p) {
    case 0: launch_plan<64, 2, 7, GIVEN_H>(L, vec); break;
    case 1: launch_plan<128, 4, 8, GIVEN_H>(L, vec); break;
    case 2: launch_plan<256, 4, 9, GIVEN_H>(L, vec); break;
    case 3: launch_plan<256, 8, 10, GIVEN_H>(L, vec); break;
    case 4: launch_plan<256, 16, 11, GIVEN_H>(L, vec); break;
    case 5: launch_plan<512, 16, 12, GIVEN_H>(L, vec); break;
    case 6: launch_plan<1024, 10, 12, GIVEN_H>(L, vec); break;
    case 7: launch_plan<1024, 12, 12, GIVEN_H>(L, vec); break;
    default: launch_plan<1024, 16, 12, GIVEN_H>(L, vec); break;
  }
  return hipGetLastError() == hipSuccess ? DRCVAR_OK : DRCVAR_ERR_LAUNCH;
}

bool params_ok(double rr, double ro, double alpha, double delta, double eps) {
  return std::isfinite(rr) && std::isfinite(ro) && std::isfinite(alpha) && alpha > 0.0 &&
         std::isfinite(delta) && std::isfinite(eps);
}

}  // namespace

extern "C" {

int drcvar_abi_version(void) { return DRCVAR_ABI_VERSION; }

const char* drcvar_strerror(int code) {
  switch (code) {
    case DRCVAR_OK: return "ok";
    case DRCVAR_ERR_INVALID_ARGUMENT: return "invalid argument";
    case DRCVAR_ERR_UNSUPPORTED: return "n_samples exceeds DRCVAR_MAX_SAMPLES";
    case DRCVAR_ERR_LAUNCH: return "HIP kernel launch failed";
    default: return "unknown error";
  }
}

int drcvar_launch_plan(int64_t n_samples, int32_t* threads_per_unit, int32_t* samples_per_thread,
                       int32_t* bins) {
  if (n_samples < 1) return DRCVAR_ERR_INVALID_ARGUMENT;
  const int p = pick_plan(n_samples);
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
  if (n_obstacles < 0 || n_steps < 0 || n_samples < 1) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (!params_ok(robot_radius, obstacle_radius, alpha, delta, epsilon))
    return DRCVAR_ERR_INVALID_ARGUMENT;
  const int64_t units = n_obstacles * n_steps;
  if (units == 0) return DRCVAR_OK;
  if (!samples || !ego_ref_pos || !out || units > 0x7fffffff) return DRCVAR_ERR_INVALID_ARGUMENT;
  Launch L{samples, units, n_steps, n_samples, stride_obstacle, stride_step, stride_sample,
           ego_ref_pos, 0, ego_stride_step,
           Params{robot_radius + obstacle_radius, alpha, delta, epsilon}, out,
           static_cast<hipStream_t>(stream)};
  return dispatch<false>(L);
}

int drcvar_offsets_given_h_f64(const double* samples, int64_t n_units, int64_t n_samples,
                               int64_t stride_unit, int64_t stride_sample, const double* h,
                               int64_t h_stride_unit, double robot_radius, double obstacle_radius,
                               double alpha, double delta, double epsilon, double* out,
                               void* stream) {
  if (n_units < 0 || n_samples < 1) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (!params_ok(robot_radius, obstacle_radius, alpha, delta, epsilon))
    return DRCVAR_ERR_INVALID_ARGUMENT;
  if (n_units == 0) return DRCVAR_OK;
  if (!samples || !h || !out || n_units > 0x7fffffff) return DRCVAR_ERR_INVALID_ARGUMENT;
  Launch L{samples, n_units, 1, n_samples, stride_unit, 0, stride_sample,
           h, h_stride_unit, 0,
           Params{robot_radius + obstacle_radius, alpha, delta, epsilon}, out,
           static_cast<hipStream_t>(stream)};
  return dispatch<true>(L);
}

}  // extern "C"
