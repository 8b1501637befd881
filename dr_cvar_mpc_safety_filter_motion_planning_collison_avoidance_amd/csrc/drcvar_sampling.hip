// drcvar_sampling.hip — obstacle sample trajectories generated in device memory, for gfx950.
//
// Reference: simulation/obstacles.py:43-77 (generate_obstacle_sample_trajectories): for every step
// t >= 1 the N samples are nominal[t] + N(0, noise_cov) (np.random.multivariate_normal), step 0 is
// the nominal start for every sample (:63).  Here every PAIR of samples (p, p + P) of a unit,
// P = ceil(N/2), is one Philox4x32-10 call (counter = (unit * P + p, stream), key = seed): its four
// 32-bit words are two (radius, angle) uniform pairs -> Box-Muller -> L z, written straight into
// the [O, T, N, 2] layout the halfspace kernel streams.  The pair's samples are half a unit apart so
// that each of the two 16-B stores of a wave writes one contiguous 1 KB (pairs of adjacent samples
// made every store instruction half-fill 16 cache lines: 0.76 ms per refill against 0.45 ms for the
// arithmetic alone).
//
// The per-sample arithmetic bounds this kernel, not the 16-B store (round 2: 163 VALU instructions
// per sample, 0.33 of HBM, VALU busy 1.02).  This form (round 3, ~80 VALU per sample in the loop):
//   * one Philox call per two samples (32-bit uniforms: radius up to 6.8 sd, angle resolution
//     2^-32 turn) — half the 20 v_mad_u64_u32 + 20 v_bitop3_b32 per sample; the round keys are
//     bumped in SALU;
//   * log u for u = (x + 1/2) 2^-32 = (2x + 1) 2^-33: frexp, the mantissa's top 9 bits (rounded)
//     pick the nearest of 257 centres c_k, r = m / c_k - 1 by one fma (|r| <= 1/512),
//     log1p(r) to r^6 — instead of a rcp/Newton division and a degree-21 series;
//   * cos / sin of 2 pi w / 2^32: the top 9 bits (rounded) pick the nearest of 512 table angles,
//     the signed remainder |b| <= pi/512 goes through sin b to b^5 and cos b - 1 to b^4, rotated by
//     the table point — instead of a quadrant fold and series to x^15 / x^16;
//   * both tables (12 KB) are copied to LDS per workgroup: a global table load would share vmcnt
//     with the wave's earlier stores, and waiting for it waited for their write acknowledgements
//     (0.678 -> 0.556 ms per C5 refill together with the packed 16-B store below);
//   * sqrt through rsq + Newton (the argument is never denormal);
//   * the series' Horner steps as v_fma_f64 with the coefficient in SGPRs (fma_sc).
// The tables are generated once (scripts/gen_sampler_tables.py, extended precision, exact hex
// literals in drcvar_sampling_tables.inc); the host mirror oracle/philox_sampler.py reads the same
// file.  Accuracy: log within a few ulp, cos / sin within ~2e-16 of extended-precision references
// (tests/test_sampling.py); kernel vs mirror to 1e-14 (FMA contraction only).
// Round 6 (78 -> 67 VALU per sample in the loop): an isotropic covariance l^2 I rides
// in the log (LogScale: the sample is nominal + sqrt(l^2 (-2 log u)) (cos, sin), two fmas); Philox's
// uniform round words are made on the host (PhiloxUniform); workgroups whose pair range lies wholly
// in the unit store with no per-pair test (store_at).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "drcvar_sampling.h"

namespace {

constexpr int kBlock = 256;
// Sample pairs per thread: two per iteration (independent Philox calls for ILP), kPairs in all.
// A thread's work must outlast the wave launch: with 2 pairs per thread the waves lived ~4 k
// cycles, the dispatcher kept only ~1.3 waves per SIMD resident and VALU was busy 52 % of the
// kernel (rocprofv3 counters, profiles/r03/sampler_pmc_pairs2.json); 8 per thread keep the SIMDs fed.
constexpr int kPairs = 8;

#include "drcvar_generator.inc"

// Units [u0, u0 + count) of the global [O, T] grid (u = o T + t); unit u is written at
// out + (o - o0) so + (t - t0) st with (o0, t0) = divmod(u0, T), so a whole [O, T, N, 2] batch
// (u0 = 0, any strides) and a flat shard [count, N, 2] (so = T su, st = su) are the same kernel.
struct SampleArgs {
  const double* nominal;
  int64_t T, N, nom_so, nom_st;
  int64_t u0, count, o0, t0;
  double l00, l10, l11;
  PhiloxUniform pu;
  int zero_first;
  double* out;
  int64_t so, st, sn;
  LogScale lg;
};

// one sample: nominal + L z, written at p.  kPacked (sample stride 2 and every sample 16-B
// aligned, decided once on the host): one 16-B store of a two-double vector — a branch per store
// let the compiler sink the common first double out of both arms and split the 16-B store into two
// 8-B ones.  kNT: nontemporal stores, for batches larger than the 256 MB MALL (the halfspace kernel
// reads them back from HBM anyway): 0.536-0.552 -> 0.531-0.536 ms per C5 refill (lab notebook
// §3c); a cache-sized batch keeps ordinary stores, which its consumer finds in the MALL.
typedef double dbl2 __attribute__((ext_vector_type(2)));
template <bool kPacked, bool kNT>
__device__ __forceinline__ void put_sample(double* p, double x, double y) {
  if constexpr (kPacked) {
    dbl2 v = {x, y};
    if constexpr (kNT)
      __builtin_nontemporal_store(v, reinterpret_cast<dbl2*>(p));
    else
      *reinterpret_cast<dbl2*>(p) = v;
  } else {
    p[0] = x;
    p[1] = y;
  }
}

// The pair of samples of one Philox call (counter g, the unit's nominal point): sample p from the
// call's first (radius, angle) words, sample p + P from its second.  kIso: the covariance is l^2 I
// and the log already carries lam = l^2 (LogScale), so a sample is nominal + radius (cos, sin);
// otherwise nominal + L z as an fma chain (the mirror rounds ny + (l10 z0 + l11 z1): a few ulp apart).
template <bool kIso>
__device__ __forceinline__ void draw_pair(uint64_t g, const SampleArgs& a, double nx, double ny,
                                          const double* s_turn, const double* s_log, double* x0,
                                          double* y0, double* x1, double* y1) {
  const Philox r = philox4x32_10(static_cast<uint32_t>(g), static_cast<uint32_t>(g >> 32), a.pu);
  double c0, sn0, c1, sn1;
  const double rad0 = sqrt_normal(scaled_neg2_log_u32(r.x[0], s_log, a.lg));
  cos_sin_u32(r.x[1], s_turn, &c0, &sn0);
  const double rad1 = sqrt_normal(scaled_neg2_log_u32(r.x[2], s_log, a.lg));
  cos_sin_u32(r.x[3], s_turn, &c1, &sn1);
  if constexpr (kIso) {
    *x0 = fma(rad0, c0, nx);
    *y0 = fma(rad0, sn0, ny);
    *x1 = fma(rad1, c1, nx);
    *y1 = fma(rad1, sn1, ny);
  } else {
    const double z00 = rad0 * c0, z01 = rad0 * sn0, z10 = rad1 * c1, z11 = rad1 * sn1;
    *x0 = fma(a.l00, z00, nx);
    *y0 = fma(a.l10, z00, fma(a.l11, z01, ny));
    *x1 = fma(a.l00, z10, nx);
    *y1 = fma(a.l10, z10, fma(a.l11, z11, ny));
  }
}

// 16-B store at a uniform base (SGPRs) + a 32-bit lane offset: global_store_dwordx4 in its
// saddr form, one v_add per pair for the offset and no 64-bit address arithmetic.  (A buffer-store
// form with the pair's offset in soffset needed no VALU at all, but on gfx950 the VALU that next
// wrote the store's data VGPRs corrupted lanes 12-15 of every 16 of the stored data now and then —
// a store-data hazard the compiler inserts no wait for when soffset is an SGPR;
// scripts/micro/sampler_check.py found it: two refills differed in ~2 400 samples.)
template <bool kNT>
__device__ __forceinline__ void store_at(char* base, uint32_t off, double x, double y) {
  dbl2 v = {x, y};
  dbl2* p = reinterpret_cast<dbl2*>(base + off);
  if constexpr (kNT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

template <bool kPacked, bool kNT, bool kIso>
__global__ __launch_bounds__(kBlock) void sample_kernel(SampleArgs a) {
  // The tables are read from LDS, not from global memory: a global table load is counted by
  // vmcnt together with the wave's earlier sample stores, and waiting for the load (in order)
  // would wait for those stores' write acknowledgements too, serialising arithmetic and stores.
  __shared__ double s_turn[kTurnLen], s_log[2 * kLogIdx];
  load_generator_tables(s_turn, s_log, kBlock, a.lg.lam);
  __syncthreads();
  const int64_t pairs = (a.N + 1) >> 1;  // Philox calls per unit
  const int64_t blk0 = static_cast<int64_t>(blockIdx.x) * (kBlock * kPairs);  // this row's first pair
  // Every pair of the workgroup's range is in the unit and has both samples (an odd N's last pair
  // has only the first): the packed layout then stores with no per-pair test and no 64-bit
  // address arithmetic (store_at).  The other workgroups take the checked loop.
  const bool full = kPacked && blk0 + kBlock * kPairs <= pairs &&
                    ((a.N & 1) == 0 || blk0 + kBlock * kPairs < pairs);
  for (int64_t k = blockIdx.y; k < a.count; k += gridDim.y) {
    const int64_t u = a.u0 + k;
    const int64_t o = u / a.T, t = u - o * a.T;
    const double* nom = a.nominal + o * a.nom_so + t * a.nom_st;
    const double nx = nom[0], ny = nom[1];
    double* dst = a.out + (o - a.o0) * a.so + (t - a.t0) * a.st;
    const int64_t sn = kPacked ? 2 : a.sn;
    const int64_t base = blk0 + threadIdx.x;
    if (a.zero_first && t == 0) {  // the noise-free first step: every sample is the nominal point
#pragma unroll 1
      for (int q = 0; q < kPairs; ++q) {
        const int64_t pidx = base + q * kBlock;
        if (pidx >= pairs) break;
        put_sample<kPacked, kNT>(dst + pidx * sn, nx, ny);
        if (pidx + pairs < a.N) put_sample<kPacked, kNT>(dst + (pidx + pairs) * sn, nx, ny);
      }
      continue;
    }
    const uint64_t g0 = static_cast<uint64_t>(u) * static_cast<uint64_t>(pairs) + static_cast<uint64_t>(base);
    if (full) {
      // first samples at dst + 16 (blk0 + lane + q kBlock) B, second ones 16 pairs B further
      char* const b0 = reinterpret_cast<char*>(dst + blk0 * 2);
      char* const b1 = reinterpret_cast<char*>(dst + (blk0 + pairs) * 2);
      const uint32_t voff = threadIdx.x * 16u;
#pragma unroll 2
      for (int q = 0; q < kPairs; ++q) {
        double x0, y0, x1, y1;
        draw_pair<kIso>(g0 + static_cast<uint64_t>(q * kBlock), a, nx, ny, s_turn, s_log, &x0, &y0, &x1, &y1);
        const uint32_t off = voff + static_cast<uint32_t>(q * kBlock * 16);
        store_at<kNT>(b0, off, x0, y0);
        store_at<kNT>(b1, off, x1, y1);
      }
      continue;
    }
#pragma unroll 2
    for (int q = 0; q < kPairs; ++q) {
      const int64_t pidx = base + q * kBlock;
      if (pidx >= pairs) break;
      double x0, y0, x1, y1;
      draw_pair<kIso>(g0 + static_cast<uint64_t>(q * kBlock), a, nx, ny, s_turn, s_log, &x0, &y0, &x1, &y1);
      put_sample<kPacked, kNT>(dst + pidx * sn, x0, y0);
      if (pidx + pairs < a.N) put_sample<kPacked, kNT>(dst + (pidx + pairs) * sn, x1, y1);
    }
  }
}

// LogScale for lam (see drcvar_generator.inc): the Horner coefficients of -P/2 in r2
// (1/192, 1/80, 1/32, 1/12, 1/4) times lam, and -2 lam ln 2 split into a 46-bit head (e * eh exact
// for |e| <= 33) and a tail, from an extended-precision product.
LogScale make_log_scale(double lam) {
  LogScale c{};
  c.lam = lam;
  c.q0 = lam * (1.0 / 192.0);
  c.q1 = lam * (1.0 / 80.0);
  c.q2 = lam * (1.0 / 32.0);
  c.q3 = lam * (1.0 / 12.0);
  c.q4 = lam * 0.25;
  const long double e2 = -2.0L * static_cast<long double>(lam) * 0.693147180559945309417232121458176568L;
  double eh = static_cast<double>(e2);
  uint64_t bits;
  std::memcpy(&bits, &eh, sizeof bits);
  bits &= ~uint64_t{0x7f};  // 53 - 7 = 46 significant bits
  std::memcpy(&eh, &bits, sizeof bits);
  c.eh = eh;
  c.el = static_cast<double>(e2 - static_cast<long double>(eh));
  return c;
}

int launch_samples(const double* nominal, int64_t n_obstacles, int64_t n_steps, int64_t nom_so,
                   int64_t nom_st, int64_t u0, int64_t count, int64_t n_samples, double l00,
                   double l10, double l11, uint64_t seed, uint64_t stream_offset,
                   int32_t zero_first_step, double* out, int64_t so, int64_t st, int64_t sn,
                   void* stream) {
  if (n_obstacles < 0 || n_steps < 0 || n_samples < 0 || u0 < 0 || count < 0)
    return DRCVAR_ERR_INVALID_ARGUMENT;
  if (n_samples > (int64_t{1} << 40) || n_obstacles > (int64_t{1} << 40) ||
      n_steps > (int64_t{1} << 40) || n_obstacles * n_steps > (int64_t{1} << 40))
    return DRCVAR_ERR_UNSUPPORTED;
  const int64_t units = n_obstacles * n_steps;
  if (u0 > units || count > units - u0) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (count == 0 || n_samples == 0) return DRCVAR_OK;
  if (!nominal || !out) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (!(l00 == l00) || !(l10 == l10) || !(l11 == l11)) return DRCVAR_ERR_INVALID_ARGUMENT;
  SampleArgs a{};
  a.nominal = nominal;
  a.T = n_steps;
  a.N = n_samples;
  a.nom_so = nom_so;
  a.nom_st = nom_st;
  a.u0 = u0;
  a.count = count;
  a.o0 = u0 / n_steps;
  a.t0 = u0 - a.o0 * n_steps;
  a.l00 = l00;
  a.l10 = l10;
  a.l11 = l11;
  a.pu = make_philox_uniform(static_cast<uint32_t>(stream_offset),
                             static_cast<uint32_t>(stream_offset >> 32), static_cast<uint32_t>(seed),
                             static_cast<uint32_t>(seed >> 32));
  a.zero_first = zero_first_step != 0;
  a.out = out;
  a.so = so;
  a.st = st;
  a.sn = sn;
  // the isotropic form (covariance l^2 I, l > 0, lam = l^2 in a range where the scaled log stays
  // normal and its coefficients finite): lam rides in the log, no L z
  const double lam = l00 * l00;
  const bool iso = l10 == 0.0 && l00 == l11 && l00 > 0.0 && std::isfinite(l00) &&
                   lam >= 0x1.0p-200 && lam <= 0x1.0p200;
  a.lg = make_log_scale(iso ? lam : 1.0);
  const int64_t per_block = int64_t{kBlock} * kPairs;  // pairs per workgroup
  const int64_t gx = ((n_samples + 1) / 2 + per_block - 1) / per_block;
  if (gx > 0x7fffffffLL) return DRCVAR_ERR_UNSUPPORTED;
  // Workgroup rows loop over units (k += gridDim.y): up to four units per row once the grid has
  // >= 8192 workgroups, so the per-workgroup LDS table copy (~4 % of the VALU work at one unit per
  // row) is amortised; small batches keep one unit per row to fill the device.
  int64_t rows = std::max((count + 3) / 4, (int64_t{8192} + gx - 1) / gx);
  rows = std::min(rows, std::min(count, int64_t{65535}));
  const unsigned gy = static_cast<unsigned>(rows);
  (void)hipGetLastError();
  const bool packed = sn == 2 && (reinterpret_cast<uintptr_t>(out) & 15) == 0 && (so & 1) == 0 &&
                      (st & 1) == 0;
  constexpr int64_t kMallBytes = int64_t{256} << 20;
  const bool nt = packed && count * n_samples * 16 > kMallBytes;
  const dim3 grid(static_cast<unsigned>(gx), gy);
  const hipStream_t s = static_cast<hipStream_t>(stream);
  if (nt && iso)
    hipLaunchKernelGGL((sample_kernel<true, true, true>), grid, dim3(kBlock), 0, s, a);
  else if (nt)
    hipLaunchKernelGGL((sample_kernel<true, true, false>), grid, dim3(kBlock), 0, s, a);
  else if (packed && iso)
    hipLaunchKernelGGL((sample_kernel<true, false, true>), grid, dim3(kBlock), 0, s, a);
  else if (packed)
    hipLaunchKernelGGL((sample_kernel<true, false, false>), grid, dim3(kBlock), 0, s, a);
  else if (iso)
    hipLaunchKernelGGL((sample_kernel<false, false, true>), grid, dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((sample_kernel<false, false, false>), grid, dim3(kBlock), 0, s, a);
  return hipGetLastError() == hipSuccess ? DRCVAR_OK : DRCVAR_ERR_LAUNCH;
}

}  // namespace

extern "C" int drcvar_sample_trajectories_f64(const double* nominal, int64_t n_obstacles,
                                              int64_t n_steps, int64_t nom_so, int64_t nom_st,
                                              int64_t n_samples, double l00, double l10, double l11,
                                              uint64_t seed, uint64_t stream_offset,
                                              int32_t zero_first_step, double* out, int64_t so,
                                              int64_t st, int64_t sn, void* stream) {
  if (n_obstacles < 0 || n_steps < 0) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (n_obstacles > (int64_t{1} << 40) || n_steps > (int64_t{1} << 40)) return DRCVAR_ERR_UNSUPPORTED;
  return launch_samples(nominal, n_obstacles, n_steps, nom_so, nom_st, 0, n_obstacles * n_steps,
                        n_samples, l00, l10, l11, seed, stream_offset, zero_first_step, out, so, st,
                        sn, stream);
}

extern "C" int drcvar_sample_units_f64(const double* nominal, int64_t n_obstacles, int64_t n_steps,
                                       int64_t nom_so, int64_t nom_st, int64_t unit_begin,
                                       int64_t unit_count, int64_t n_samples, double l00,
                                       double l10, double l11, uint64_t seed,
                                       uint64_t stream_offset, int32_t zero_first_step,
                                       double* out, int64_t su, int64_t sn, void* stream) {
  if (n_steps <= 0 && unit_count > 0) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (n_steps > (int64_t{1} << 40) || su > (int64_t{1} << 40)) return DRCVAR_ERR_UNSUPPORTED;
  // (o - o0) T su + (t - t0) su = (u - u0) su
  return launch_samples(nominal, n_obstacles, n_steps, nom_so, nom_st, unit_begin, unit_count,
                        n_samples, l00, l10, l11, seed, stream_offset, zero_first_step, out,
                        n_steps * su, su, sn, stream);
}
