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

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "drcvar_sampling.h"

namespace {

constexpr int kBlock = 256;
// Sample pairs per thread: two per iteration (independent Philox calls for ILP), kPairs in all.
// A thread's work must outlast the wave launch: with 2 pairs per thread the waves lived ~4 k
// cycles, the dispatcher kept only ~1.3 waves per SIMD resident and VALU was busy 52 % of the
// kernel (rocprofv3 counters, profiles/r03/sampler_pmc_pairs2.json); 8 per thread keep the SIMDs fed.
constexpr int kPairs = 8;

#include "drcvar_sampling_tables.inc"

struct Philox {
  uint32_t x[4];
};

__device__ __forceinline__ Philox philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                uint32_t k0, uint32_t k1) {
  constexpr uint64_t kM0 = 0xD2511F53u, kM1 = 0xCD9E8D57u;
  constexpr uint32_t kW0 = 0x9E3779B9u, kW1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = kM0 * c0, p1 = kM1 * c2;  // one v_mad_u64_u32 each
    uint32_t n0, n2;  // hi(p1) ^ c1 ^ k0, hi(p0) ^ c3 ^ k1 (the key words are uniform: SGPRs)
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n0) : "v"(static_cast<uint32_t>(p1 >> 32)), "v"(c1), "s"(k0));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n2) : "v"(static_cast<uint32_t>(p0 >> 32)), "v"(c3), "s"(k1));
    c0 = n0;
    c1 = static_cast<uint32_t>(p1);
    c2 = n2;
    c3 = static_cast<uint32_t>(p0);
    // The key schedule is bumped in SALU each round (volatile: otherwise all twenty round keys are
    // hoisted out of the sample loop, spilled to VGPR lanes and read back with one v_readlane per
    // use — VALU work in a VALU-bound kernel).
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(k0) : "s"(kW0) : "scc");
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(k1) : "s"(kW1) : "scc");
  }
  return Philox{{c0, c1, c2, c3}};
}

// fma with a uniform third operand held in SGPRs (the polynomial coefficients): as v_fma_f64 with
// an SGPR source instead of the compiler's v_mov_b64 of a VGPR-held coefficient + v_fmac_f64 —
// one VALU instruction per Horner step instead of two.  Same IEEE fma, same bits.
__device__ __forceinline__ double fma_sc(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}

// -2 log u for the uniform u = (x + 1/2) 2^-32 in the open interval (0, 1) of a 32-bit word (at
// most 33 significant bits: exact, in [2^-33, 1 - 2^-33], never 0 or 1).  It is formed as
// w = 2x + 1 (one fma with inline constants, exact) and u = w 2^-33, folded into the exponent.
// u = m 2^e, m in [1/2, 1); the top 9 mantissa bits, rounded, pick the nearest centre
// c_k = 1/2 + k/512 (k = 0..256; c_256 = 1 exactly, so log u keeps its relative accuracy as u -> 1);
// r = m (1/c_k) - 1 (|r| <= 1/512 + 2^-52); log m = log1p(r) - log(1/c_k),
// log1p(r) = r + r^2 P(r), P to r^4 (the next term, r^7 / 7, is below 2^-56 of r).
// The factor -2 of Box-Muller is folded in exactly: the LDS table holds -2/c_k and 2 log(1/c_k)
// (indexed by the 9 bits themselves, each centre stored for both of its indices), the fma gives
// r2 = -2r, the Horner coefficients are those of P scaled by powers of two so that the sum is
// -P/2 in r2, and -2 log1p(r) = r2 + r2^2 (-P/2).  Every step is the unscaled step times a power
// of two, so the result is bitwise -2 times the unscaled evaluation (what the host mirror,
// oracle/philox_sampler.py, computes) — one multiply less.
__device__ __forceinline__ double neg2_log_u32(uint32_t x, const double* log_t) {
  const double w = fma(static_cast<double>(x), 2.0, 1.0);
  const double m = __builtin_amdgcn_frexp_mant(w);
  const int e = __builtin_amdgcn_frexp_exp(w) - 33;
  const uint32_t idx = __builtin_amdgcn_ubfe(static_cast<uint32_t>(__double2hiint(m)), 11, 9);
  const double ninv2 = log_t[2 * idx], log_inv2 = log_t[2 * idx + 1];  // -2/c_k, 2 log(1/c_k)
  const double r2 = fma(m, ninv2, 2.0);                                 // -2 r
  double q = (-1.0 / 6.0) * (-1.0 / 32.0);
  q = fma_sc(q, r2, (1.0 / 5.0) * (1.0 / 16.0));
  q = fma_sc(q, r2, (-1.0 / 4.0) * (-1.0 / 8.0));
  q = fma_sc(q, r2, (1.0 / 3.0) * (1.0 / 4.0));
  q = fma_sc(q, r2, (-1.0 / 2.0) * (-1.0 / 2.0));                     // -P(r) / 2
  const double m2log1p = fma(r2 * r2, q, r2);                           // -2 log1p(r)
  constexpr double kLn2Hi = 0x1.62e42fefa3800p-1, kLn2Lo = 0x1.ef35793c76730p-45;
  const double de = static_cast<double>(e);
  return fma(de, -2.0 * kLn2Hi, fma(de, -2.0 * kLn2Lo, log_inv2 + m2log1p));
}

// sqrt(-2 log u).  The argument is >= 2^-33 ln 4 > 0, never denormal, so rsq + two Newton-Raphson
// steps (Goldschmidt form) replace the library sqrt and its rescaling.
__device__ __forceinline__ double box_muller_radius(uint32_t x, const double* log_t) {
  const double y = neg2_log_u32(x, log_t);
  const double rs = __builtin_amdgcn_rsq(y);
  double h = 0.5 * rs, r = y * rs;
  const double e = fma(-r, h, 0.5);
  r = fma(r, e, r);
  h = fma(h, e, h);
  return fma(fma(-r, r, y), h, r);
}

// (cos, sin)(2 pi w / 2^32): table point k = round(w / 2^23) mod 512 (32-bit wrap-around), signed
// remainder rem = w - k 2^23 in [-2^22, 2^22), b = 2 pi rem / 2^32 in [-pi/512, pi/512);
// sin b = b + b^3 (-1/6 + b^2/120) (next term b^7/5040: 1e-17 of b), cos b - 1 = b^2 (-1/2 + b^2/24)
// (next term b^6/720 < 8e-17), and (cos, sin)(a + b) = (C (1 + cm1) - S sb, S (1 + cm1) + C sb)
// with (C, S) = kTurn[k].
__device__ __forceinline__ void cos_sin_u32(uint32_t w, const double* turn, double* cs, double* sn) {
  const uint32_t k = (w + (1u << 22)) >> 23;
  const int32_t rem = __builtin_amdgcn_sbfe(static_cast<int32_t>(w), 0, 23);  // = w - k 2^23
  constexpr double kTurn32 = 6.28318530717958647692 * 0x1.0p-32;
  const double b = static_cast<double>(rem) * kTurn32;
  const double z = b * b;
  const double ps = fma_sc(z, 1.0 / 120.0, -1.0 / 6.0);
  const double sb = fma(b * z, ps, b);
  const double pc = fma_sc(z, 1.0 / 24.0, -0.5);
  const double cm1 = z * pc;
  const double C = turn[2 * k], S = turn[2 * k + 1];
  *cs = fma(C, cm1, fma(-S, sb, C));
  *sn = fma(S, cm1, fma(C, sb, S));
}

// Units [u0, u0 + count) of the global [O, T] grid (u = o T + t); unit u is written at
// out + (o - o0) so + (t - t0) st with (o0, t0) = divmod(u0, T), so a whole [O, T, N, 2] batch
// (u0 = 0, any strides) and a flat shard [count, N, 2] (so = T su, st = su) are the same kernel.
struct SampleArgs {
  const double* nominal;
  int64_t T, N, nom_so, nom_st;
  int64_t u0, count, o0, t0;
  double l00, l10, l11;
  uint32_t k0, k1, s0, s1;
  int zero_first;
  double* out;
  int64_t so, st, sn;
};

// one sample: nominal + L z, written at p.  kPacked (sample stride 2 and every sample 16-B
// aligned, decided once on the host): one 16-B store of a two-double vector — a branch per store
// let the compiler sink the common first double out of both arms and split the 16-B store into two
// 8-B ones.  kNT: nontemporal stores, for batches larger than the 256 MB MALL (the halfspace kernel
// reads them back from HBM anyway): 0.536-0.552 -> 0.531-0.536 ms per C5 refill
// (scripts/micro/gpu_samp_nt.sh); a cache-sized batch keeps ordinary stores, which its consumer
// finds in the MALL.
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

template <bool kPacked, bool kNT>
__global__ __launch_bounds__(kBlock) void sample_kernel(SampleArgs a) {
  // The tables are read from LDS, not from global memory: a global table load is counted by
  // vmcnt together with the wave's earlier sample stores, and waiting for the load (in order)
  // would wait for those stores' write acknowledgements too, serialising arithmetic and stores.
  constexpr int kTurnLen = sizeof(kTurn) / sizeof(double);
  constexpr int kLogIdx = 2 * (sizeof(kLogT) / sizeof(double) / 2 - 1);  // 512 nine-bit indices
  __shared__ double s_turn[kTurnLen], s_log[2 * kLogIdx];
  for (int i = threadIdx.x; i < kTurnLen + kLogIdx; i += kBlock) {
    if (i < kTurnLen) {
      s_turn[i] = kTurn[i];
    } else {  // index j -> centre (j + 1) / 2, scaled by -2 (exact)
      const int j = i - kTurnLen, c = (j + 1) >> 1;
      s_log[2 * j] = -2.0 * kLogT[2 * c];
      s_log[2 * j + 1] = -2.0 * kLogT[2 * c + 1];
    }
  }
  __syncthreads();
  const int64_t pairs = (a.N + 1) >> 1;  // Philox calls per unit
  for (int64_t k = blockIdx.y; k < a.count; k += gridDim.y) {
    const int64_t u = a.u0 + k;
    const int64_t o = u / a.T, t = u - o * a.T;
    const double* nom = a.nominal + o * a.nom_so + t * a.nom_st;
    const double nx = nom[0], ny = nom[1];
    double* dst = a.out + (o - a.o0) * a.so + (t - a.t0) * a.st;
    const int64_t sn = kPacked ? 2 : a.sn;
    const int64_t base = (static_cast<int64_t>(blockIdx.x) * kBlock * kPairs) + threadIdx.x;
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
#pragma unroll 2
    for (int q = 0; q < kPairs; ++q) {
      const int64_t pidx = base + q * kBlock;
      if (pidx >= pairs) break;
      const uint64_t g = g0 + static_cast<uint64_t>(q * kBlock);
      const Philox r = philox4x32_10(static_cast<uint32_t>(g), static_cast<uint32_t>(g >> 32),
                                     a.s0, a.s1, a.k0, a.k1);
      double c0, s0, c1, s1;
      const double rad0 = box_muller_radius(r.x[0], s_log);
      cos_sin_u32(r.x[1], s_turn, &c0, &s0);
      const double rad1 = box_muller_radius(r.x[2], s_log);
      cos_sin_u32(r.x[3], s_turn, &c1, &s1);
      const double z00 = rad0 * c0, z01 = rad0 * s0, z10 = rad1 * c1, z11 = rad1 * s1;
      // nominal + L z as an fma chain (the mirror rounds ny + (l10 z0 + l11 z1): a few ulp apart)
      const double x0 = fma(a.l00, z00, nx);
      const double y0 = fma(a.l10, z00, fma(a.l11, z01, ny));
      const double x1 = fma(a.l00, z10, nx);
      const double y1 = fma(a.l10, z10, fma(a.l11, z11, ny));
#ifdef DRCVAR_SAMPLER_NO_STORE  // diagnostic: the arithmetic alone (stores only for a sentinel)
      if (x0 + y0 + x1 + y1 == 1234.5) put_sample<kPacked, kNT>(dst + pidx * sn, x0, y0);
#else
      put_sample<kPacked, kNT>(dst + pidx * sn, x0, y0);
      if (pidx + pairs < a.N) put_sample<kPacked, kNT>(dst + (pidx + pairs) * sn, x1, y1);
#endif
    }
  }
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
  a.k0 = static_cast<uint32_t>(seed);
  a.k1 = static_cast<uint32_t>(seed >> 32);
  a.s0 = static_cast<uint32_t>(stream_offset);
  a.s1 = static_cast<uint32_t>(stream_offset >> 32);
  a.zero_first = zero_first_step != 0;
  a.out = out;
  a.so = so;
  a.st = st;
  a.sn = sn;
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
  if (nt)
    hipLaunchKernelGGL((sample_kernel<true, true>), grid, dim3(kBlock), 0, s, a);
  else if (packed)
    hipLaunchKernelGGL((sample_kernel<true, false>), grid, dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((sample_kernel<false, false>), grid, dim3(kBlock), 0, s, a);
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
