// drcvar_sampling.hip — obstacle sample trajectories generated in device memory, for gfx950.
//
// Reference: simulation/obstacles.py:43-77 (generate_obstacle_sample_trajectories): for every step
// t >= 1 the N samples are nominal[t] + N(0, noise_cov) (np.random.multivariate_normal), step 0 is
// the nominal start for every sample (:63).  Here every sample is one Philox4x32-10 call (counter =
// global sample index and stream, key = seed) -> two 53-bit uniforms -> Box-Muller -> L z, written
// straight into the [O, T, N, 2] layout the halfspace kernel streams.
//
// The per-sample arithmetic is what bounds this kernel, not the 16-B store: with the library's
// fp64 log (98 VALU instructions) and sincospi (71) plus Philox's 40 quarter-rate 32-bit
// multiplies it ran at 0.21 of HBM.  So the Box-Muller pieces are written for this input domain:
//   * Philox rounds use one v_mad_u64_u32 per product (the 64-bit product gives both halves) and
//     one v_bitop3_b32 (3-input XOR, truth table 0x96) per output word;
//   * log u1 for u1 in (0, 1): frexp, f = m - 1 with m in [sqrt(1/2), sqrt(2)), s = f / (2 + f),
//     log(1 + f) = 2 atanh(s) as a degree-21 odd series in s (|s| <= 0.1716: truncation < 1e-17);
//   * cos/sin of 2 pi u2 straight from the 64 raw bits of u2: the top two bits (rounded) are the
//     quadrant, the signed remainder |x| <= pi/4 goes through Taylor series to x^15 / x^16;
//   * sqrt through rsq + Newton (the argument is never denormal);
//   * the series' Horner steps as v_fma_f64 with the coefficient in SGPRs (fma_sc): the compiler
//     otherwise copied a VGPR-held coefficient into the accumulator before each v_fmac_f64
//     (190 -> 163 VALU instructions per sample, 0.838 -> 0.775 ms per 128 M samples, same bits);
// All four agree with the libm functions to a few ulp (tests/test_sampling.py checks the host
// mirror oracle/philox_sampler.py against numpy's log/sin/cos and the kernel against the mirror).

#include <hip/hip_runtime.h>

#include <cstdint>

#include "drcvar_sampling.h"

namespace {

constexpr int kBlock = 256;
constexpr int kPerThread = 4;  // samples per thread (independent Philox calls for ILP)

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
    k0 += kW0;
    k1 += kW1;
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

// Uniform in the open interval (0, 1) from the top 52 bits: (v + 1/2) 2^-52 needs 53 significant
// bits, so it is exact, and lies in [2^-53, 1 - 2^-53].  (A 53-bit v would round v + 1/2 up to
// 2^53 for v = 2^53 - 1, i.e. u = 1 and log u = 0 -> rsq(-0) = -inf -> a NaN sample.)
__device__ __forceinline__ double uniform52(uint32_t hi, uint32_t lo) {
  const uint64_t v = (static_cast<uint64_t>(hi) << 32 | lo) >> 12;
  return (static_cast<double>(v) + 0.5) * 0x1.0p-52;
}

// log(x) for 0 < x <= 1 (normal).  x = m 2^e with m in [sqrt(1/2), sqrt(2)); f = m - 1 is exact;
// log m = 2 atanh(s), s = f / (2 + f), summed as 2 s + s^3 P(s^2) with P the atanh series to s^21.
__device__ __forceinline__ double log_unit(double x) {
  double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1)
  int e = __builtin_amdgcn_frexp_exp(x);
  const bool lo = m < 0.70710678118654752440;
  m = lo ? m + m : m;
  e = lo ? e - 1 : e;
  const double f = m - 1.0;
  const double d = 2.0 + f;  // in [1.7, 2.5]: a plain reciprocal + Newton division is exact enough
  double r = __builtin_amdgcn_rcp(d);
  r = fma(fma(-d, r, 1.0), r, r);
  r = fma(fma(-d, r, 1.0), r, r);
  double sq = f * r;
  sq = fma(fma(-d, sq, f), r, sq);
  const double z = sq * sq;
  double p = 2.0 / 21.0;
  p = fma_sc(p, z, 2.0 / 19.0);
  p = fma_sc(p, z, 2.0 / 17.0);
  p = fma_sc(p, z, 2.0 / 15.0);
  p = fma_sc(p, z, 2.0 / 13.0);
  p = fma_sc(p, z, 2.0 / 11.0);
  p = fma_sc(p, z, 2.0 / 9.0);
  p = fma_sc(p, z, 2.0 / 7.0);
  p = fma_sc(p, z, 2.0 / 5.0);
  p = fma_sc(p, z, 2.0 / 3.0);
  const double logm = fma(sq * z, p, sq + sq);
  constexpr double kLn2Hi = 0x1.62e42fefa3800p-1, kLn2Lo = 0x1.ef35793c76730p-45;
  const double de = static_cast<double>(e);
  return fma(de, kLn2Hi, fma(de, kLn2Lo, logm));
}

// sqrt(-2 log u1).  The argument is >= 2^-52 (u1 <= 1 - 2^-53), never denormal, so rsq + two
// Newton-Raphson steps (Goldschmidt form) replace the library sqrt and its rescaling.
__device__ __forceinline__ double box_muller_radius(double u1) {
  const double y = -2.0 * log_unit(u1);
  double h = 0.5 * __builtin_amdgcn_rsq(y), r = y * (h + h);
  const double e = fma(-r, h, 0.5);
  r = fma(r, e, r);
  h = fma(h, e, h);
  return fma(fma(-r, r, y), h, r);
}

// (cos, sin)(2 pi w / 2^64): quadrant q = round(w / 2^62) mod 4, remainder x = 2 pi (w - q 2^62) /
// 2^64 in [-pi/4, pi/4) (53 significant bits of it kept), Taylor series to x^15 (sin) / x^16 (cos).
__device__ __forceinline__ void cos_sin_turn(uint32_t whi, uint32_t wlo, double* cs, double* sn) {
  const uint64_t w = static_cast<uint64_t>(whi) << 32 | wlo;
  const uint32_t q = static_cast<uint32_t>((w + (uint64_t{1} << 61)) >> 62);
  const int64_t rem = static_cast<int64_t>(w - (static_cast<uint64_t>(q) << 62)) >> 11;
  constexpr double kTurn = 6.28318530717958647692 * 0x1.0p-53;
  const double x = static_cast<double>(rem) * kTurn;
  const double z = x * x;
  double ps = -1.0 / 1307674368000.0;
  ps = fma_sc(ps, z, 1.0 / 6227020800.0);
  ps = fma_sc(ps, z, -1.0 / 39916800.0);
  ps = fma_sc(ps, z, 1.0 / 362880.0);
  ps = fma_sc(ps, z, -1.0 / 5040.0);
  ps = fma_sc(ps, z, 1.0 / 120.0);
  ps = fma_sc(ps, z, -1.0 / 6.0);
  const double s = fma(x * z, ps, x);
  double pc = 1.0 / 20922789888000.0;
  pc = fma_sc(pc, z, -1.0 / 87178291200.0);
  pc = fma_sc(pc, z, 1.0 / 479001600.0);
  pc = fma_sc(pc, z, -1.0 / 3628800.0);
  pc = fma_sc(pc, z, 1.0 / 40320.0);
  pc = fma_sc(pc, z, -1.0 / 720.0);
  pc = fma_sc(pc, z, 1.0 / 24.0);
  pc = fma_sc(pc, z, -0.5);
  const double c = fma(z, pc, 1.0);
  // theta = q pi/2 + x: q=0 (c, s), 1 (-s, c), 2 (-c, -s), 3 (s, -c)
  const bool swap = q & 1;
  const double a = swap ? s : c, b = swap ? c : s;
  *cs = ((q + 1) & 2) ? -a : a;
  *sn = (q & 2) ? -b : b;
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

__global__ __launch_bounds__(kBlock) void sample_kernel(SampleArgs a) {
  for (int64_t k = blockIdx.y; k < a.count; k += gridDim.y) {
    const int64_t u = a.u0 + k;
    const int64_t o = u / a.T, t = u - o * a.T;
    const double* nom = a.nominal + o * a.nom_so + t * a.nom_st;
    const double nx = nom[0], ny = nom[1];
    double* dst = a.out + (o - a.o0) * a.so + (t - a.t0) * a.st;
    const bool noise = !(a.zero_first && t == 0);
    const int64_t base = (static_cast<int64_t>(blockIdx.x) * kBlock * kPerThread) + threadIdx.x;
#pragma unroll
    for (int q = 0; q < kPerThread; ++q) {
      const int64_t i = base + q * kBlock;
      if (i >= a.N) break;
      double x = nx, y = ny;
      if (noise) {
        const uint64_t g = static_cast<uint64_t>(u) * static_cast<uint64_t>(a.N) + static_cast<uint64_t>(i);
        const Philox r = philox4x32_10(static_cast<uint32_t>(g), static_cast<uint32_t>(g >> 32),
                                       a.s0, a.s1, a.k0, a.k1);
        const double rad = box_muller_radius(uniform52(r.x[0], r.x[1]));
        double sn, cs;
        cos_sin_turn(r.x[2], r.x[3], &cs, &sn);
        const double z0 = rad * cs, z1 = rad * sn;
        x = nx + a.l00 * z0;
        y = ny + (a.l10 * z0 + a.l11 * z1);
      }
      double* p = dst + i * a.sn;
      if (a.sn == 2 && (reinterpret_cast<uintptr_t>(p) & 15) == 0) {
        *reinterpret_cast<double2*>(p) = make_double2(x, y);
      } else {
        p[0] = x;
        p[1] = y;
      }
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
  const int64_t per_block = int64_t{kBlock} * kPerThread;
  const int64_t gx = (n_samples + per_block - 1) / per_block;
  if (gx > 0x7fffffffLL) return DRCVAR_ERR_UNSUPPORTED;
  const unsigned gy = static_cast<unsigned>(count < 65535 ? count : 65535);
  (void)hipGetLastError();
  hipLaunchKernelGGL(sample_kernel, dim3(static_cast<unsigned>(gx), gy), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), a);
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
