// drcvar_sampling.hip — obstacle sample trajectories generated in device memory, for gfx950.
//
// Reference: simulation/obstacles.py:43-77 (generate_obstacle_sample_trajectories): for every step
// t >= 1 the N samples are nominal[t] + N(0, noise_cov) (np.random.multivariate_normal), step 0 is
// the nominal start for every sample (:63).  Here every sample is one Philox4x32-10 call (counter =
// global sample index and stream, key = seed) -> two 53-bit uniforms -> Box-Muller -> L z, written
// straight into the [O, T, N, 2] layout the halfspace kernel streams.  Bandwidth-bound on the
// 16-B store per sample (the fp64 log / sincospi per sample sit under the store time).

#include <hip/hip_runtime.h>

#include <cstdint>

#include "drcvar_sampling.h"

namespace {

constexpr int kBlock = 256;
constexpr int kPerThread = 2;  // samples per thread (independent Philox calls for ILP)

struct Philox {
  uint32_t x[4];
};

__device__ __forceinline__ Philox philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                uint32_t k0, uint32_t k1) {
  constexpr uint32_t kM0 = 0xD2511F53u, kM1 = 0xCD9E8D57u;
  constexpr uint32_t kW0 = 0x9E3779B9u, kW1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(kM0, c0), lo0 = kM0 * c0;
    const uint32_t hi1 = __umulhi(kM1, c2), lo1 = kM1 * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += kW0;
    k1 += kW1;
  }
  return Philox{{c0, c1, c2, c3}};
}

// 53-bit uniform in the open interval (0, 1)
__device__ __forceinline__ double uniform53(uint32_t hi, uint32_t lo) {
  const uint64_t v = (static_cast<uint64_t>(hi) << 32 | lo) >> 11;
  return (static_cast<double>(v) + 0.5) * 0x1.0p-53;
}

struct SampleArgs {
  const double* nominal;
  int64_t O, T, N, nom_so, nom_st;
  double l00, l10, l11;
  uint32_t k0, k1, s0, s1;
  int zero_first;
  double* out;
  int64_t so, st, sn;
};

__global__ __launch_bounds__(kBlock) void sample_kernel(SampleArgs a) {
  const int64_t units = a.O * a.T;
  for (int64_t u = blockIdx.y; u < units; u += gridDim.y) {
    const int64_t o = u / a.T, t = u - o * a.T;
    const double* nom = a.nominal + o * a.nom_so + t * a.nom_st;
    const double nx = nom[0], ny = nom[1];
    double* dst = a.out + o * a.so + t * a.st;
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
        const double u1 = uniform53(r.x[0], r.x[1]);
        const double u2 = uniform53(r.x[2], r.x[3]);
        const double rad = sqrt(-2.0 * log(u1));
        double sn, cs;
        sincospi(2.0 * u2, &sn, &cs);
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

}  // namespace

extern "C" int drcvar_sample_trajectories_f64(const double* nominal, int64_t n_obstacles,
                                              int64_t n_steps, int64_t nom_so, int64_t nom_st,
                                              int64_t n_samples, double l00, double l10, double l11,
                                              uint64_t seed, uint64_t stream_offset,
                                              int32_t zero_first_step, double* out, int64_t so,
                                              int64_t st, int64_t sn, void* stream) {
  if (n_obstacles < 0 || n_steps < 0 || n_samples < 0) return DRCVAR_ERR_INVALID_ARGUMENT;
  const int64_t units = n_obstacles * n_steps;
  if (units == 0 || n_samples == 0) return DRCVAR_OK;
  if (!nominal || !out) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (!(l00 == l00) || !(l10 == l10) || !(l11 == l11)) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (n_samples > (int64_t{1} << 40) || units > (int64_t{1} << 40)) return DRCVAR_ERR_UNSUPPORTED;
  SampleArgs a{};
  a.nominal = nominal;
  a.O = n_obstacles;
  a.T = n_steps;
  a.N = n_samples;
  a.nom_so = nom_so;
  a.nom_st = nom_st;
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
  const unsigned gy = static_cast<unsigned>(units < 65535 ? units : 65535);
  (void)hipGetLastError();
  hipLaunchKernelGGL(sample_kernel, dim3(static_cast<unsigned>(gx), gy), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? DRCVAR_OK : DRCVAR_ERR_LAUNCH;
}
