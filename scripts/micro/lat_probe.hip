// lat_probe.hip — cycles per operation of one wave on gfx950 (s_memtime): dependent and
// independent fp64 FMA chains, 64-bit DPP broadcasts, quad permutes, rcp, ds_bpermute and an LDS
// store -> load round trip.  A cost model for the Riccati step (scripts/micro/riccati_dpp.hip).
//   hipcc --offload-arch=gfx950 -O3 scripts/micro/lat_probe.hip -o lat_probe && ./lat_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 256;

template <int CTRL>
__device__ __forceinline__ double dpp32x2(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const long long x = __builtin_bit_cast(long long, v);
  const long long y = __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, y);
}

__global__ __launch_bounds__(64) void probe(const double* in, double* out, long long* cyc) {
  __shared__ double lds[256];
  const int lane = threadIdx.x;
  const double a = in[lane], b = in[64 + lane];
  double x = in[128 + lane], y = x + 1.0, z = x + 2.0, w = x + 3.0;
  long long t0, t1;
  int slot = 0;
#define TIME(body)                                        \
  t0 = __builtin_amdgcn_s_memtime();                      \
  body;                                                   \
  __builtin_amdgcn_s_waitcnt(0);                          \
  t1 = __builtin_amdgcn_s_memtime();                      \
  if (lane == 0) cyc[slot] = t1 - t0;                     \
  ++slot;
  // 0: dependent fma chain
  TIME(for (int i = 0; i < N; ++i) x = fma(x, a, b));
  // 1: four independent chains (N / 4 each)
  TIME(for (int i = 0; i < N / 4; ++i) { x = fma(x, a, b); y = fma(y, a, b); z = fma(z, a, b); w = fma(w, a, b); });
  // 2: dependent v_mov_b64_dpp row_newbcast + fma
  TIME(for (int i = 0; i < N; ++i) x = fma(dpp64<0x153>(x), a, b));
  // 3: dependent quad_perm (2 x v_mov_b32_dpp) + fma
  TIME(for (int i = 0; i < N; ++i) x = fma(dpp32x2<0x55>(x), a, b));
  // 4: dependent rcp + one Newton step
  TIME(for (int i = 0; i < N; ++i) { const double r = __builtin_amdgcn_rcp(x); x = fma(r, fma(-x, r, 1.0), r) + b; });
  // 5: dependent ds_bpermute (2 x b32) + fma
  TIME(for (int i = 0; i < N; ++i) {
    const int addr = ((lane + 4) & 63) * 4;
    const int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(x));
    const int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(x));
    x = fma(__hiloint2double(hi, lo), a, b);
  });
  // 6: LDS store -> load round trip + fma
  TIME(for (int i = 0; i < N; ++i) {
    lds[lane] = x;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    x = fma(lds[(lane + 1) & 63], a, b);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  });
  // 7: dependent v_mul_f64 chain
  TIME(for (int i = 0; i < N; ++i) x = x * a);
  // 8: independent fma, 8 chains
  {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = x + q;
    TIME(for (int i = 0; i < N / 8; ++i) {
      v[0] = fma(v[0], a, b); v[1] = fma(v[1], a, b); v[2] = fma(v[2], a, b); v[3] = fma(v[3], a, b);
      v[4] = fma(v[4], a, b); v[5] = fma(v[5], a, b); v[6] = fma(v[6], a, b); v[7] = fma(v[7], a, b);
    });
#pragma unroll
    for (int q = 0; q < 8; ++q) x += v[q];
  }
  // 9: dependent v_add_f64
  TIME(for (int i = 0; i < N; ++i) x = x + a);
  // 10: 32-bit dependent integer add chain (VALU cadence)
  {
    int u = __double2loint(x);
    TIME(for (int i = 0; i < N; ++i) u = u * 3 + lane);
    x += u;
  }
  out[lane] = x + y + z + w;
}

int main() {
  double *in, *out;
  long long* cyc;
  hipMalloc(&in, 192 * 8);
  hipMalloc(&out, 64 * 8);
  hipMalloc(&cyc, 32 * 8);
  double h[192];
  for (int i = 0; i < 192; ++i) h[i] = 1.0 + 1e-3 * i;
  hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
  const char* names[] = {"dependent fma f64", "4 independent fma chains", "dpp64 newbcast + fma",
                         "quad_perm 2xb32 + fma", "rcp + newton (3 ops)", "ds_bpermute 2xb32 + fma",
                         "lds st->ld + fma", "dependent mul f64", "8 independent fma chains",
                         "dependent add f64", "dependent int mad (2 ops)"};
  for (int rep = 0; rep < 2; ++rep) {
    probe<<<1, 64>>>(in, out, cyc);
    hipDeviceSynchronize();
    long long c[11];
    hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost);
    if (rep == 1)
      for (int i = 0; i < 11; ++i) std::printf("%-28s %6.1f cycles per iteration\n", names[i], (double)c[i] / N);
  }
  return 0;
}
