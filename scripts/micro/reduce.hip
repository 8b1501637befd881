// Calibration (diagnostic, not shipped): cycles of fp64 wave-reduction variants on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rows_f64(double v) {
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
  v += dpp_f64<0x140>(v);
  return v;
}
__device__ __forceinline__ double red_readlane(double v) {
  v = rows_f64(v);
  return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}
__device__ __forceinline__ double swap16(double v, bool first) {
  auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
  auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
  return first ? __hiloint2double(hi[0], lo[0]) : __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double red_permlane(double v) {
  v = rows_f64(v);
  {
    auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
    auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
  }
  {
    auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
    auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
  }
  return v;
}
__device__ __forceinline__ float rows_f32(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  v = __int_as_float(a[0]) + __int_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(b[0]) + __int_as_float(b[1]);
}

template <int V, int K>
__global__ void bench(unsigned long long* out, double* sink, int iters) {
  const int lane = threadIdx.x & 63;
  double v[K];
  float f[K];
  for (int k = 0; k < K; ++k) { v[k] = lane * 1e-3 + k; f[k] = lane * 1e-3f + k; }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if constexpr (V == 0) v[k] = red_readlane(v[k]) * 1e-2 + lane;
      if constexpr (V == 1) v[k] = red_permlane(v[k]) * 1e-2 + lane;
      if constexpr (V == 2) f[k] = rows_f32(f[k]) * 1e-2f + lane;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int k = 0; k < K; ++k) s += v[k] + f[k];
  sink[threadIdx.x] = s;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}

template <int V, int K>
void run(const char* name, unsigned long long* d_out, double* d_sink) {
  const int iters = 200;
  hipLaunchKernelGGL((bench<V, K>), dim3(1), dim3(64), 0, 0, d_out, d_sink, iters);
  unsigned long long h = 0;
  (void)hipMemcpy(&h, d_out, sizeof(h), hipMemcpyDeviceToHost);
  printf("%-28s K=%d: %8.1f cycles per iteration (all K values)\n", name, K, (double)h / iters);
}

int main() {
  unsigned long long* d_out;
  double* d_sink;
  (void)hipMalloc(&d_out, 64);
  (void)hipMalloc(&d_sink, 64 * 8);
  run<0, 1>("readlane combine", d_out, d_sink);
  run<0, 7>("readlane combine", d_out, d_sink);
  run<1, 1>("permlane combine", d_out, d_sink);
  run<1, 7>("permlane combine", d_out, d_sink);
  run<2, 1>("f32 permlane", d_out, d_sink);
  run<2, 5>("f32 permlane", d_out, d_sink);
  // correctness: permlane result equals readlane result on lane data
  return 0;
}
