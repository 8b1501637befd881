// Calibration microbenchmarks (diagnostic, not shipped): shader cycles of basic operations on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

__global__ void calib(unsigned long long* out, double* sink, int iters) {
  __shared__ double lds[1024];
  const int tid = threadIdx.x;
  for (int i = tid; i < 1024; i += blockDim.x) lds[i] = 1.0 + i * 1e-6;
  __syncthreads();
  double a = 1.0 + tid * 1e-9, b = 0.999999, c = 1e-7;
  unsigned long long t0, t1;
  // 1. dependent fp64 fma chain
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) a = fma(a, b, c);
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[0] = t1 - t0;
  // 2. 8 independent chains
  double x[8];
  for (int k = 0; k < 8; ++k) x[k] = a + k;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = fma(x[k], b, c);
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[1] = t1 - t0;
  // 3. readlane chain: value -> readlane -> fma -> ...
  double r = a;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) r = fma(readlane_f64(r, i & 63), b, c);
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[2] = t1 - t0;
  // 4. barrier cost (all waves)
  __syncthreads();
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) __syncthreads();
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[3] = t1 - t0;
  // 5. dependent LDS load chain
  int idx = tid & 63;
  double acc = 0.0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    const double v = lds[idx];
    acc += v;
    idx = (static_cast<int>(v * 1e6) + i) & 1023;
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[4] = t1 - t0;
  // 6. fp64 division chain
  double dv = a;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) dv = 1.0 / (dv + 1.0);
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[5] = t1 - t0;
  // 7. s_memtime itself: back to back
  t0 = __builtin_amdgcn_s_memtime();
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[6] = t1 - t0;
  // 8. wall clock reference: s_memrealtime over the dependent fma chain
  unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) a = fma(a, b, c);
  unsigned long long w1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) out[7] = w1 - w0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) a = fma(a, b, c);
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[8] = t1 - t0;
  sink[tid] = a + x[0] + x[7] + r + acc + dv;
}

int main() {
  unsigned long long* d_out;
  double* d_sink;
  hipMalloc(&d_out, 16 * sizeof(unsigned long long));
  hipMalloc(&d_sink, 1024 * sizeof(double));
  const int iters = 1000;
  for (int threads : {64, 256}) {
    hipLaunchKernelGGL(calib, dim3(1), dim3(threads), 0, 0, d_out, d_sink, iters);
    hipDeviceSynchronize();
    unsigned long long h[16];
    hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
    printf("threads %d (per iteration, memtime ticks):\n", threads);
    const char* names[] = {"dep fma", "8 indep fma chains (per iter = 8 fma)", "readlane->fma chain",
                           "barrier", "dep LDS load", "fp64 div chain", "memtime pair (total)",
                           "realtime ticks (100MHz) for 1000 dep fma", "memtime ticks same"};
    for (int k = 0; k < 9; ++k)
      printf("  %-45s %8.2f\n", names[k], k == 6 || k == 7 || k == 8 ? (double)h[k] : (double)h[k] / iters);
  }
  return 0;
}
