// Probe of v_mfma_f64_16x16x4_f64 on gfx950 (design tool for the Riccati recursion of
// csrc/drcvar_mpc.hip): (1) the operand / result lane maps, checked with exact integer data
// (A[i][k] at lane i + 16k, B[k][j] at lane j + 16k, D[g + 4r][j] at lane j + 16g, register r);
// (2) cycles per step of a chain of dependent MFMAs whose result feeds the next one's B operand
// (the solve recurrence x_{k+1} = F x_k + g), against the same chain in VALU fp64 FMAs with DPP.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(const double* A, const double* B, const double* C, double* D) {
  const int l = threadIdx.x;
  const double a = A[(l & 15) * 4 + (l >> 4)];   // A [16][4]
  const double b = B[(l >> 4) * 16 + (l & 15)];  // B [4][16]
  d4 c;
  for (int r = 0; r < 4; ++r) c[r] = C[((l >> 4) + 4 * r) * 16 + (l & 15)];
  const d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = d[r];
}

__global__ void chain_kernel(const double* F, int steps, double* out, long long* cycles) {
  const int l = threadIdx.x;
  const double a = F[l];  // any A operand
  double b = (l & 15) == 0 ? 1.0 : 0.0;
  d4 c = {0.0, 0.0, 0.0, 0.0};
  const long long t0 = clock64();
  for (int s = 0; s < steps; ++s) {
    const d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    b = d[0] * 0.5;  // the result (D layout, register 0) as the next B operand
  }
  const long long t1 = clock64();
  out[l] = b;
  if (l == 0) cycles[0] = t1 - t0;
}

__global__ void chain_direct_kernel(const double* F, int steps, double* out, long long* cycles) {
  const int l = threadIdx.x;
  const double a = F[l] * 1e-3;
  double b = (l & 15) == 0 ? 1.0 : 0.0;
  d4 c = {0.0, 0.0, 0.0, 0.0};
  const long long t0 = clock64();
  for (int s = 0; s < steps; ++s) {
    const d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    b = d[0];  // the result register as the next B operand, nothing between
  }
  const long long t1 = clock64();
  out[l] = b;
  if (l == 0) cycles[0] = t1 - t0;
}

__global__ void chain_acc_kernel(const double* F, int steps, double* out, long long* cycles) {
  const int l = threadIdx.x;
  const double a = F[l] * 1e-3, b = F[l + 64] * 1e-3;
  d4 c = {0.0, 0.0, 0.0, 0.0};
  const long long t0 = clock64();
  for (int s = 0; s < steps; ++s) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  const long long t1 = clock64();
  out[l] = c[0] + c[1] + c[2] + c[3];
  if (l == 0) cycles[0] = t1 - t0;
}

template <int CTRL>
__device__ __forceinline__ double qb(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

__global__ void dpp_chain_kernel(const double* F, int steps, double* out, long long* cycles) {
  const int l = threadIdx.x;
  const double f0 = F[l] * 1e-3, f1 = F[l + 64] * 1e-3, f2 = F[l + 128] * 1e-3, f3 = F[l + 192] * 1e-3;
  double v = 1.0;
  const long long t0 = clock64();
  for (int s = 0; s < steps; ++s)
    v = fma(f0, qb<0x00>(v), fma(f1, qb<0x55>(v), 0.25)) + fma(f2, qb<0xAA>(v), f3 * qb<0xFF>(v));
  const long long t1 = clock64();
  out[l] = v;
  if (l == 0) cycles[0] = t1 - t0;
}

__global__ void valu_chain_kernel(const double* F, int steps, double* out, long long* cycles) {
  const int l = threadIdx.x;
  const double f0 = F[l], f1 = F[l + 64], f2 = F[l + 128], f3 = F[l + 192];
  double v = 1.0;
  const long long t0 = clock64();
  for (int s = 0; s < steps; ++s) {
    // quad broadcast of the previous state + 4 FMAs (the round-3 solve step)
    const double v0 = __shfl(v, (l & ~3) | 0, 64), v1 = __shfl(v, (l & ~3) | 1, 64);
    const double v2 = __shfl(v, (l & ~3) | 2, 64), v3 = __shfl(v, (l & ~3) | 3, 64);
    v = fma(f0, v0, fma(f1, v1, 0.25)) + fma(f2, v2, f3 * v3);
  }
  const long long t1 = clock64();
  out[l] = v;
  if (l == 0) cycles[0] = t1 - t0;
}

__global__ void swap_kernel(int* out) {
  const int l = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane16_swap(l, l + 100, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
}

int main() {
  double hA[64], hB[64], hC[256], hD[256];
  srand(7);
  for (int i = 0; i < 64; ++i) hA[i] = rand() % 7 - 3, hB[i] = rand() % 5 - 2;
  for (int i = 0; i < 256; ++i) hC[i] = rand() % 9 - 4;
  double *A, *B, *C, *D, *F, *out;
  long long* cyc;
  hipMalloc(&A, 512); hipMalloc(&B, 512); hipMalloc(&C, 2048); hipMalloc(&D, 2048);
  hipMalloc(&F, 2048); hipMalloc(&out, 512); hipMalloc(&cyc, 8);
  hipMemcpy(A, hA, 512, hipMemcpyHostToDevice);
  hipMemcpy(B, hB, 512, hipMemcpyHostToDevice);
  hipMemcpy(C, hC, 2048, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(layout_kernel, 1, 64, 0, 0, A, B, C, D);
  hipMemcpy(hD, D, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double want = hC[i * 16 + j];
      for (int k = 0; k < 4; ++k) want += hA[i * 4 + k] * hB[k * 16 + j];
      bad += want != hD[i * 16 + j];
    }
  printf("layout check: %d of 256 entries differ\n", bad);
  hipMemcpy(F, hC, 2048, hipMemcpyHostToDevice);
  long long c = 0;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(chain_kernel, 1, 64, 0, 0, F, 1000, out, cyc);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("dependent mfma_f64_16x16x4 chain: %.1f cycles per step\n", c / 1000.0);
    hipLaunchKernelGGL(chain_direct_kernel, 1, 64, 0, 0, F, 1000, out, cyc);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("dependent mfma chain, result straight into B: %.1f cycles per step\n", c / 1000.0);
    hipLaunchKernelGGL(chain_acc_kernel, 1, 64, 0, 0, F, 1000, out, cyc);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("dependent mfma chain through the accumulator C: %.1f cycles per step\n", c / 1000.0);
    hipLaunchKernelGGL(dpp_chain_kernel, 1, 64, 0, 0, F, 1000, out, cyc);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("dependent VALU DPP quad-broadcast + 4 fma chain: %.1f cycles per step\n", c / 1000.0);
    hipLaunchKernelGGL(valu_chain_kernel, 1, 64, 0, 0, F, 1000, out, cyc);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("dependent VALU quad-broadcast + 4 fma chain: %.1f cycles per step\n", c / 1000.0);
  }
  int* sw;
  int hsw[128];
  hipMalloc(&sw, 512);
  hipLaunchKernelGGL(swap_kernel, 1, 64, 0, 0, sw);
  hipMemcpy(hsw, sw, 512, hipMemcpyDeviceToHost);
  printf("permlane16_swap(old = lane, src = lane + 100): [0] =");
  for (int i = 0; i < 64; i += 4) printf(" %d", hsw[i]);
  printf("\n  [1] =");
  for (int i = 0; i < 64; i += 4) printf(" %d", hsw[64 + i]);
  printf("\n");
  return 0;
}
