// riccati_dpp.hip — micro-benchmark of the NX = 4, NU = 2 Riccati factorisation step on one wave
// (csrc/drcvar_mpc.hip, riccati_factor_wave0): the product's LDS form (P, T = PA, U = PB handed
// through LDS, two round trips per step) against a register form (lane 4i + j holds P_ij; row i by
// DPP quad broadcasts, U and every entry of P by v_mov_b64 row_newbcast; the A'PA and L'Ri L terms
// summed in a symmetric-exact order so that P stays exactly symmetric without a transpose).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/micro/riccati_dpp.hip -o /tmp/riccati_dpp
//   /tmp/riccati_dpp [H] [reps] [weight scale]
//
// Prints cycles per horizon step (s_memtime, wave 0) of each form and the largest relative
// difference of Kg, Ri and P_0 against a host long-double recursion on the same data.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

constexpr int NX = 4, NU = 2, kMx = 4, HM = 64;

struct L {
  double *Am, *Bm, *Cm, *Qm, *Rm, *P, *T, *U, *Kg, *Ri, *S, *DU, *junk, *QB;
};
__device__ inline L carve(double* b) {
  L s;
  s.Am = b; b += 16;
  s.Bm = b; b += 8;
  s.Cm = b; b += 8;
  s.Qm = b; b += 16;
  s.Rm = b; b += 4;
  s.P = b; b += 16;
  s.T = b; b += 16;
  s.U = b; b += 8;
  s.Kg = b; b += HM * NU * NX;
  s.Ri = b; b += HM * NU * NU;
  s.S = b; b += 3 * HM;
  s.DU = b; b += NU * HM;
  s.junk = b; b += 64;
  s.QB = b; b += 20 * HM;
  return s;
}
constexpr int kLdsDoubles = 16 + 8 + 8 + 16 + 4 + 16 + 16 + 8 + HM * 8 + HM * 4 + 3 * HM + 2 * HM + 64 + 20 * HM;

__device__ __forceinline__ void wave_lds_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
__device__ __forceinline__ double rcp(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(r, fma(-x, r, 1.0), r);
}

// ---------------- V0: the product's LDS form (riccati_factor_wave0, NU = 2, NX = 4) ----------------
__device__ inline bool fact_lds(const L& s, int H) {
  const int tid = threadIdx.x, lane = tid & 63;
  bool ok = true;
  if (tid < 64) {
    constexpr int NX2 = NX * NX;
    const int e = lane < NX2 ? lane : 0;
    const int i = e / NX, j = e % NX;
    const int uc = j < NU ? j : 0;
    double Acol[NX], Bcol[NX];
#pragma unroll
    for (int m = 0; m < NX; ++m) {
      Acol[m] = s.Am[m * kMx + j];
      Bcol[m] = s.Bm[m * NU + uc];
    }
    const double c0i = s.Cm[i], c1i = s.Cm[kMx + i], c0j = s.Cm[j], c1j = s.Cm[kMx + j];
    const double q2 = 2.0 * s.Qm[i * kMx + j];
    double ai[NX], Bm[NX][NU], R2[NU][NU];
#pragma unroll
    for (int m = 0; m < NX; ++m) {
      ai[m] = s.Am[m * kMx + i];
#pragma unroll
      for (int c = 0; c < NU; ++c) Bm[m][c] = s.Bm[m * NU + c];
    }
#pragma unroll
    for (int c = 0; c < NU; ++c)
#pragma unroll
      for (int d = 0; d < NU; ++d) R2[c][d] = 2.0 * s.Rm[c * NU + d];
    auto qb = [&](int k) {
      const double S00 = s.S[k], S01 = s.S[H + k], S11 = s.S[2 * H + k];
      return q2 + c0i * (S00 * c0j + S01 * c1j) + c1i * (S01 * c0j + S11 * c1j);
    };
    if (lane < NX2 && i >= j) {
      const double v = qb(H - 1);
      s.P[i * kMx + j] = v;
      s.P[j * kMx + i] = v;
    }
    for (int k = H - 1; k >= 0 && ok; --k) {
      wave_lds_fence();
      {
        double prow[NX];
#pragma unroll
        for (int m = 0; m < NX; ++m) prow[m] = s.P[i * kMx + m];
        double t = 0.0, uu = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) {
          t += prow[m] * Acol[m];
          uu += prow[m] * Bcol[m];
        }
        if (lane < NX2) s.T[i * kMx + j] = t;
        if (lane < NX2 && j < NU) s.U[i * NU + j] = uu;
      }
      wave_lds_fence();
      double ti[NX], tj[NX], Um[NX][NU], du[NU];
#pragma unroll
      for (int m = 0; m < NX; ++m) {
        ti[m] = s.T[m * kMx + i];
        tj[m] = s.T[m * kMx + j];
#pragma unroll
        for (int c = 0; c < NU; ++c) Um[m][c] = s.U[m * NU + c];
      }
#pragma unroll
      for (int c = 0; c < NU; ++c) du[c] = s.DU[k * NU + c];
      const double qnext = k > 0 ? qb(k - 1) : 0.0;
      double Re[NU][NU];
#pragma unroll
      for (int c = 0; c < NU; ++c)
#pragma unroll
        for (int d = 0; d < NU; ++d) {
          double acc = R2[c][d] + (c == d ? du[c] : 0.0);
#pragma unroll
          for (int m = 0; m < NX; ++m) acc += Bm[m][c] * Um[m][d];
          Re[c][d] = acc;
        }
      const double det = Re[0][0] * Re[1][1] - Re[0][1] * Re[1][0];
      const double id = rcp(det);
      double Ri[2][2] = {{Re[1][1] * id, -Re[0][1] * id}, {-Re[1][0] * id, Re[0][0] * id}};
      ok = Re[0][0] > 0.0 && det > 0.0 && isfinite(det) && isfinite(Re[0][0]);
      double Li[NU], Lj[NU], Kj[NU];
#pragma unroll
      for (int c = 0; c < NU; ++c) {
        double li = 0.0, lj = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) {
          li += Bm[m][c] * ti[m];
          lj += Bm[m][c] * tj[m];
        }
        Li[c] = li;
        Lj[c] = lj;
      }
#pragma unroll
      for (int c = 0; c < NU; ++c) {
        double acc = 0.0;
#pragma unroll
        for (int d = 0; d < NU; ++d) acc += Ri[c][d] * Lj[d];
        Kj[c] = acc;
      }
      if (lane < NX2 && i == j) {
#pragma unroll
        for (int c = 0; c < NU; ++c) s.Kg[(k * NU + c) * NX + j] = Kj[c];
      }
      if (lane < NX2 && k > 0 && i >= j) {
        double acc = qnext;
#pragma unroll
        for (int m = 0; m < NX; ++m) acc += ai[m] * tj[m];
#pragma unroll
        for (int c = 0; c < NU; ++c) acc -= Li[c] * Kj[c];
        s.P[i * kMx + j] = acc;
        s.P[j * kMx + i] = acc;
      }
      if (lane == 0) {
#pragma unroll
        for (int c = 0; c < NU; ++c)
#pragma unroll
          for (int d = 0; d < NU; ++d) s.Ri[(k * NU + c) * NU + d] = Ri[c][d];
      }
    }
  }
  return ok;
}

// ---------------- V1: register form ----------------
template <int CTRL>
__device__ __forceinline__ double quad_bcast_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// lane n of each row of 16 (v_mov_b64_dpp row_newbcast:n)
template <int N>
__device__ __forceinline__ double row_bcast_f64(double v) {
  const long long x = __builtin_bit_cast(long long, v);
  const long long y = __builtin_amdgcn_mov_dpp(x, 0x150 + N, 0xF, 0xF, false);
  return __builtin_bit_cast(double, y);
}
__device__ __forceinline__ double dpp_ror8_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x128, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x128, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double bperm_f64(double v, int addr) {
  const int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(v));
  return __hiloint2double(hi, lo);
}
// (no contraction into fma: the symmetric-exact sums rely on separately rounded products)
__device__ __forceinline__ double mul_rn(double a, double b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ double add_rn(double a, double b) {
#pragma clang fp contract(off)
  return a + b;
}

// Lane l = 4 i + j (every row of 16 lanes computes the same) holds P_ij.  Per step:
//   row i of P (quad broadcasts) -> U_{i, j&1} = (P B)_{i, j&1};  U (8 entries) and the 10 unique
//   entries of P to every lane by row_newbcast (canonical order, so every lane sums in the same
//   order);  Re = Rb + B'U, Ri = Re^-1 (identical in every lane);  L_.x = U'A_.x for x = i, j;
//   Kg_.j = Ri L_.j;  P_ij = Qb_ij + sum_{m<=n} G^{ij}_mn P_mn - L_.i' Ri L_.j, where
//   G^{ij}_mn = A_mi A_nj + A_ni A_mj (m < n), A_mi A_mj (m = n), and the last term in the
//   product-then-sum form (L_0i L_1j + L_1i L_0j): both are invariant under i <-> j bit for bit,
//   so P_ij and P_ji come out identical and P stays exactly symmetric.
__device__ inline bool fact_reg(const L& s, int H) {
  const int tid = threadIdx.x, lane = tid & 63;
  bool ok = true;
  if (tid < 64) {
    const int l = lane & 15, i = l >> 2, j = l & 3;
    const int ia = i > j ? i : j, jb = i > j ? j : i;  // canonical (lower-triangle) roles
    double Bm[4][2], Ai[4], Aj[4], Bc[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      Bm[m][0] = s.Bm[m * NU];
      Bm[m][1] = s.Bm[m * NU + 1];
      Ai[m] = s.Am[m * kMx + i];
      Aj[m] = s.Am[m * kMx + j];
      Bc[m] = s.Bm[m * NU + (j & 1)];
    }
    double G[10];
    {
      int q = 0;
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n <= m; ++n) {  // (m, n), m >= n: entry P_mn held by lane 4m + n
          const double a = s.Am[m * kMx + ia], b = s.Am[n * kMx + jb];
          const double c = s.Am[n * kMx + ia], d = s.Am[m * kMx + jb];
          G[q++] = m == n ? mul_rn(a, b) : add_rn(mul_rn(a, b), mul_rn(c, d));
        }
    }
    const double c0a = s.Cm[ia], c1a = s.Cm[kMx + ia], c0b = s.Cm[jb], c1b = s.Cm[kMx + jb];
    const double q2 = 2.0 * s.Qm[ia * kMx + jb];
    const double R00 = 2.0 * s.Rm[0], R01 = 2.0 * s.Rm[1], R11 = 2.0 * s.Rm[3];
    auto qb = [&](int k) {  // Qb_{k+1}(ia, jb): the same value in lanes (i, j) and (j, i)
      const double S00 = s.S[k], S01 = s.S[H + k], S11 = s.S[2 * H + k];
      return q2 + c0a * (S00 * c0b + S01 * c1b) + c1a * (S01 * c0b + S11 * c1b);
    };
    double p = qb(H - 1);
    // stores: every lane writes, lanes with equal values to equal addresses (the 16-lane rows
    // replicate each other): Kg[k][i & 1][j] and Ri[k][l & 3] (Ri00, Ri01, Ri10 = Ri01, Ri11)
    double* kg_at = s.Kg + ((H - 1) * NU + (i & 1)) * NX + j;
    double* ri_at = s.Ri + (H - 1) * 4 + (l & 3);
    const int rsel = l & 3;
    for (int k = H - 1; k >= 0; --k) {
      const double du0 = s.DU[k * NU], du1 = s.DU[k * NU + 1];
      const double qn = qb(k > 0 ? k - 1 : 0);  // (unused at k = 0)
      // row i of P
      const double r0 = quad_bcast_f64<0x00>(p), r1 = quad_bcast_f64<0x55>(p);
      const double r2 = quad_bcast_f64<0xAA>(p), r3 = quad_bcast_f64<0xFF>(p);
      const double uu = fma(r3, Bc[3], fma(r2, Bc[2], fma(r1, Bc[1], r0 * Bc[0])));  // U_{i, j&1}
      // U in canonical order: U_mc from lane 4m + c
      const double U00 = row_bcast_f64<0>(uu), U01 = row_bcast_f64<1>(uu);
      const double U10 = row_bcast_f64<4>(uu), U11 = row_bcast_f64<5>(uu);
      const double U20 = row_bcast_f64<8>(uu), U21 = row_bcast_f64<9>(uu);
      const double U30 = row_bcast_f64<12>(uu), U31 = row_bcast_f64<13>(uu);
      // every unique entry of P (lane 4m + n, m >= n)
      const double P00 = row_bcast_f64<0>(p), P10 = row_bcast_f64<4>(p), P11 = row_bcast_f64<5>(p);
      const double P20 = row_bcast_f64<8>(p), P21 = row_bcast_f64<9>(p), P22 = row_bcast_f64<10>(p);
      const double P30 = row_bcast_f64<12>(p), P31 = row_bcast_f64<13>(p), P32 = row_bcast_f64<14>(p);
      const double P33 = row_bcast_f64<15>(p);
      const double Re00 = fma(Bm[3][0], U30, fma(Bm[2][0], U20, fma(Bm[1][0], U10, fma(Bm[0][0], U00, R00 + du0))));
      const double Re01 = fma(Bm[3][0], U31, fma(Bm[2][0], U21, fma(Bm[1][0], U11, fma(Bm[0][0], U01, R01))));
      const double Re11 = fma(Bm[3][1], U31, fma(Bm[2][1], U21, fma(Bm[1][1], U11, fma(Bm[0][1], U01, R11 + du1))));
      const double det = fma(Re00, Re11, -(Re01 * Re01));
      const double id = rcp(det);
      // (a non-finite Re00 makes det non-finite or NaN; NaN fails every comparison)
      ok = ok && Re00 > 0.0 && det > 0.0 && det < __builtin_huge_val();
      const double Ri00 = Re11 * id, Ri01 = -Re01 * id, Ri11 = Re00 * id;
      // L_cx = sum_m U_mc A_mx, x = i, j
      const double L0i = fma(U30, Ai[3], fma(U20, Ai[2], fma(U10, Ai[1], U00 * Ai[0])));
      const double L1i = fma(U31, Ai[3], fma(U21, Ai[2], fma(U11, Ai[1], U01 * Ai[0])));
      const double L0j = fma(U30, Aj[3], fma(U20, Aj[2], fma(U10, Aj[1], U00 * Aj[0])));
      const double L1j = fma(U31, Aj[3], fma(U21, Aj[2], fma(U11, Aj[1], U01 * Aj[0])));
      const double K0j = fma(Ri01, L1j, Ri00 * L0j), K1j = fma(Ri11, L1j, Ri01 * L0j);
      // A'PA (symmetric-exact)
      double apa = G[0] * P00;
      apa = fma(G[1], P10, apa);
      apa = fma(G[2], P11, apa);
      apa = fma(G[3], P20, apa);
      apa = fma(G[4], P21, apa);
      apa = fma(G[5], P22, apa);
      apa = fma(G[6], P30, apa);
      apa = fma(G[7], P31, apa);
      apa = fma(G[8], P32, apa);
      apa = fma(G[9], P33, apa);
      const double m00 = mul_rn(L0i, L0j), m11 = mul_rn(L1i, L1j);
      const double m01 = add_rn(mul_rn(L0i, L1j), mul_rn(L1i, L0j));
      const double lrl = fma(m00, Ri00, fma(m01, Ri01, m11 * Ri11));
      *kg_at = (i & 1) ? K1j : K0j;
      *ri_at = rsel == 0 ? Ri00 : (rsel == 3 ? Ri11 : Ri01);
      kg_at -= NU * NX;
      ri_at -= 4;
      p = (qn + apa) - lrl;
    }
  }
  return ok;
}


// ---------------- V2: register form, M-form ----------------
// P_k = Qb_k + A' M A,  M = P - U Ri U' (U = P B, Ri = (Rb + B'U)^-1): lane 4m + n forms M_mn from
// the broadcast U (symmetric-exact: products rounded separately, then summed in an order that is
// invariant under m <-> n), the 10 unique M_mn reach every lane by row_newbcast and A'MA sums them
// with the loop-invariant symmetric weights G^{ij}.  Per step the wave reads one record of the
// step table built in front of the loop (QB[k]: the 16 entries of Qb_k in canonical roles, then
// Rb00, Rb11 of step k), so no Qb arithmetic or S / DU addressing sits in the loop.  Kg = Ri U'A
// (column j per lane) and Ri are stored by lanes 0..3 / 0 (the others into scratch: no branch).
// A failed pivot is not tested per step: the minimum over the steps of det and Re00 and the
// finiteness of P_0 (a NaN or infinity anywhere propagates into it) give the same verdict.
__device__ inline void qb_table(const L& s, int H) {  // by the factorisation's own wave, lane = step
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < 64) {
    const double q2[4][4] = {{2.0 * s.Qm[0], 2.0 * s.Qm[1], 2.0 * s.Qm[2], 2.0 * s.Qm[3]},
                             {2.0 * s.Qm[kMx], 2.0 * s.Qm[kMx + 1], 2.0 * s.Qm[kMx + 2], 2.0 * s.Qm[kMx + 3]},
                             {2.0 * s.Qm[2 * kMx], 2.0 * s.Qm[2 * kMx + 1], 2.0 * s.Qm[2 * kMx + 2], 2.0 * s.Qm[2 * kMx + 3]},
                             {2.0 * s.Qm[3 * kMx], 2.0 * s.Qm[3 * kMx + 1], 2.0 * s.Qm[3 * kMx + 2], 2.0 * s.Qm[3 * kMx + 3]}};
    for (int kk = lane; kk < H; kk += 64) {  // weights of step kk -> record kk + 1 (kk = H - 1: record 0)
      const int rk = kk + 1 < H ? kk + 1 : 0;
      const double S00 = s.S[kk], S01 = s.S[H + kk], S11 = s.S[2 * H + kk];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b <= a; ++b) {
          const double c0a = s.Cm[a], c1a = s.Cm[kMx + a], c0b = s.Cm[b], c1b = s.Cm[kMx + b];
          const double v = q2[a][b] + c0a * (S00 * c0b + S01 * c1b) + c1a * (S01 * c0b + S11 * c1b);
          s.QB[rk * 20 + a * 4 + b] = v;
          s.QB[rk * 20 + b * 4 + a] = v;
        }
      s.QB[kk * 20 + 16] = 2.0 * s.Rm[0] + s.DU[kk * NU];
      s.QB[kk * 20 + 17] = 2.0 * s.Rm[3] + s.DU[kk * NU + 1];
    }
  }
}
__device__ inline bool fact_reg2(const L& s, int H) {
  const int tid = threadIdx.x, lane = tid & 63;
  bool ok = true;
  if (tid < 64) {
    qb_table(s, H);
    wave_lds_fence();
    const int l = lane & 15, i = l >> 2, j = l & 3;
    const int ia = i > j ? i : j, jb = i > j ? j : i;
    double Bm[4][2], Aj[4], Bc[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      Bm[m][0] = s.Bm[m * NU];
      Bm[m][1] = s.Bm[m * NU + 1];
      Aj[m] = s.Am[m * kMx + j];
      Bc[m] = s.Bm[m * NU + (j & 1)];
    }
    double G[10];
    {
      int q = 0;
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n <= m; ++n) {
          const double a = s.Am[m * kMx + ia], b = s.Am[n * kMx + jb];
          const double c = s.Am[n * kMx + ia], d = s.Am[m * kMx + jb];
          G[q++] = m == n ? mul_rn(a, b) : add_rn(mul_rn(a, b), mul_rn(c, d));
        }
    }
    const double R01 = 2.0 * s.Rm[1];
    const int src_j0 = ((lane & ~15) + 4 * j) * 4, src_j1 = src_j0 + 4;  // byte addresses of ds_bpermute
    // lane (i, j) forms M_{ia, jb}: U rows ia and jb are picked once per step by the canonical
    // broadcast below (row selectors as loop-invariant lane masks)
    const double* rec = s.QB + (H - 1) * 20;
    double p = s.QB[l];  // the terminal Qb (record 0)
    double mn = 1.0;
    double* kg_at = l < 4 ? s.Kg + (H - 1) * NU * NX + j : s.junk + 2 * l;
    const int kg_step = l < 4 ? NU * NX : 0;
    double* ri_at = l == 0 ? s.Ri + (H - 1) * 4 : s.junk + 32 + 2 * l;
    const int ri_step = l == 0 ? 4 : 0;
    for (int k = H - 1; k >= 0; --k) {
      const double qn = rec[l];  // Qb_k = qb(k - 1) (unused at k = 0, where record 0 is the terminal)
      const double rb00 = rec[16], rb11 = rec[17];
      rec -= 20;
      const double r0 = quad_bcast_f64<0x00>(p), r1 = quad_bcast_f64<0x55>(p);
      const double r2 = quad_bcast_f64<0xAA>(p), r3 = quad_bcast_f64<0xFF>(p);
      const double uu = fma(r3, Bc[3], fma(r2, Bc[2], fma(r1, Bc[1], r0 * Bc[0])));  // U_{i, j&1}
      const double U00 = row_bcast_f64<0>(uu), U01 = row_bcast_f64<1>(uu);
      const double U10 = row_bcast_f64<4>(uu), U11 = row_bcast_f64<5>(uu);
      const double U20 = row_bcast_f64<8>(uu), U21 = row_bcast_f64<9>(uu);
      const double U30 = row_bcast_f64<12>(uu), U31 = row_bcast_f64<13>(uu);
      const double Re00 = fma(Bm[3][0], U30, fma(Bm[2][0], U20, fma(Bm[1][0], U10, fma(Bm[0][0], U00, rb00))));
      const double Re01 = fma(Bm[3][0], U31, fma(Bm[2][0], U21, fma(Bm[1][0], U11, fma(Bm[0][0], U01, R01))));
      const double Re11 = fma(Bm[3][1], U31, fma(Bm[2][1], U21, fma(Bm[1][1], U11, fma(Bm[0][1], U01, rb11))));
      const double det = fma(Re00, Re11, -(Re01 * Re01));
      const double id = rcp(det);
      mn = fmin(mn, fmin(det, Re00));
      const double Ri00 = Re11 * id, Ri01 = -Re01 * id, Ri11 = Re00 * id;
      // rows i and j of U for M_ij (only the lanes i >= j are broadcast below): row i from the
      // lane's own quad (quad_perm), row j from lanes 4j, 4j + 1 of its row (ds_bpermute, whose
      // latency hides behind Re and its inverse)
      const double Ua0 = quad_bcast_f64<0x00>(uu), Ua1 = quad_bcast_f64<0x55>(uu);
      const double Ub0 = bperm_f64(uu, src_j0), Ub1 = bperm_f64(uu, src_j1);
      const double m00 = mul_rn(Ua0, Ub0), m11 = mul_rn(Ua1, Ub1);
      const double m01 = add_rn(mul_rn(Ua0, Ub1), mul_rn(Ua1, Ub0));
      const double M = p - fma(m00, Ri00, fma(m01, Ri01, m11 * Ri11));
      const double M00 = row_bcast_f64<0>(M), M10 = row_bcast_f64<4>(M), M11 = row_bcast_f64<5>(M);
      const double M20 = row_bcast_f64<8>(M), M21 = row_bcast_f64<9>(M), M22 = row_bcast_f64<10>(M);
      const double M30 = row_bcast_f64<12>(M), M31 = row_bcast_f64<13>(M), M32 = row_bcast_f64<14>(M);
      const double M33 = row_bcast_f64<15>(M);
      // Kg_.j = Ri U'A_.j (off the chain)
      const double L0j = fma(U30, Aj[3], fma(U20, Aj[2], fma(U10, Aj[1], U00 * Aj[0])));
      const double L1j = fma(U31, Aj[3], fma(U21, Aj[2], fma(U11, Aj[1], U01 * Aj[0])));
      const double K0j = fma(Ri01, L1j, Ri00 * L0j), K1j = fma(Ri11, L1j, Ri01 * L0j);
      kg_at[0] = K0j;
      kg_at[NX] = K1j;
      kg_at -= kg_step;
      ri_at[0] = Ri00;
      ri_at[1] = Ri01;
      ri_at[2] = Ri01;
      ri_at[3] = Ri11;
      ri_at -= ri_step;
      double a0 = G[0] * M00, a1 = G[1] * M10;
      a0 = fma(G[2], M11, a0);
      a1 = fma(G[3], M20, a1);
      a0 = fma(G[4], M21, a0);
      a1 = fma(G[5], M22, a1);
      a0 = fma(G[6], M30, a0);
      a1 = fma(G[7], M31, a1);
      a0 = fma(G[8], M32, a0);
      a1 = fma(G[9], M33, a1);
      p = qn + (a0 + a1);
    }
    ok = mn > 0.0 && __builtin_isfinite(p);
  }
  return ok;
}

// ---------------- V3: planar isotropic models (A = [[a00 I, a01 I], [a10 I, a11 I]], B = [[b0 I], [b1 I]]) ----
// (the reference's double integrator: a00 = a11 = 1, a01 = dt, a10 = 0, b0 = dt^2 / 2, b1 = dt).
// With i = 2 bi + xi: A_mi = a[bm][bi] when m % 2 == xi, so every sum over the state couples a lane
// only with lanes l ^ 2 (the other column block), l ^ 8 (the other row block) and l ^ 10:
//   U_ic = b0 P_{i,c} + b1 P_{i,c+2}               (quad_perm within quad i)
//   Re_cd = Rb_cd + b0 U_{c,d} + b1 U_{c+2,d}       (row_newbcast of U)
//   M_ij = P_ij - U_i Ri U_j'                       (rows i: quad_perm, j: ds_bpermute)
//   P'_ij = Qb_ij + c00 M_ij + (c01 M_{i,j^2} + c10 M_{i^2,j}) + c11 M_{i^2,j^2}
// with c00 = a[bi][bi] a[bj][bj], c01 = a[bi][bi] a[1-bj][bj], c10 = a[1-bi][bi] a[bj][bj],
// c11 = a[1-bi][bi] a[1-bj][bj] (products rounded separately; the middle pair summed first), which
// is invariant under i <-> j bit for bit: P stays exactly symmetric.  The wave stores U_k (lanes
// j < 2) and Ri_k; the gains Kg_k = Ri_k U_k' A follow in a parallel pass.
__device__ inline bool fact_iso(const L& s, int H) {
  const int tid = threadIdx.x, lane = tid & 63;
  bool ok = true;
  if (tid < 64) {
    qb_table(s, H);
    wave_lds_fence();
    const int l = lane & 15, i = l >> 2, j = l & 3, bi = i >> 1, bj = j >> 1;
    // coefficients from A (read at the block positions) and B
    const double a00 = s.Am[0], a01 = s.Am[2], a10 = s.Am[2 * kMx], a11 = s.Am[2 * kMx + 2];
    const double b0 = s.Bm[0], b1 = s.Bm[2 * NU];
    const double aa[2][2] = {{a00, a01}, {a10, a11}};
    const double c00 = mul_rn(aa[bi][bi], aa[bj][bj]), c01 = mul_rn(aa[bi][bi], aa[1 - bj][bj]);
    const double c10 = mul_rn(aa[1 - bi][bi], aa[bj][bj]), c11 = mul_rn(aa[1 - bi][bi], aa[1 - bj][bj]);
    const double R01 = 2.0 * s.Rm[1];
    const int src_j0 = ((lane & ~15) + 4 * j) * 4, src_j1 = src_j0 + 4;
    const double* rec = s.QB + (H - 1) * 20;
    double p = s.QB[l];
    double mn = 1.0;
    // U_k: lane 4i + c (c < 2) holds U_{i,c}; stores into Kg's slot k as [i][c] (the others: scratch)
    double* u_at = j < 2 ? s.Kg + (H - 1) * 8 + i * 2 + j : s.junk + l;
    const int u_step = j < 2 ? 8 : 0;
    double* ri_at = l == 0 ? s.Ri + (H - 1) * 4 : s.junk + 32 + 2 * l;
    const int ri_step = l == 0 ? 4 : 0;
    for (int k = H - 1; k >= 0; --k) {
      const double qn = rec[l];
      const double rb00 = rec[16], rb11 = rec[17];
      rec -= 20;
      // U_{i, j&1} = b0 P_{i, j&1} + b1 P_{i, (j&1) + 2}
      const double pa = quad_bcast_f64<0x44>(p), pb = quad_bcast_f64<0xEE>(p);  // [0,1,0,1], [2,3,2,3]
      const double uu = fma(b1, pb, b0 * pa);
      const double U00 = row_bcast_f64<0>(uu), U01 = row_bcast_f64<1>(uu), U11 = row_bcast_f64<5>(uu);
      const double U20 = row_bcast_f64<8>(uu), U21 = row_bcast_f64<9>(uu), U31 = row_bcast_f64<13>(uu);
      const double Ub0 = bperm_f64(uu, src_j0), Ub1 = bperm_f64(uu, src_j1);
      __builtin_amdgcn_sched_barrier(0);  // both permutes issue here; their latency hides behind Re
      const double Ua0 = quad_bcast_f64<0x00>(uu), Ua1 = quad_bcast_f64<0x55>(uu);
      *u_at = uu;
      u_at -= u_step;
      const double Re00 = fma(b1, U20, fma(b0, U00, rb00));
      const double Re01 = fma(b1, U21, fma(b0, U01, R01));
      const double Re11 = fma(b1, U31, fma(b0, U11, rb11));
      const double det = fma(Re00, Re11, -(Re01 * Re01));
      const double id = rcp(det);
      mn = fmin(mn, fmin(det, Re00));
      const double Ri00 = Re11 * id, Ri01 = -Re01 * id, Ri11 = Re00 * id;
      ri_at[0] = Ri00;
      ri_at[1] = Ri01;
      ri_at[2] = Ri01;
      ri_at[3] = Ri11;
      ri_at -= ri_step;
      const double m00 = mul_rn(Ua0, Ub0), m11 = mul_rn(Ua1, Ub1);
      const double m01 = add_rn(mul_rn(Ua0, Ub1), mul_rn(Ua1, Ub0));
      const double M = p - fma(m00, Ri00, fma(m01, Ri01, m11 * Ri11));
      const double Mc = quad_bcast_f64<0x4E>(M);  // l ^ 2: [2,3,0,1]
      const double Mr = dpp_ror8_f64(M);           // l ^ 8
      const double Md = quad_bcast_f64<0x4E>(Mr);  // l ^ 10
      const double t = add_rn(mul_rn(c01, Mc), mul_rn(c10, Mr));
      p = qn + add_rn(add_rn(mul_rn(c00, M), t), mul_rn(c11, Md));
    }
    ok = mn > 0.0 && __builtin_isfinite(p);
  }
  return ok;
}
// Kg_k = Ri_k U_k' A from the stored U_k (in Kg's slot), one thread per step
__device__ inline void iso_gains(const L& s, int H) {
  for (int k = threadIdx.x; k < H; k += blockDim.x) {
    double U[4][2], Ri[2][2];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      U[m][0] = s.Kg[k * 8 + m * 2];
      U[m][1] = s.Kg[k * 8 + m * 2 + 1];
    }
    Ri[0][0] = s.Ri[k * 4];
    Ri[0][1] = s.Ri[k * 4 + 1];
    Ri[1][0] = s.Ri[k * 4 + 2];
    Ri[1][1] = s.Ri[k * 4 + 3];
    double K[2][4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      double L0 = 0.0, L1 = 0.0;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        L0 += U[m][0] * s.Am[m * kMx + x];
        L1 += U[m][1] * s.Am[m * kMx + x];
      }
      K[0][x] = Ri[0][0] * L0 + Ri[0][1] * L1;
      K[1][x] = Ri[1][0] * L0 + Ri[1][1] * L1;
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int x = 0; x < 4; ++x) s.Kg[(k * NU + c) * NX + x] = K[c][x];
  }
}

template <int V>
__global__ __launch_bounds__(512) void bench(const double* in, double* out, long long* cyc, int H, int reps) {
  extern __shared__ double lds[];
  const L s = carve(lds);
  const int t = threadIdx.x;
  // in: A[16] B[8] C[8] Q[16] R[4] S[3H] DU[2H]
  for (int e = t; e < 16; e += blockDim.x) { s.Am[e] = in[e]; s.Qm[e] = in[32 + e]; }
  for (int e = t; e < 8; e += blockDim.x) { s.Bm[e] = in[16 + e]; s.Cm[e] = in[24 + e]; }
  for (int e = t; e < 4; e += blockDim.x) s.Rm[e] = in[48 + e];
  for (int e = t; e < 3 * H; e += blockDim.x) s.S[e] = in[52 + e];
  for (int e = t; e < 2 * H; e += blockDim.x) s.DU[e] = in[52 + 3 * H + e];
  __syncthreads();
  long long total = 0;
  bool ok = true;
  for (int r = 0; r < reps; ++r) {
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (V == 0) ok = fact_lds(s, H);
    else if constexpr (V == 1) ok = fact_reg(s, H);
    else if constexpr (V == 2) ok = fact_reg2(s, H);
    else {
      ok = fact_iso(s, H);
      __syncthreads();
      iso_gains(s, H);
    }
    wave_lds_fence();
    const long long t1 = __builtin_amdgcn_s_memtime();
    total += t1 - t0;
    __syncthreads();
  }
  if (t == 0) {
    cyc[0] = total;
    cyc[1] = ok;
  }
  for (int e = t; e < H * 8; e += blockDim.x) out[e] = s.Kg[e];
  for (int e = t; e < H * 4; e += blockDim.x) out[H * 8 + e] = s.Ri[e];
}

// host reference (long double), the plain recursion of riccati_factor
static void host_ref(const std::vector<double>& in, int H, std::vector<long double>& Kg, std::vector<long double>& Ri) {
  const double* A = in.data();
  const double* B = in.data() + 16;
  const double* C = in.data() + 24;
  const double* Q = in.data() + 32;
  const double* R = in.data() + 48;
  const double* S = in.data() + 52;
  const double* DU = in.data() + 52 + 3 * H;
  auto qb = [&](int k, int i, int j) -> long double {
    long double S00 = S[k], S01 = S[H + k], S11 = S[2 * H + k];
    return 2.0L * Q[i * 4 + j] + (long double)C[i] * (S00 * C[j] + S01 * C[4 + j]) + (long double)C[4 + i] * (S01 * C[j] + S11 * C[4 + j]);
  };
  long double P[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) P[i][j] = qb(H - 1, i, j);
  Kg.assign(H * 8, 0);
  Ri.assign(H * 4, 0);
  for (int k = H - 1; k >= 0; --k) {
    long double U[4][2] = {}, T[4][4] = {};
    for (int i = 0; i < 4; ++i)
      for (int m = 0; m < 4; ++m) {
        for (int c = 0; c < 2; ++c) U[i][c] += P[i][m] * B[m * 2 + c];
        for (int j = 0; j < 4; ++j) T[i][j] += P[i][m] * A[m * 4 + j];
      }
    long double Re[2][2];
    for (int c = 0; c < 2; ++c)
      for (int d = 0; d < 2; ++d) {
        long double acc = 2.0L * R[c * 2 + d] + (c == d ? DU[k * 2 + c] : 0.0);
        for (int m = 0; m < 4; ++m) acc += B[m * 2 + c] * U[m][d];
        Re[c][d] = acc;
      }
    long double det = Re[0][0] * Re[1][1] - Re[0][1] * Re[1][0];
    long double ri[2][2] = {{Re[1][1] / det, -Re[0][1] / det}, {-Re[1][0] / det, Re[0][0] / det}};
    long double Lm[2][4] = {};
    for (int c = 0; c < 2; ++c)
      for (int j = 0; j < 4; ++j)
        for (int m = 0; m < 4; ++m) Lm[c][j] += B[m * 2 + c] * T[m][j];
    long double K[2][4] = {};
    for (int c = 0; c < 2; ++c)
      for (int j = 0; j < 4; ++j)
        for (int d = 0; d < 2; ++d) K[c][j] += ri[c][d] * Lm[d][j];
    for (int c = 0; c < 2; ++c)
      for (int j = 0; j < 4; ++j) Kg[(k * 2 + c) * 4 + j] = K[c][j];
    for (int c = 0; c < 4; ++c) Ri[k * 4 + c] = ri[c / 2][c % 2];
    if (k > 0) {
      long double Pn[4][4];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          long double acc = qb(k - 1, i, j);
          for (int m = 0; m < 4; ++m) acc += A[m * 4 + i] * T[m][j];
          for (int c = 0; c < 2; ++c) acc -= Lm[c][i] * K[c][j];
          Pn[i][j] = acc;
        }
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) P[i][j] = 0.5L * (Pn[i][j] + Pn[j][i]);
    }
  }
}

int main(int argc, char** argv) {
  const int H = argc > 1 ? std::atoi(argv[1]) : 50;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 200;
  const double wscale = argc > 3 ? std::atof(argv[3]) : 1e3;
  const double dt = 0.2;
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U01(0.0, 1.0);
  for (int trial = 0; trial < 3; ++trial) {
    std::vector<double> in(52 + 5 * H, 0.0);
    double* A = in.data();
    double* B = in.data() + 16;
    double* C = in.data() + 24;
    double* Q = in.data() + 32;
    double* R = in.data() + 48;
    for (int i = 0; i < 4; ++i) A[i * 4 + i] = 1.0;
    A[0 * 4 + 2] = dt;
    A[1 * 4 + 3] = dt;
    B[0 * 2 + 0] = 0.5 * dt * dt;
    B[1 * 2 + 1] = 0.5 * dt * dt;
    B[2 * 2 + 0] = dt;
    B[3 * 2 + 1] = dt;
    if (trial == 2) {  // a dense A, B (general model)
      for (int e = 0; e < 16; ++e) A[e] += 0.05 * (U01(rng) - 0.5);
      for (int e = 0; e < 8; ++e) B[e] += 0.05 * (U01(rng) - 0.5);
    }
    C[0] = 1.0;
    C[4 + 1] = 1.0;
    for (int i = 0; i < 4; ++i) Q[i * 4 + i] = 2.0;
    R[0] = R[3] = 1.0;
    double* S = in.data() + 52;
    double* DU = in.data() + 52 + 3 * H;
    const double ws = trial == 0 ? 1.0 : wscale;
    for (int k = 0; k < H; ++k) {  // S_k = sum of w h h' over a few rows (PSD)
      double s00 = 0, s01 = 0, s11 = 0;
      for (int r = 0; r < 3; ++r) {
        const double th = 6.283 * U01(rng), w = ws * std::pow(10.0, 4.0 * U01(rng) - 2.0);
        s00 += w * std::cos(th) * std::cos(th);
        s01 += w * std::cos(th) * std::sin(th);
        s11 += w * std::sin(th) * std::sin(th);
      }
      S[k] = s00;
      S[H + k] = s01;
      S[2 * H + k] = s11;
      DU[2 * k] = ws * 1e-2 * U01(rng);
      DU[2 * k + 1] = ws * 1e-2 * U01(rng);
    }
    std::vector<long double> Kr, Rr;
    host_ref(in, H, Kr, Rr);
    double *din, *dout;
    long long* dcyc;
    CHECK(hipMalloc(&din, in.size() * 8));
    CHECK(hipMalloc(&dout, H * 12 * 8));
    CHECK(hipMalloc(&dcyc, 16));
    CHECK(hipMemcpy(din, in.data(), in.size() * 8, hipMemcpyHostToDevice));
    for (int v = 0; v < 4; ++v) {
      if (v == 3 && trial == 2) continue;  // (the isotropic form needs the block structure)
      const size_t lds = kLdsDoubles * 8;
      if (v == 0) bench<0><<<1, 512, lds>>>(din, dout, dcyc, H, reps);
      else if (v == 1) bench<1><<<1, 512, lds>>>(din, dout, dcyc, H, reps);
      else if (v == 2) bench<2><<<1, 512, lds>>>(din, dout, dcyc, H, reps);
      else bench<3><<<1, 512, lds>>>(din, dout, dcyc, H, reps);
      CHECK(hipGetLastError());
      CHECK(hipDeviceSynchronize());
      std::vector<double> out(H * 12);
      long long cyc[2];
      CHECK(hipMemcpy(out.data(), dout, H * 12 * 8, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(cyc, dcyc, 16, hipMemcpyDeviceToHost));
      double ek = 0, er = 0;
      for (int e = 0; e < H * 8; ++e)
        ek = std::fmax(ek, (double)(std::fabs(out[e] - (double)Kr[e]) / (1e-300 + std::fabs((double)Kr[(e / 8) * 8]) + std::fabs((double)Kr[(e / 8) * 8 + 4]) + std::fabs((double)Kr[e]))));
      for (int e = 0; e < H * 4; ++e)
        er = std::fmax(er, (double)(std::fabs(out[H * 8 + e] - (double)Rr[e]) / (std::fabs((double)Rr[(e / 4) * 4]) + std::fabs((double)Rr[(e / 4) * 4 + 3]))));
      std::printf("trial %d (%s, weights x%g) %s: %.1f cycles/step, ok %lld, max rel err Kg %.2e Ri %.2e\n", trial,
                  trial == 2 ? "dense A,B" : "double integrator", ws, v == 0 ? "LDS form     " : v == 1 ? "register form" : v == 2 ? "M-form       " : "isotropic    ",
                  (double)cyc[0] / reps / H, cyc[1], ek, er);
    }
    CHECK(hipFree(din));
    CHECK(hipFree(dout));
    CHECK(hipFree(dcyc));
  }
  return 0;
}
