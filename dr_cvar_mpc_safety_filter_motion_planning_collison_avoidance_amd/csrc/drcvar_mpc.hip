// drcvar_mpc.hip — the MPC safety-filter QP that consumes the safe halfspaces, for gfx950.
//
// Reference: core/mpc_filter.py:40-178 (MPCSafetyFilter.filter_trajectory) builds, per call, a
// CVXPY problem over x [H+1, nx], u [H, nu] and one slack per halfspace, solves it with the default
// QP solver and falls back to a rolled-out input sequence (_fallback, :180-219) when the solve does
// not succeed.  Here every problem of a batch is one workgroup that runs a primal-dual Mehrotra
// interior-point method to convergence without leaving the device.
//
// Formulation (input space; the dynamics are eliminated once on the host, drcvar_mpc_model_init):
//   positions  p_{k+1} = c_k + sum_{j<=k} Mp[k-j] u_j,  Mp[i] = C A^i B,  c_k = C A^{k+1} x0
//   objective  1/2 u'H0 u + f'u + sum_r 50 s_r + 50 s_r^2,  H0 = 2(Gx'QGx + R), f = F1 x0 - F2 xr
//   rows       halfspace r (step k):   h.p_{k+1} + g - s_r <= 0      (w_hs, lambda_hs)
//              slack sign:             -s_r <= 0                      (w_s,  lambda_s)
//              input box (optional):   u_j - u_max <= 0, u_min - u_j <= 0
//              position box (optional): p - p_max <= 0, p_min - p <= 0 (per step and coordinate)
// Newton system: the slack columns are diagonal and are eliminated per row, so the halfspaces of
// step k reach the input-space Hessian only through the 2x2 matrix S_k = sum_r omega_r h_r h_r'
// and the right-hand side through a 2-vector per step:
//   K = H0 + diag(D_box) + sum_k Mp_k' S_k Mp_k    (n x n, n = nu*H <= 120)
// K is never formed: it is the Hessian of a linear-quadratic problem over the horizon, so each
// Newton system is solved by a Riccati recursion (O(H nx^3), see riccati_factor) — the
// per-iteration cost is O(rows) streaming + O(H nx^3), independent of the number of obstacles.  Rows live in a per-problem workspace ([O, 64] SoA arrays, lane = halfspace step, so
// every row pass is a coalesced sweep); per-step sums are combined across waves in a fixed order,
// so the solver is deterministic.
//
// Iteration (Mehrotra predictor-corrector, identical to oracle-independent prototype
// scripts/mpc_condensed_proto.py):
//   P1 residuals, weights, per-step S / v / affine z          -> r_du, convergence test
//   Riccati factorisation; affine direction (solve); P2 affine step length
//   P3 affine gap + corrector rhs split as base + sigma*mu*unit; corrector direction (solve)
//   P4 corrector step length; P5 update (step 0.995 of the way to the boundary)
// Affine directions of a row are recomputed from (state, dp_aff) instead of being stored.

#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "drcvar_mpc.h"

// Build parts (compile time of the kernel templates): without DRCVAR_MPC_PART this file is the
// whole library part; with -DDRCVAR_MPC_PART=0 only the host code (model condensing, queries,
// argument checks), with -DDRCVAR_MPC_PART=k (1..4) only the kernels of the k-input models and
// their launcher.  _native.build() compiles the five parts concurrently.
#if !defined(DRCVAR_MPC_PART)
#define DRCVAR_MPC_HOST_PART 1
#define DRCVAR_MPC_DEVICE_PART(k) 1
#else
#define DRCVAR_MPC_HOST_PART (DRCVAR_MPC_PART == 0)
#define DRCVAR_MPC_DEVICE_PART(k) (DRCVAR_MPC_PART == (k))
#endif
#define DRCVAR_MPC_ANY_DEVICE_PART \
  (DRCVAR_MPC_DEVICE_PART(1) || DRCVAR_MPC_DEVICE_PART(2) || DRCVAR_MPC_DEVICE_PART(3) || DRCVAR_MPC_DEVICE_PART(4))

// types shared by the parts (the launch arguments cross from the host part to the kernel parts)
namespace drcvar_mpc_detail {

struct BlobLayout {
  int64_t H0, F1, F2, Mp, CA, A, B, C, Q, R, UF1, UF2, UFOK, ISO, total;
};

inline BlobLayout blob_layout(int nx, int nu, int H) {
  const int64_t n = static_cast<int64_t>(nu) * H;
  BlobLayout L{};
  int64_t o = 0;
  L.H0 = o; o += n * n;
  L.F1 = o; o += n * nx;
  L.F2 = o; o += n * H * nx;
  L.Mp = o; o += static_cast<int64_t>(H) * 2 * nu;
  L.CA = o; o += static_cast<int64_t>(H) * 2 * nx;
  L.A = o; o += nx * nx;
  L.B = o; o += nx * nu;
  L.C = o; o += 2 * nx;
  L.Q = o; o += nx * nx;
  L.R = o; o += nu * nu;
  // the tracking optimum without rows, u_free = -H0^-1 f = UF1 x0 + UF2 xr (the starting point):
  // UF1 = -H0^-1 F1 [n x nx], UF2 = H0^-1 F2 [n x H*nx]; UFOK = 1 when H0 factored (else u = 0)
  L.UF1 = o; o += n * nx;
  L.UF2 = o; o += n * H * nx;
  L.UFOK = o; o += 1;
  // 1 for a planar isotropic model (nx = 4, nu = 2, A = [[a00 I, a01 I], [a10 I, a11 I]],
  // B = [[b0 I], [b1 I]]: the reference's double integrator): the register-form factorisation
  L.ISO = o; o += 1;
  L.total = o;
  return L;
}

struct MpcArgs {
  const double* blob;
  BlobLayout off;
  int nx, nu, H, n, K, O;
  int has_u, has_p;
  double umin[DRCVAR_MPC_MAX_INPUTS], umax[DRCVAR_MPC_MAX_INPUTS], pmin[2], pmax[2];
  const double* hs_h;
  const double* hs_g;
  int64_t h_sp, h_so, h_sk, g_sp, g_so, g_sk;
  const double* x0;
  int64_t x0_sp;
  const double* xr;
  int64_t xr_sp, xr_st;
  const double* uf;
  int64_t uf_sp, uf_st;
  double* x_out;
  double* u_out;
  double* info;
  double* ws;
  int64_t ws_off, ws_pp;  // per-problem region b at ws + ws_off + b * ws_pp
  int cl_size;            // workgroups per problem (clustered form)
  uint64_t spin_ticks;    // bound of one cluster wait, in ticks of the 100 MHz s_memrealtime clock
  // test hooks (drcvar_mpc_options.debug_*; 0 = off): the first polish makes no attempt; workgroup
  // perturb_group - 1 scales its step length at iteration perturb_iter; workgroup stall_group - 1
  // leaves before the final exchange
  int force_resume, perturb_group, perturb_iter, stall_group;
  int max_iter;
  double tol;
  int polish;
};

// one launcher per input count, each defined in its own part
int launch_nu1(const MpcArgs& args, int64_t n_problems, hipStream_t stream);
int launch_nu2(const MpcArgs& args, int64_t n_problems, hipStream_t stream);
int launch_nu3(const MpcArgs& args, int64_t n_problems, hipStream_t stream);
int launch_nu4(const MpcArgs& args, int64_t n_problems, hipStream_t stream);
int device_cus();

}  // namespace drcvar_mpc_detail

namespace {
using namespace drcvar_mpc_detail;

// Threads per problem: 256 for batches (two workgroups per CU), 512 for launches of a few
// problems (two waves per SIMD hide the row passes' fp64 latency; the chip has CUs to spare).
// Device code below is written against kBlock / kWaves, which the kernel defines from its
// BLK parameter; helpers take the wave count as a template argument.
constexpr int kMaxWaves = 8;
constexpr int kFewProblems = 128;  // at most this many problems per launch: 512-thread form
constexpr int kShortHorizon = 32;  // horizon capacity of the 128-thread (many problems) form
constexpr int kStepPad = 64;  // workspace pitch: one lane per halfspace step
// h0, h1, g, s, w_hs, lambda_hs, w_s, lambda_s, then s and w_hs saved across a failed polish
constexpr int kRowArrays = 10;
// per workgroup: the best iterate u (n <= DRCVAR_MPC_MAX_DECISION, padded to 128), then the bound
// states saved across a failed polish (bx [4 n], px [8 H]: <= 992)
constexpr int kBestPad = 128 + 1024;
constexpr int kRowStride = kRowArrays * kStepPad;  // one obstacle's block of the workspace
constexpr double kSlackLin = 50.0;    // core/mpc_filter.py:143
constexpr double kSlackHess = 100.0;  // d^2/ds^2 of 50 s^2, core/mpc_filter.py:144
constexpr double kStepFrac = 0.995;
constexpr double kHuge = 1e300;
constexpr int kPerStepQ = 7;          // per-step partial sums carried by one reduction
constexpr double kPolishRho = 1e6;    // method-of-multipliers penalty of the polish
constexpr int kPolishIters = 12;      // multiplier passes per active-set guess
constexpr int kPolishAttempts = 6;    // active-set corrections
constexpr double kPolishMerit = 1e-5; // polish only from an iterate this close to the optimum
// early polish (round 6): the first round polishes as soon as its merit is <= kEarlyPolishMerit,
// from the predictor's active-set guess at that iterate, with at most kEarlyPolishAttempts
// corrections; the polish certifies itself (sign conditions and equality residuals), and one that
// fails restores the iterate and resumes the interior-point method to the tolerance.  Round 5 did
// this only on a stall (merit fallen less than tenfold over two iterations: the straggler of
// tests/golden/qp_h30_straggler.npz); polishing every problem from 1e-2 instead of iterating to
// tol = 1e-7 first (scripts/micro/patches/early_polish_knobs.diff, interleaved on one box,
// profiles/r06/early_polish/): the C5 fixture 10 -> 8 iterations, 0.574 -> 0.478 ms; main.py's
// mean filter 15 -> 12, 0.785 -> 0.681 ms; the straggler 11 -> 7; 1 024 distinct problems 0.405 ->
// 0.341 ms (mean 5.3 -> 3.3 iterations); every problem optimal and polished, |u - oracle| <= 7e-10.
// From 3e-2 the guess failed on the mean filter (three attempts, then the resume: 1.02 ms); with
// two attempts from 1e-2 one problem of the 1 024 needed the resume (0.420 ms); 1e-3 / 3e-3 /
// 1e-4 polish one or two iterations later.  With many halfspace rows (kManyRowsObstacles) the
// threshold is 1.5e-2 (profiles/r06/early_polish/r6_final_thresholds/): the C5 fixture 8 -> 7
// iterations, 0.479 -> 0.443 ms; main.py's mean filter and the synthetic C5 problems unchanged.
// Few rows keep 1e-2: from 1.5e-2 the 1 024-problem batch slows 0.342 -> 0.384 ms.
constexpr double kEarlyPolishMerit = 1e-2;
constexpr double kEarlyPolishMeritMany = 1.5e-2;
constexpr int kEarlyPolishAttempts = 3;  // active-set corrections of an early polish
constexpr double kPolishDualTol = 1e-7;
constexpr int kManyRowsObstacles = 64;  // interior-point start for many halfspace rows (below)
constexpr double kStartMuMany = 20.0;   // barrier parameter of the starting point, >= 64 obstacles
constexpr double kStartMuFew = 1.0;     // ... fewer obstacles
constexpr double kStartDualCap = 0.5 * kSlackLin;  // largest starting lambda_hs
constexpr double kStartBoxMargin = 0.05;  // starting inputs at least this fraction of the box inside
constexpr double kStartFloorW = 1e-2;     // smallest starting slack of a bound row
constexpr int kResumeIters = 8;         // interior-point iterations after a failed polish
constexpr double kResumeTol = 1e-3;     // ... towards tol * kResumeTol
constexpr double kPolishEqTol = 1e-12;  // multiplier passes stop at |E u - e| <= this * (1 + max|g|)

// clustered form (see cluster_combine)
constexpr int kClusterMaxProblems = 8;
constexpr int kClusterMinObstacles = 64;
constexpr int kClusterObstaclesPerGroup = 16;  // C5: 16 workgroups (8..32 measured within 4 %)
constexpr int kClusterMax = 32;
// threads per workgroup of the clustered form (256 measured 3-7 % slower at every shape)
constexpr int kClusterBlock = 512;
constexpr int kClusterCUs = 256;  // workspace sizing; launches use the device's own CU count
constexpr int kRec = 512;                        // doubles per exchange record
constexpr int kRecScalars = kPerStepQ * 64;      // [kPerStepQ][64] per-step sums, then scalars
constexpr int kRecDigest = kRecScalars + 8;      // the publishing workgroup's state digest
constexpr int kCtrlDoubles = 16;                 // 128-B control block per problem (the counter)
constexpr int kClusterScratch = kMaxWaves * 4 + 8;  // LDS doubles of the exchange
constexpr int kCxGaveUp = kMaxWaves * 4, kCxScalars = kMaxWaves * 4 + 1, kCxDiverged = kMaxWaves * 4 + 5;
static_assert(kCxDiverged < kClusterScratch, "exchange scratch");
constexpr unsigned long long kAbortBias = 1ull << 40;
constexpr int kDefaultSpinUs = 10000;            // 10 ms: a C5 solve is ~1 ms
enum { kOpSum = 0, kOpMax = 1, kOpMin = 2 };
// exchange sites (mixed into the published digest)
enum { kSiteStart = 1, kSiteP1, kSiteP23, kSiteP4, kSitePolishHess, kSitePolishRhs, kSitePolishEq,
       kSitePolishSign, kSitePolishBad, kSiteFinal };

#ifdef DRCVAR_MPC_STAMPS
// diagnostic build only: per-category shader-clock totals of problem 0..kStampProblems-1
constexpr int kStampProblems = 64, kStampSlots = 20;
__device__ unsigned long long g_mpc_stamps[kStampProblems * kStampSlots];
__device__ unsigned long long g_cl_stamps[8];  // cluster exchange sub-phases, problem 0, group 0
// per workgroup of problem 0's cluster (index cl.id < 32), summed over its exchanges: the 100 MHz
// clock at its arrival and at its release, and the count — relative arrival order over the cluster
__device__ unsigned long long g_cl_arrive[3 * 32];
// per-wave spans of the P1 phase (workgroup 0 of problem 0): [wave][0] = cycles from the barrier
// before the factorisation to the wave's end of its P1 work, summed over iterations; [wave][1] = count
__device__ unsigned long long g_wave_stamps[16];
#define WAVE_SPAN_BEGIN() const unsigned long long wspan0_ = __builtin_amdgcn_s_memtime()
#define WAVE_SPAN_END()                                                                     \
  do {                                                                                      \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (threadIdx.x >> 6) < 8) {              \
      atomicAdd(&g_wave_stamps[2 * (threadIdx.x >> 6)], __builtin_amdgcn_s_memtime() - wspan0_); \
      atomicAdd(&g_wave_stamps[2 * (threadIdx.x >> 6) + 1], 1ull);                          \
    }                                                                                       \
  } while (0)
#define CL_STAMP(k)                                                     \
  do {                                                                  \
    if (threadIdx.x == 0 && blockIdx.x == 0) {                          \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();     \
      g_cl_stamps[(k)] += now_ - cl_t0;                                 \
      cl_t0 = now_;                                                     \
    }                                                                   \
  } while (0)
#define MPC_PHASE(k)                                                    \
  do {                                                                  \
    if (threadIdx.x == 0) {                                             \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();     \
      stamp_acc[(k)] += now_ - stamp_last;                              \
      stamp_last = now_;                                                \
    }                                                                   \
  } while (0)
#else
#define CL_STAMP(k) \
  do {              \
  } while (0)
#define MPC_PHASE(k) \
  do {               \
  } while (0)
#define WAVE_SPAN_BEGIN() \
  do {                    \
  } while (0)
#define WAVE_SPAN_END() \
  do {                  \
  } while (0)
#endif

#if DRCVAR_MPC_ANY_DEVICE_PART
// LDS arrays (doubles); offsets from LdsPlan below.
struct Lds {
  double* Am;     // [nx][kMx] A          (model, copied from the blob at setup)
  double* Bm;     // [nx][NU] B
  double* Cm;     // [2][kMx] C
  double* Qm;     // [nx][kMx] Q
  double* Rm;     // [NU][NU] R
  double* P;      // [nx][kMx] Riccati cost-to-go
  double* T;      // [nx][kMx] P A
  double* U;      // [nx][NU] P B
  double* Kg;     // [H][NU][NX] feedback gains Re^-1 B'PA
  double* Ri;     // [H][NU][NU] Re^-1
  double* SM;     // [H][NX][NX] solve maps F_k = A' - Kg_k' B' (NX <= 4)
  double* SV;     // [H + 1][NX] solve recurrences' sources and states (NX <= 4)
  double* u;      // [n] inputs (the iterate)
  double* dua;    // [n] affine direction
  double* du;     // [n] corrector direction
  double* rdu;    // [n] dual residual of the inputs
  double* f;      // [n] linear cost
  double* DU;     // [n] box weights
  double* rU;     // [n] box rhs term (affine, then corrector base)
  double* rUu;    // [n] box rhs term (corrector unit)
  double* bx;     // [4][n] box state wUu, lUu, wUl, lUl
  double* c;      // [2H] free-response positions
  double* p;      // [2H] positions of the iterate
  double* dpa;    // [2H] affine position direction
  double* dp;     // [2H] corrector position direction
  double* v;      // [2H] per-step sum of lambda_hs h (+ position-box duals)
  double* za;     // [2H] per-step affine rhs, then corrector base
  double* zu;     // [2H] per-step corrector unit
  double* px;     // [4][2H] position-box state wPu, lPu, wPl, lPl
  double* S;      // [3][H] per-step 2x2 weights (S00, S01, S11)
  double* Mp;     // [H][2][NU] C A^i B
  double* xs;     // [H+1][nx] rollout
  double* red;    // [kWaves][kPerStepQ][64] per-step partial sums
  double* sc;     // [64] block scalars
  bool iso;       // planar isotropic model (blob ISO): riccati_factor_iso
};

// Fixed LDS plan per size class: every array sits at a compile-time offset, so LDS addresses are
// immediates and no scalar registers hold array bases.  One plan covers every model (n <= NMAX =
// DRCVAR_MPC_MAX_DECISION, H <= HM = DRCVAR_MPC_MAX_HORIZON): with the Riccati recursion there is
// no n x n matrix, and the plan stays under 80 KB (two workgroups per CU).
constexpr int kMx = DRCVAR_MPC_MAX_STATES;  // row stride of the state-dimension matrices in LDS
constexpr int kMu = DRCVAR_MPC_MAX_INPUTS;
// NW waves per workgroup (the per-step partial sums), NU inputs and NX (padded) states (the
// per-step Riccati factors and, for NX <= 4, the parallel-scan buffers)
template <int NW, int NU, int NX, int HMX = DRCVAR_MPC_MAX_HORIZON>
struct LdsPlan {
  static constexpr int HM = HMX;  // horizon capacity of the plan
  static constexpr int NMAX = NU * HM < DRCVAR_MPC_MAX_DECISION ? NU * HM : DRCVAR_MPC_MAX_DECISION;
  static constexpr int Am = 0;
  static constexpr int Bm = Am + kMx * kMx;
  static constexpr int Cm = Bm + kMx * kMu;
  static constexpr int Qm = Cm + 2 * kMx;
  static constexpr int Rm = Qm + kMx * kMx;
  static constexpr int P = Rm + kMu * kMu;
  static constexpr int T = P + kMx * kMx;
  static constexpr int U = T + kMx * kMx;
  static constexpr int Kg = U + kMx * kMu;
  static constexpr int Ri = Kg + HM * NU * NX;
  static constexpr int SM = Ri + HM * NU * NU;                   // solve: [HM][NX][NX] maps
  static constexpr int SV = SM + (NX <= 4 ? HM * NX * NX : 0);   // solve: [HM + 1][NX] vectors
  static constexpr int u = SV + (NX <= 4 ? (HM + 1) * NX : 0);
  static constexpr int dua = u + NMAX;
  static constexpr int du = dua + NMAX;
  static constexpr int rdu = du + NMAX;
  static constexpr int f = rdu + NMAX;
  static constexpr int DU = f + NMAX;
  static constexpr int rU = DU + NMAX;
  static constexpr int rUu = rU + NMAX;
  static constexpr int bx = rUu + NMAX;
  static constexpr int c = bx + 4 * NMAX;
  static constexpr int p = c + 2 * HM;
  static constexpr int dpa = p + 2 * HM;
  static constexpr int dp = dpa + 2 * HM;
  static constexpr int v = dp + 2 * HM;
  static constexpr int za = v + 2 * HM;
  static constexpr int zu = za + 2 * HM;
  static constexpr int px = zu + 2 * HM;
  static constexpr int S = px + 8 * HM;
  static constexpr int Mp = S + 3 * HM;
  static constexpr int xs = Mp + 2 * DRCVAR_MPC_MAX_INPUTS * HM;
  static constexpr int red = xs + (HM + 1) * DRCVAR_MPC_MAX_STATES;
  static constexpr int sc = red + NW * kPerStepQ * 64;
  static constexpr int total = sc + 64;
};
static_assert(LdsPlan<4, 4, 4>::total * 8 <= 80 * 1024, "256-thread plan: two workgroups per CU");
static_assert(LdsPlan<4, 4, 8>::total * 8 <= 80 * 1024, "256-thread plan: two workgroups per CU");
static_assert(LdsPlan<8, 4, 8>::total * 8 <= 160 * 1024, "512-thread plan exceeds the LDS");
static_assert(LdsPlan<2, 2, 4, kShortHorizon>::total * 8 <= 40 * 1024,
              "128-thread short-horizon plan, two inputs: four workgroups per CU");
static_assert(LdsPlan<2, 4, 4, kShortHorizon>::total * 8 <= 160 * 1024 / 3 &&
                  LdsPlan<2, 4, 8, kShortHorizon>::total * 8 <= 160 * 1024 / 3,
              "128-thread short-horizon plan: at least three workgroups per CU");

template <int NW, int NU, int NX, int HMX>
__device__ inline Lds carve(double* base, bool iso) {
  using P = LdsPlan<NW, NU, NX, HMX>;
  Lds s;
  s.iso = NU == 2 && NX == 4 && iso;
  s.Am = base + P::Am;
  s.Bm = base + P::Bm;
  s.Cm = base + P::Cm;
  s.Qm = base + P::Qm;
  s.Rm = base + P::Rm;
  s.P = base + P::P;
  s.T = base + P::T;
  s.U = base + P::U;
  s.Kg = base + P::Kg;
  s.Ri = base + P::Ri;
  s.SM = base + P::SM;
  s.SV = base + P::SV;
  s.u = base + P::u;
  s.dua = base + P::dua;
  s.du = base + P::du;
  s.rdu = base + P::rdu;
  s.f = base + P::f;
  s.DU = base + P::DU;
  s.rU = base + P::rU;
  s.rUu = base + P::rUu;
  s.bx = base + P::bx;
  s.c = base + P::c;
  s.p = base + P::p;
  s.dpa = base + P::dpa;
  s.dp = base + P::dp;
  s.v = base + P::v;
  s.za = base + P::za;
  s.zu = base + P::zu;
  s.px = base + P::px;
  s.S = base + P::S;
  s.Mp = base + P::Mp;
  s.xs = base + P::xs;
  s.red = base + P::red;
  s.sc = base + P::sc;
  return s;
}

// ---- reductions (butterflies: every lane ends with the bitwise-identical value) ----
// DPP row permutations (each an involution: quad xor 1, quad xor 2, half mirror, mirror) combine
// within rows of 16 lanes, then the gfx950 lane swaps (permlane16 / permlane32) combine the rows;
// no LDS on the chain (the __shfl_xor butterfly is six ds_bpermute round trips).  Every lane of
// the wave must be active.
template <int CTRL>
__device__ __forceinline__ double dpp_row_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <class F>
__device__ __forceinline__ double wave_butterfly(double v, F op) {
  v = op(v, dpp_row_f64<0xB1>(v));   // quad_perm [1,0,3,2]
  v = op(v, dpp_row_f64<0x4E>(v));   // quad_perm [2,3,0,1]
  v = op(v, dpp_row_f64<0x141>(v));  // row_half_mirror
  v = op(v, dpp_row_f64<0x140>(v));  // row_mirror
  {
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = op(__hiloint2double(hi[0], lo[0]), __hiloint2double(hi[1], lo[1]));
  }
  {
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = op(__hiloint2double(hi[0], lo[0]), __hiloint2double(hi[1], lo[1]));
  }
  return v;
}
// Lane moves of the register-form factorisation (riccati_factor_iso): a DPP permutation within
// rows of 16 lanes (two v_mov_b32_dpp), lane n of each row to the whole row (one v_mov_b64_dpp
// row_newbcast, gfx950), and an arbitrary source lane (ds_bpermute: the LDS crossbar, ~75 cycles)
template <int CTRL>
__device__ __forceinline__ double dpp_mov_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int N>
__device__ __forceinline__ double row_bcast_f64(double v) {
  const long long x = __builtin_bit_cast(long long, v);
  const long long y = __builtin_amdgcn_mov_dpp(x, 0x150 + N, 0xF, 0xF, false);
  return __builtin_bit_cast(double, y);
}
__device__ __forceinline__ double bperm_f64(double v, int byte_addr) {
  const int lo = __builtin_amdgcn_ds_bpermute(byte_addr, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(byte_addr, __double2hiint(v));
  return __hiloint2double(hi, lo);
}
// separately rounded product and sum (never contracted into an fma): the symmetric-exact sums of
// riccati_factor_iso rely on a * b == b * a and a + b == b + a bit for bit
__device__ __forceinline__ double mul_rn(double a, double b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ double add_rn(double a, double b) {
#pragma clang fp contract(off)
  return a + b;
}

// The interior-point block sums keep the xor butterfly (distances 32, 16, ..., 1): the DPP tree
// associates the sum differently, and that rounding was enough to turn one degenerate test
// instance (generic1, H = 64, more binding rows than inputs) from a successful polish into an
// OPTIMAL_INACCURATE answer.  Max / min are exact in any order and take the DPP form; the cluster
// exchange's sums (a new code path) take the DPP form too.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  return wave_butterfly(v, [](double a, double b) { return a + b; });
}
__device__ __forceinline__ double wave_max(double v) {
  return wave_butterfly(v, [](double a, double b) { return fmax(a, b); });
}
__device__ __forceinline__ double wave_min(double v) {
  return wave_butterfly(v, [](double a, double b) { return fmin(a, b); });
}

// Three block-wide reductions (sum, max, max) in one LDS round trip; waves combined in order.
template <int kWaves>
__device__ inline void block_sum_max_max(double& a, double& b, double& c, double* sc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  a = wave_sum(a);
  b = wave_max(b);
  c = wave_max(c);
  if (lane == 0) {
    sc[wave] = a;
    sc[kWaves + wave] = b;
    sc[2 * kWaves + wave] = c;
  }
  __syncthreads();
  a = sc[0];
  b = sc[kWaves];
  c = sc[2 * kWaves];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) {
    a += sc[w];
    b = fmax(b, sc[kWaves + w]);
    c = fmax(c, sc[2 * kWaves + w]);
  }
  __syncthreads();
}

template <int kWaves>
__device__ inline double block_min(double a, double* sc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  a = wave_min(a);
  if (lane == 0) sc[3 * kWaves + wave] = a;
  __syncthreads();
  double r = sc[3 * kWaves];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) r = fmin(r, sc[3 * kWaves + w]);
  __syncthreads();
  return r;
}

template <int kWaves>
__device__ inline double block_sum(double a, double* sc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  a = wave_sum(a);
  if (lane == 0) sc[4 * kWaves + wave] = a;
  __syncthreads();
  double r = sc[4 * kWaves];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) r += sc[4 * kWaves + w];
  __syncthreads();
  return r;
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// 1/x from the hardware estimate plus one Newton step (~1 ulp; the IEEE division sequence is
// ~10 dependent instructions and the row passes perform a dozen per halfspace row)
__device__ __forceinline__ double rcp(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(r, fma(-x, r, 1.0), r);
}

// step-to-boundary ratio; only feeds the 0.995 fraction of the step length, so the raw estimate
__device__ __forceinline__ double ratio(double x, double dx) {
  return dx < 0.0 ? -x * __builtin_amdgcn_rcp(dx) : kHuge;
}

// Central-path slack of a halfspace row with residual r at barrier parameter mu: the root s >
// max(r, 0) of g(s) = (50 + 100 s)(s - r) s - mu (2 s - r), i.e. 50 + 100 s = mu / (s - r) + mu / s.
// g is convex and increasing beyond max(r, 0) (g'' = 600 s + 100 - 200 r > 0 there) and
// g(max(r, 0)) <= 0, so Newton's method from a point where g > 0 (s0 = max(r, 0) + 1 + mu / 50, for
// mu <= 75) decreases monotonically to the root and never leaves (max(r, 0), s0].
__device__ inline double start_slack(double r, double mu) {
  double sv = fmax(r, 0.0) + 1.0 + mu * (1.0 / kSlackLin);
  for (int i = 0; i < 60; ++i) {
    const double a = kSlackLin + kSlackHess * sv, b = sv - r;
    const double gv = a * b * sv - mu * (2.0 * sv - r);
    const double gd = kSlackHess * b * sv + a * (2.0 * sv - r) - 2.0 * mu;
    const double step = gv / gd;
    sv -= step;
    if (!(step > 1e-14 * sv)) break;  // converged (or not finite: stop)
  }
  return sv;
}

// p[2k+i] = c[2k+i] + sum_{j<=k} Mp[k-j][i][:] . u[j*nu : (j+1)*nu].  The sum over j is split
// into PARTS interleaved partial sums (threads (t, part)), combined in a fixed order through the
// per-step scratch s.red — a chain of k/PARTS instead of k dependent steps.  The caller
// synchronises after (s.red is free at every call site).
template <int NU, int kBlock>
__device__ inline void positions(const Lds& s, const double* u, double* out, const double* c, int H) {
  constexpr int PARTS = kBlock >= 512 ? 4 : 2;
  double* part_sum = s.red;  // [2H][PARTS]
  for (int e = threadIdx.x; e < 2 * H * PARTS; e += kBlock) {
    const int t = e / PARTS, part = e - (e / PARTS) * PARTS;
    const int k = t >> 1, i = t & 1;
    double acc = 0.0;
    for (int j = part; j <= k; j += PARTS) {
      const double* m = s.Mp + ((k - j) * 2 + i) * NU;
#pragma unroll
      for (int a = 0; a < NU; ++a) acc += m[a] * u[j * NU + a];
    }
    part_sum[e] = acc;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * H; t += kBlock) {
    double acc = c ? c[t] : 0.0;
#pragma unroll
    for (int part = 0; part < PARTS; ++part) acc += part_sum[t * PARTS + part];
    out[t] = acc;
  }
}

// out[j*nu+a] (+)= sum_{k>=j} sum_i Mp[k-j][i][a] z[2k+i]
template <int NU>
__device__ inline double gp_transpose(const Lds& s, const double* z, int j_a, int H) {
  const int j = j_a / NU, a = j_a - j * NU;
  double acc = 0.0;
  for (int k = j; k < H; ++k) {
    const double* m = s.Mp + (k - j) * 2 * NU;
    acc += m[a] * z[2 * k] + m[NU + a] * z[2 * k + 1];
  }
  return acc;
}

// Gp' z (and, with H0row, H0 u as well) as interleaved partial sums: part_sum[j * PARTS + part]
// holds the terms k - j = part, part + PARTS, ... (and l = part, part + PARTS, ... of the H0 row),
// so no thread carries a chain longer than ~H / PARTS; the caller combines the parts in order.
template <int NU, int kBlock>
__device__ inline void gpt_parts(const Lds& s, const double* z, const double* H0, const double* u,
                                 double* part_sum, int n, int H) {
  constexpr int PARTS = kBlock >= 512 ? 4 : 2;
  for (int e = threadIdx.x; e < n * PARTS; e += kBlock) {
    const int j_a = e / PARTS, part = e - (e / PARTS) * PARTS;
    const int j = j_a / NU, a = j_a - (j_a / NU) * NU;
    double acc = 0.0;
    for (int k = j + part; k < H; k += PARTS) {
      const double* m = s.Mp + (k - j) * 2 * NU;
      acc += m[a] * z[2 * k] + m[NU + a] * z[2 * k + 1];
    }
    if (H0) {
      const double* h0r = H0 + static_cast<int64_t>(j_a) * n;
      for (int l = part; l < n; l += PARTS) acc += h0r[l] * u[l];
    }
    part_sum[e] = acc;
  }
}
// One thread's (Gp' z)[j_a] (+ (H0 u)[j_a] with H0), summed exactly as gpt_parts + parts_total do
// it (the PARTS interleaved partial sums, combined in order): the same bits from one thread, for
// the waves that form the affine rhs beside the factorisation
template <int NU, int kBlock>
__device__ inline double gpt_row(const Lds& s, const double* z, const double* H0, const double* u,
                                 int j_a, int n, int H) {
  constexpr int PARTS = kBlock >= 512 ? 4 : 2;
  const int j = j_a / NU, a = j_a - (j_a / NU) * NU;
  double tot = 0.0;
#pragma unroll
  for (int part = 0; part < PARTS; ++part) {
    double acc = 0.0;
    for (int k = j + part; k < H; k += PARTS) {
      const double* m = s.Mp + (k - j) * 2 * NU;
      acc += m[a] * z[2 * k] + m[NU + a] * z[2 * k + 1];
    }
    if (H0) {
      const double* h0r = H0 + static_cast<int64_t>(j_a) * n;
      for (int l = part; l < n; l += PARTS) acc += h0r[l] * u[l];
    }
    tot = part == 0 ? acc : tot + acc;
  }
  return tot;
}

template <int kBlock>
__device__ __forceinline__ double parts_total(const double* part_sum, int j) {
  constexpr int PARTS = kBlock >= 512 ? 4 : 2;
  double acc = part_sum[j * PARTS];
#pragma unroll
  for (int part = 1; part < PARTS; ++part) acc += part_sum[j * PARTS + part];
  return acc;
}

// ---------------------------------------------------------------------------------------------
// Newton systems by Riccati recursion.  The condensed Hessian
//   K = blockdiag(2R + diag(DU_k)) + Gx' blockdiag(2Q + C'S_k C) Gx
// is never formed: K du = b is the optimality condition of the linear-quadratic problem
//   min 1/2 sum_k (x_{k+1}'Qb_{k+1} x_{k+1} + du_k'Rb_k du_k) - b'du,  x_{k+1} = A x_k + B du_k,
//   x_0 = 0,  Qb_{k+1} = 2Q + C'S_k C,  Rb_k = 2R + diag(DU_k),
// solved by the backward recursion (P_H = Qb_H)
//   Re_k = Rb_k + B'P B,  L_k = B'P A,  Kg_k = Re_k^-1 L_k,  P_k = Qb_k + A'P A - L_k'Kg_k
// and, per right-hand side, p_H = 0, ge_k = B'p - b_k, kff_k = -Re_k^-1 ge_k, p_k = A'p - Kg_k'ge_k
// followed by the forward pass du_k = kff_k - Kg_k x_k, x_{k+1} = A x_k + B du_k.
// O(H nx^3) per factorisation and O(H nx^2) per solve instead of O(n^3) / O(n^2), and no n x n
// matrix in LDS.  P is formed from its lower triangle and mirrored, so it is exactly symmetric (an
// unsymmetrised recursion drifts: ~1e-4 relative error at H = 50 in the prototype, 1e-12 with).
// Near an interior-point solution Re_k carries barrier weights up to ~1e11 and its computed
// inverse is only cond(Re) * eps accurate; in the form above that error goes straight into P
// (-L'dKg), and on rare problems P loses definiteness (diagonal -2e3 where ~1e1 was right) until a
// pivot fails.  A factorisation that fails is therefore repeated in the gain-stationary form
//   P_k = Qb_k + A'P A - L'Kg - Kg'L + Kg'Re Kg      (= the form above when Kg = Re^-1 L exactly)
// whose error in Kg enters only to second order, as dKg' Re dKg >= 0 (the Joseph form's property
// without its extra hand-off).  It is not the default: measured on every test problem it costs
// interior-point iterations (H = 20: 9 -> 15), its P no longer matching the gains the solves use.
// Close to the optimum (merit <= kPolishMerit) a failed pivot is the normal end of the interior-
// point phase and the polish takes over instead.
// One wave runs the recursion (lanes = matrix entries); its LDS hand-offs need no barrier.
// ---------------------------------------------------------------------------------------------
// LDS instructions of one wave complete in issue order; this only keeps the compiler from moving
// the wave's LDS accesses across the hand-off.
__device__ __forceinline__ void wave_lds_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// Inverse of a symmetric positive-definite NU x NU matrix (Gauss-Jordan without pivoting, which is
// stable for SPD input; pivot reciprocals by rcp + Newton, ~1 ulp, instead of the long IEEE
// division sequence on the recursion's critical path).  False on a non-positive or non-finite
// pivot.
template <int NU>
__device__ __forceinline__ bool spd_inverse(double (&a)[NU][NU], double (&inv)[NU][NU]) {
  if constexpr (NU == 1) {
    const double piv = a[0][0];
    inv[0][0] = rcp(piv);
    return piv > 0.0 && isfinite(piv);
  } else if constexpr (NU == 2) {  // closed form
    const double det = a[0][0] * a[1][1] - a[0][1] * a[1][0];
    const double id = rcp(det);
    inv[0][0] = a[1][1] * id;
    inv[1][1] = a[0][0] * id;
    inv[0][1] = -a[0][1] * id;
    inv[1][0] = -a[1][0] * id;
    return a[0][0] > 0.0 && det > 0.0 && isfinite(det) && isfinite(a[0][0]);
  }
  bool ok = true;
#pragma unroll
  for (int r = 0; r < NU; ++r)
#pragma unroll
    for (int c = 0; c < NU; ++c) inv[r][c] = r == c ? 1.0 : 0.0;
#pragma unroll
  for (int q = 0; q < NU; ++q) {
    const double piv = a[q][q];
    ok = ok && piv > 0.0 && isfinite(piv);
    const double ip = rcp(piv);
#pragma unroll
    for (int c = 0; c < NU; ++c) {
      a[q][c] *= ip;
      inv[q][c] *= ip;
    }
#pragma unroll
    for (int r = 0; r < NU; ++r) {
      if (r == q) continue;
      const double f = a[r][q];
#pragma unroll
      for (int c = 0; c < NU; ++c) {
        a[r][c] -= f * a[q][c];
        inv[r][c] -= f * inv[q][c];
      }
    }
  }
  return ok;
}

// (Round 3 measured a register form of the NX = 4 step — P in registers, rows and columns moved by
// DPP quad broadcasts and ds_swizzle, ~26 cross-lane moves per step — and did not keep it: C5 QP
// 0.948 -> 1.033 ms)

// (Round 4 measured a matrix-core form of the NX = 4, NU <= 2 step — P kept in the result layout of
// v_mfma_f64_16x16x4_f64, X = P [A | B], [A'; B'] X + [Qb; Rb], P_k = D2 - L'Kg and (P_k + P_k')/2
// as four dependent matrix instructions plus the 2 x 2 inverse — and did not keep it: correct,
// but C5 QP 0.740 -> 0.760 ms; a dependent f64 matrix instruction costs ~100 cycles)

// Wave 0's part: the recursion (Kg, Ri into LDS; s.sc[62] = 0 on success, 1 on a failed pivot).
// No barrier: the interior-point loop runs it beside the other waves' work (riccati_factor below
// is the plain form: this, a barrier, riccati_factor_finish).
constexpr bool kPipe = true;
// The progress words of the pipelined affine solve (int slots in s.sc[56..57]): the factorisation's
// last finished step and the dual-residual wave's last finished input step (both count down from
// H; kProgAbort after a failed pivot, which releases the follower).
constexpr int kProgAbort = -1000;
__device__ __forceinline__ int* prog_word(const Lds& s, int q) { return reinterpret_cast<int*>(s.sc + 56 + q); }
// Release / acquire at workgroup scope, restricted to LDS (the "local" address-space fence): the
// step's LDS stores complete before the word (one lgkmcnt wait; no global-memory wait), and the
// reader's loads of the step's data follow its read of the word.
__device__ __forceinline__ void lds_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local"); }
__device__ __forceinline__ void lds_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); }
__device__ __forceinline__ void prog_publish(const Lds& s, int q, int k) {
  lds_release();
  __hip_atomic_store(prog_word(s, q), k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // every lane
}
// (a poll is one LDS read; between polls the waiting wave sleeps ~256 cycles, a quarter of a
// factorisation step, so that its reads do not queue in front of the factorisation's own)
__device__ __forceinline__ void prog_wait(const Lds& s, int q, int k) {
  while (__hip_atomic_load(prog_word(s, q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > k)
    __builtin_amdgcn_s_sleep(4);
  lds_acquire();
}


// ---- Register-form factorisation of planar isotropic models (round 5) ----
// For NX = 4, NU = 2 with A = [[a00 I, a01 I], [a10 I, a11 I]] and B = [[b0 I], [b1 I]] (the
// reference's double integrator; blob ISO), the recursion runs on one wave with P in registers:
// lane 4i + j (every row of 16 lanes alike) holds P_ij, and the step
//   U = P B:     U_ic = b0 P_{i,c} + b1 P_{i,c+2}              (quad_perm within quad i)
//   Re = Rb + B'U,  Ri = Re^-1                                  (U by row_newbcast: every lane alike)
//   M = P - U Ri U':  M_ij from rows i (quad_perm) and j (ds_bpermute, issued early)
//   P_k = Qb_k + A'M A = Qb_k + c00 M_ij + (c01 M_{i,j^2} + c10 M_{i^2,j}) + c11 M_{i^2,j^2}
// couples a lane only with lanes l ^ 2, l ^ 8, l ^ 10 (quad_perm, row_ror:8), and with
// c00 = a[bi][bi] a[bj][bj], c01 = a[bi][bi] a[1-bj][bj], c10 = a[1-bi][bi] a[bj][bj],
// c11 = a[1-bi][bi] a[1-bj][bj] (i = 2 bi + xi), every product rounded separately and the middle
// pair added first, the update is invariant under i <-> j bit for bit: P stays exactly symmetric
// with no transpose (the LDS form forms the lower triangle and mirrors it).  No LDS round trip sits
// on the chain: the step reads one record of a table built in front of the loop (the 10 canonical
// entries of Qb_k and Rb_k's diagonal) and writes Ri_k, the gains Kg_k and the solve map F_k, the
// last two formed off the chain from U_k (so riccati_maps has nothing left to do).  Measured on the bench's
// model (scripts/micro/riccati_dpp.hip, one wave): ~500 cycles per step against 921 for the LDS
// form, the same accuracy against a long-double recursion.  A failed pivot is not tested per step:
// the minimum over the steps of det(Re) and Re00, and P_0 finite (a NaN or infinity anywhere
// reaches it), give the same verdict at the end.
// The table sits in s.red behind the pipelined solve's forward sources ([4 H]): records [H][12].
__device__ __forceinline__ double* iso_qb(const Lds& s, int H) { return s.red + 4 * H; }
__device__ __forceinline__ int iso_canon(int a, int b) { return a * (a + 1) / 2 + b; }  // a >= b

template <bool kPublish>
__device__ __forceinline__ void riccati_factor_iso(const Lds& s, int H) {
  const int lane = threadIdx.x & 63;
  double* qbt = iso_qb(s, H);
  // the table, lane = step: record k holds Qb_k = qb(k - 1) (record 0: the terminal qb(H - 1)) and
  // Rb_k's diagonal; the entries as the LDS form sums them (2 Q_ab + C'S C, lower triangle)
  for (int kk = lane; kk < H; kk += 64) {
    const int rk = kk + 1 < H ? kk + 1 : 0;
    const double S00 = s.S[kk], S01 = s.S[H + kk], S11 = s.S[2 * H + kk];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b <= a; ++b) {
        const double c0a = s.Cm[a], c1a = s.Cm[kMx + a], c0b = s.Cm[b], c1b = s.Cm[kMx + b];
        qbt[rk * 12 + iso_canon(a, b)] =
            2.0 * s.Qm[a * kMx + b] + c0a * (S00 * c0b + S01 * c1b) + c1a * (S01 * c0b + S11 * c1b);
      }
    qbt[kk * 12 + 10] = 2.0 * s.Rm[0] + s.DU[kk * 2];
    qbt[kk * 12 + 11] = 2.0 * s.Rm[3] + s.DU[kk * 2 + 1];
  }
  wave_lds_fence();
  const int l = lane & 15, i = l >> 2, j = l & 3, bi = i >> 1, bj = j >> 1;
  const int ia = i > j ? i : j, jb = i > j ? j : i;
  const int qoff = iso_canon(ia, jb);
  const double aa[2][2] = {{s.Am[0], s.Am[2]}, {s.Am[2 * kMx], s.Am[2 * kMx + 2]}};
  const double b0 = s.Bm[0], b1 = s.Bm[2 * 2];
  const double c00 = mul_rn(aa[bi][bi], aa[bj][bj]), c01 = mul_rn(aa[bi][bi], aa[1 - bj][bj]);
  const double c10 = mul_rn(aa[1 - bi][bi], aa[bj][bj]), c11 = mul_rn(aa[1 - bi][bi], aa[1 - bj][bj]);
  const double R01 = 2.0 * s.Rm[1];
  const int src_j0 = ((lane & ~15) + 4 * j) * 4, src_j1 = src_j0 + 4;  // ds_bpermute byte addresses
  const double* rec = qbt + (H - 1) * 12;
  double p = qbt[qoff];  // the terminal Qb
  double mn = 1.0;
  // per step, off the chain: the gains Kg_k (lanes j < 2: Kg[k][u = j][x = i]) and the solve map
  // F_k = A' - Kg_k' B' (lane 4i + j: F_k[i][j], every lane of the row of 16 a distinct entry), from
  // L_{d,i} = (U'A)_{d,i} = alpha_i U_{i,d} + beta_i U_{i^2,d} (alpha_i = a[bi][bi], beta_i =
  // a[1-bi][bi]; row i ^ 2 of U by row_ror:8); Ri_k by lane 0.  Lanes without a slot write the
  // same instructions into scratch (s.P / s.T, unused by this form).
  const double alpha = aa[bi][bi], beta = aa[1 - bi][bi];
  const double Aji = s.Am[j * kMx + i], Bj0 = s.Bm[j * 2], Bj1 = s.Bm[j * 2 + 1];
  double* kg_at = j < 2 ? s.Kg + (H - 1) * 8 + j * 4 + i : s.P + l;
  const int kg_step = j < 2 ? 8 : 0;
  double* sm_at = s.SM + (H - 1) * 16 + l;
  double* ri_at = l == 0 ? s.Ri + (H - 1) * 4 : s.P + 16 + l;
  const int ri_step = l == 0 ? 4 : 0;
  for (int k = H - 1; k >= 0; --k) {
    const double qn = rec[qoff];  // Qb_k (not used at k = 0)
    const double rb00 = rec[10], rb11 = rec[11];
    rec -= 12;
    const double pa = dpp_mov_f64<0x44>(p), pb = dpp_mov_f64<0xEE>(p);  // quad_perm [0,1,0,1], [2,3,2,3]
    const double uu = fma(b1, pb, b0 * pa);                                // U_{i, j & 1}
    const double Ub0 = bperm_f64(uu, src_j0), Ub1 = bperm_f64(uu, src_j1);  // row j of U
    __builtin_amdgcn_sched_barrier(0);  // both permutes issue here: their latency hides behind Re
    const double U00 = row_bcast_f64<0>(uu), U01 = row_bcast_f64<1>(uu), U11 = row_bcast_f64<5>(uu);
    const double U20 = row_bcast_f64<8>(uu), U21 = row_bcast_f64<9>(uu), U31 = row_bcast_f64<13>(uu);
    const double Ua0 = dpp_mov_f64<0x00>(uu), Ua1 = dpp_mov_f64<0x55>(uu);  // row i of U
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
    {  // gains and solve map of step k
      const double Uo0 = dpp_mov_f64<0x128>(Ua0), Uo1 = dpp_mov_f64<0x128>(Ua1);  // row i ^ 2
      const double L0 = fma(beta, Uo0, alpha * Ua0), L1 = fma(beta, Uo1, alpha * Ua1);
      const double K0 = fma(Ri01, L1, Ri00 * L0), K1 = fma(Ri11, L1, Ri01 * L0);
      *kg_at = (j & 1) ? K1 : K0;
      kg_at -= kg_step;
      *sm_at = fma(-K1, Bj1, fma(-K0, Bj0, Aji));
      sm_at -= 16;
    }
    if constexpr (kPublish) prog_publish(s, 0, k);  // Kg_k, Ri_k, F_k are out
    const double m00 = mul_rn(Ua0, Ub0), m11 = mul_rn(Ua1, Ub1);
    const double m01 = add_rn(mul_rn(Ua0, Ub1), mul_rn(Ua1, Ub0));
    const double M = p - fma(m00, Ri00, fma(m01, Ri01, m11 * Ri11));
    const double Mc = dpp_mov_f64<0x4E>(M);   // l ^ 2: quad_perm [2,3,0,1]
    const double Mr = dpp_mov_f64<0x128>(M);  // l ^ 8: row_ror:8
    const double Md = dpp_mov_f64<0x4E>(Mr);  // l ^ 10
    const double t = add_rn(mul_rn(c01, Mc), mul_rn(c10, Mr));
    p = qn + add_rn(add_rn(mul_rn(c00, M), t), mul_rn(c11, Md));
  }
  const bool ok = mn > 0.0 && __builtin_isfinite(p);
  const bool all_ok = __ballot(!ok) == 0ull;  // uniform
  if (lane == 0) {
    s.sc[62] = all_ok ? 0.0 : 1.0;
    s.sc[61] = 1.0;  // the solve maps are formed (riccati_maps has nothing to do)
  }
  if constexpr (kPublish) {
    if (!all_ok) prog_publish(s, 0, kProgAbort);
  }
}

template <int NU, int NX, bool kStationary = false, bool kPublish = false>
__device__ __forceinline__ void riccati_factor_wave0(const Lds& s, int H) {
  const int tid = threadIdx.x, lane = tid & 63;
  double* flag = s.sc + 62;
  if constexpr (NU == 2 && NX == 4 && !kStationary) {
    if (s.iso) {  // uniform
      if (tid < 64) riccati_factor_iso<kPublish>(s, H);
      return;
    }
  }
  if (tid < 64) {
    if (lane == 0) s.sc[61] = 0.0;  // this form writes the gains itself
    constexpr int NX2 = NX * NX;
    const int e = lane < NX2 ? lane : 0;
    const int i = e / NX, j = e % NX;  // entry (i, j) owned by lane < NX2
    // stage (a) operands held in registers: column j of A (for T) and, for the lanes that also
    // compute U = P B, column c of B
    // U = P B: entry (i, j) for j < NU from the same row of P as T (no second row load)
    const int uc = j < NU ? j : 0;
    double Acol[NX], Bcol[NX];
#pragma unroll
    for (int m = 0; m < NX; ++m) {
      Acol[m] = s.Am[m * kMx + j];
      Bcol[m] = s.Bm[m * NU + uc];
    }
    const double c0i = s.Cm[i], c1i = s.Cm[kMx + i], c0j = s.Cm[j], c1j = s.Cm[kMx + j];
    const double q2 = 2.0 * s.Qm[i * kMx + j];
    // loop-invariant operands of stage (b) in registers (the wave fences keep the compiler from
    // hoisting LDS loads out of the step loop itself)
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
    auto qb = [&](int k) {  // Qb_{k+1} = 2Q + C'S_k C, entry (i, j)
      const double S00 = s.S[k], S01 = s.S[H + k], S11 = s.S[2 * H + k];
      return q2 + c0i * (S00 * c0j + S01 * c1j) + c1i * (S01 * c0j + S11 * c1j);
    };
    if (lane < NX2 && i >= j) {
      const double v = qb(H - 1);
      s.P[i * kMx + j] = v;
      s.P[j * kMx + i] = v;
    }
    bool ok = true;
    for (int k = H - 1; k >= 0 && ok; --k) {
      wave_lds_fence();
      // (a) T = P A (lane = entry), U = P B (lane = entry of U)
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
      // (b) every operand in one batch: T columns i and j, U, B, the weights of step k
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
      // Re = Rb + B'U (every lane, identical) and its inverse
      double Re[NU][NU], Ri[NU][NU];
#pragma unroll
      for (int c = 0; c < NU; ++c)
#pragma unroll
        for (int d = 0; d < NU; ++d) {
          double acc = R2[c][d] + (c == d ? du[c] : 0.0);
#pragma unroll
          for (int m = 0; m < NX; ++m) acc += Bm[m][c] * Um[m][d];
          Re[c][d] = acc;
        }
      ok = spd_inverse<NU>(Re, Ri);
      double Li[NU], Lj[NU], Ki[NU], Kj[NU];
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
        double acc = 0.0, acci = 0.0;
#pragma unroll
        for (int d = 0; d < NU; ++d) {
          acc += Ri[c][d] * Lj[d];
          acci += Ri[c][d] * Li[d];
        }
        Kj[c] = acc;
        Ki[c] = acci;  // only the stationary form reads it
      }
      if (lane < NX2 && i == j) {
#pragma unroll
        for (int c = 0; c < NU; ++c) s.Kg[(k * NU + c) * NX + j] = Kj[c];
      }
      if (lane < NX2 && k > 0 && i >= j) {
        // Qb + A'P A - L'Kg - Kg'L + Kg'Re Kg, entry (i, j); Re_cd = Rb + B'U recomputed from the
        // registers it was formed from (the inversion overwrote it)
        double acc = qnext;
#pragma unroll
        for (int m = 0; m < NX; ++m) acc += ai[m] * tj[m];
        if constexpr (kStationary) {
          double corr = 0.0;
#pragma unroll
          for (int c = 0; c < NU; ++c) {
            double rk = 0.0;
#pragma unroll
            for (int d = 0; d < NU; ++d) {
              double re = R2[c][d] + (c == d ? du[c] : 0.0);
#pragma unroll
              for (int m = 0; m < NX; ++m) re += Bm[m][c] * Um[m][d];
              rk += re * Kj[d];
            }
            corr += Ki[c] * rk - Li[c] * Kj[c] - Ki[c] * Lj[c];
          }
          acc += corr;
        } else {
#pragma unroll
          for (int c = 0; c < NU; ++c) acc -= Li[c] * Kj[c];
        }
        s.P[i * kMx + j] = acc;
        s.P[j * kMx + i] = acc;
      }
      if (lane == 0) {
#pragma unroll
        for (int c = 0; c < NU; ++c)
#pragma unroll
          for (int d = 0; d < NU; ++d) s.Ri[(k * NU + c) * NU + d] = Ri[c][d];
      }
      if constexpr (kPublish) prog_publish(s, 0, k);  // Kg_k, Ri_k are out
    }
    if (lane == 0) *flag = ok ? 0.0 : 1.0;
    if constexpr (kPublish) {
      if (!ok) prog_publish(s, 0, kProgAbort);
    }
  }
}

// After a barrier behind riccati_factor_wave0: its outcome (uniform) and, for NX <= 4, the solve
// maps.  Every thread calls it.
template <int NU, int NX>
__device__ __forceinline__ bool riccati_maps(const Lds& s, int H, bool ok) {
  const int tid = threadIdx.x;
  if constexpr (NX <= 4) {
    if (ok && s.sc[61] != 0.0) return ok;  // uniform: the isotropic form wrote the maps itself
    if (ok) {  // the solves' maps F_k = A' - Kg_k' B' (row-major [k][r][c] in s.SM), once per factor
      for (int e = tid; e < H * 16; e += static_cast<int>(blockDim.x)) {
        const int k = e >> 4, r = (e >> 2) & 3, c = e & 3;
        double acc = s.Am[c * kMx + r];
#pragma unroll
        for (int u = 0; u < NU; ++u) acc -= s.Kg[(k * NU + u) * NX + r] * s.Bm[c * NU + u];
        s.SM[e] = acc;
      }
      __syncthreads();
    }
  }
  return ok;
}
template <int NU, int NX>
__device__ __forceinline__ bool riccati_factor_finish(const Lds& s, int H) {
  return riccati_maps<NU, NX>(s, H, s.sc[62] == 0.0);  // uniform
}

template <int NU, int NX, bool kStationary = false>
__device__ __forceinline__ bool riccati_factor(const Lds& s, int H) {
  riccati_factor_wave0<NU, NX, kStationary>(s, H);
  __syncthreads();
  return riccati_factor_finish<NU, NX>(s, H);
}

// Solve K x = b with the factorisation above; b in x[0..n) (LDS), overwritten by the solution.
// Vectors travel between lanes by readlane (lane m < NX holds entry m), so a step of either pass
// has no LDS round trip on its critical path; the step's gains are loaded one step ahead.
template <int NU, int NX>
__device__ __forceinline__ void riccati_solve(const Lds& s, int H, double* x) {
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid < 64) {
    const int li = lane < NX ? lane : 0;
    double Acol[NX], Arow[NX], Bm[NX][NU], Brow[NU];
#pragma unroll
    for (int m = 0; m < NX; ++m) {
      Acol[m] = s.Am[m * kMx + li];
      Arow[m] = s.Am[li * kMx + m];
#pragma unroll
      for (int c = 0; c < NU; ++c) Bm[m][c] = s.Bm[m * NU + c];
    }
#pragma unroll
    for (int c = 0; c < NU; ++c) Brow[c] = s.Bm[li * NU + c];
    // backward: ge_k = B'p - b_k, kff_k = -Re_k^-1 ge_k (into x), p <- A'p - Kg_k'ge_k.
    // The step data (Kg_k column, Re_k^-1, b_k) are loaded two steps ahead (two register sets,
    // loop unrolled by two), so no LDS latency sits on the recursion's chain.
    struct BackStep {
      double kgl[NU], ri[NU][NU], bk[NU];
    };
    auto load_b = [&](BackStep& d, int k) {
      if (k < 0) return;
#pragma unroll
      for (int c = 0; c < NU; ++c) {
        d.kgl[c] = s.Kg[(k * NU + c) * NX + li];
        d.bk[c] = x[k * NU + c];
#pragma unroll
        for (int e = 0; e < NU; ++e) d.ri[c][e] = s.Ri[(k * NU + c) * NU + e];
      }
    };
    double p = 0.0;
    auto back_step = [&](const BackStep& d, int k) {
      double pv[NX];
#pragma unroll
      for (int m = 0; m < NX; ++m) pv[m] = readlane_f64(p, m);
      double ge[NU];
#pragma unroll
      for (int c = 0; c < NU; ++c) {
        double acc = -d.bk[c];
#pragma unroll
        for (int m = 0; m < NX; ++m) acc += Bm[m][c] * pv[m];
        ge[c] = acc;
      }
      double np = 0.0, mine = 0.0;
#pragma unroll
      for (int m = 0; m < NX; ++m) np += Acol[m] * pv[m];
#pragma unroll
      for (int c = 0; c < NU; ++c) {
        np -= d.kgl[c] * ge[c];
        double kff = 0.0;
#pragma unroll
        for (int e = 0; e < NU; ++e) kff -= d.ri[c][e] * ge[e];
        mine = lane == c ? kff : mine;
      }
      p = lane < NX ? np : 0.0;
      wave_lds_fence();
      if (lane < NU) x[k * NU + lane] = mine;  // kff_k (b_k was consumed two steps earlier)
    };
    {
      BackStep d0, d1;
      load_b(d0, H - 1);
      load_b(d1, H - 2);
      for (int k = H - 1; k >= 0; k -= 2) {
        back_step(d0, k);
        load_b(d0, k - 2);
        if (k - 1 < 0) break;
        back_step(d1, k - 1);
        load_b(d1, k - 3);
      }
    }
    wave_lds_fence();
    // forward: du_k = kff_k - Kg_k x_k, x_{k+1} = A x_k + B du_k (step data two steps ahead)
    struct FwdStep {
      double kg[NU][NX], ff[NU];
    };
    auto load_f = [&](FwdStep& d, int k) {
      if (k >= H) return;
#pragma unroll
      for (int c = 0; c < NU; ++c) {
        d.ff[c] = x[k * NU + c];
#pragma unroll
        for (int m = 0; m < NX; ++m) d.kg[c][m] = s.Kg[(k * NU + c) * NX + m];
      }
    };
    double xs = 0.0;
    auto fwd_step = [&](const FwdStep& d, int k) {
      double xv[NX];
#pragma unroll
      for (int m = 0; m < NX; ++m) xv[m] = readlane_f64(xs, m);
      double du[NU], mine = 0.0;
#pragma unroll
      for (int c = 0; c < NU; ++c) {
        double acc = d.ff[c];
#pragma unroll
        for (int m = 0; m < NX; ++m) acc -= d.kg[c][m] * xv[m];
        du[c] = acc;
        mine = lane == c ? acc : mine;
      }
      double nxs = 0.0;
#pragma unroll
      for (int m = 0; m < NX; ++m) nxs += Arow[m] * xv[m];
#pragma unroll
      for (int c = 0; c < NU; ++c) nxs += Brow[c] * du[c];
      xs = lane < NX ? nxs : 0.0;
      wave_lds_fence();
      if (lane < NU) x[k * NU + lane] = mine;
    };
    {
      FwdStep d0, d1;
      load_f(d0, 0);
      load_f(d1, 1);
      for (int k = 0; k < H; k += 2) {
        fwd_step(d0, k);
        load_f(d0, k + 2);
        if (k + 1 >= H) break;
        fwd_step(d1, k + 1);
        load_f(d1, k + 3);
      }
    }
  }
  __syncthreads();
}

// Solve K x = b for NX <= 4 (the reference's double integrator and every smaller model).  Both
// passes are affine recurrences in the state dimension,
//   backward  p_k = F_k p_{k+1} + Kg_k' b_k       (p_H = 0),   F_k = A' - Kg_k' B'
//   forward   x_{k+1} = F_k' x_k + B kff_k         (x_0 = 0),   kff_k = -Re_k^-1 (B' p_{k+1} - b_k)
// with the maps F_k built once per factorisation (riccati_factor, s.SM).  Everything that is per
// step runs on all threads (the sources Kg_k' b_k, kff_k, B kff_k, du_k); only the two
// recurrences run on one wave: lane i (mod 4) holds entry i of the state, the previous state
// reaches every lane of its quad by DPP quad broadcasts (no LDS on the chain) and the step's map
// row is loaded one step ahead — ~H short steps per pass and four barriers per solve, instead of
// the 2 ceil(log2 H) + 6 barrier-separated levels of the parallel scan this replaced.
// (the quad's four entries are those of lanes 0..3 in every row of 16 (the quads replicate each
// other), so each reaches every lane by one v_mov_b64 row_newbcast instead of two 32-bit quad_perm
// moves: the same bits, half the instructions on the recurrences' chains)
__device__ __forceinline__ double affine4(double w, const double (&f)[4], double v) {
  const double v0 = row_bcast_f64<0>(v), v1 = row_bcast_f64<1>(v);
  const double v2 = row_bcast_f64<2>(v), v3 = row_bcast_f64<3>(v);
  return fma(f[0], v0, fma(f[1], v1, w)) + fma(f[2], v2, f[3] * v3);
}

// one step of a recurrence: the map row / column and the source, loaded four steps ahead.  The
// horizon is padded to a multiple of four (the backward pass keeps p_H = 0 through the padding,
// the forward pass ends with it), and the loads past either end read step 0 unconditionally, so
// the unrolled loop has no branch but its back edge (branches in it, or a mask applied at the
// load, made the compiler drain every outstanding prefetch each step).
struct StepData {
  double f[4], w;
  bool in;  // a real step (false for the padding)
};
__device__ __forceinline__ void load_back(StepData& d, const double* M, const double* W, int k, int i,
                                          int H) {
  d.in = k >= 0 && k < H;
  const int kk = d.in ? k : 0;  // the padding reads step 0 and is discarded where it is used
#pragma unroll
  for (int m = 0; m < 4; ++m) d.f[m] = M[(kk * 4 + i) * 4 + m];  // row i of F_k
  d.w = W[kk * 4 + i];
}
__device__ __forceinline__ void load_fwd(StepData& d, const double* M, const double* G, int k, int i,
                                         int H) {
  d.in = k < H;
  const int kk = d.in ? k : 0;
#pragma unroll
  for (int m = 0; m < 4; ++m) d.f[m] = M[(kk * 4 + m) * 4 + i];  // column i of F_k
  d.w = G[kk * 4 + i];
}

// With pos: also the positions the solution produces, pos[2k+i] = c[2k+i] + (C x_{k+1})_i (c may
// be null: 0) — read off the forward pass's states instead of a separate Mp convolution.
// With z (per-step 2-vectors, [2H]): K x = b - Gp' z without forming Gp' z — z_k is the linear
// cost C'z_k on the state x_{k+1} of the LQ problem, so it enters the backward pass as a source,
// p_k = C'z_{k-1} + F_k p_{k+1} + Kg_k' b_k with p_H = C'z_{H-1} (the value function's linear term),
// instead of a Gp' z convolution (n rows of ~H / PARTS terms) and its two barriers.
// Two halves: dpp_backward leaves kff_k = -Re_k^-1 (B' p_{k+1} - b_k) in x and the forward
// sources B kff_k in s.red; dpp_forward runs the forward recurrence and writes du = kff - Kg x.
// (The interior-point loop's affine solve runs the backward half beside the factorisation,
// affine_backward_follow, and only the forward half after it.)
// The parallel tail of the backward half, after the recurrence left p_k in s.SV: kff_k = -Re_k^-1
// (B' p_{k+1} - b_k) into kff (may be b: in place), the forward sources B kff_k into s.red.  Ends
// with a barrier.
template <int NU, int kBlock>
__device__ __forceinline__ void dpp_backward_tail(const Lds& s, int H, const double* b, double* kff_out) {
  const int t = threadIdx.x;
  const double* W = s.SV;
  double* G = s.red;
  for (int e = t; e < H * 4; e += kBlock) {
    const int k = e >> 2, i = e & 3;
    double ge[NU], kff[NU];
#pragma unroll
    for (int c = 0; c < NU; ++c) {
      double acc = -b[k * NU + c];
#pragma unroll
      for (int m = 0; m < 4; ++m) acc += s.Bm[m * NU + c] * W[(k + 1) * 4 + m];  // p_H = W[H]
      ge[c] = acc;
    }
    double gi = 0.0;
#pragma unroll
    for (int c = 0; c < NU; ++c) {
      double acc = 0.0;
#pragma unroll
      for (int d = 0; d < NU; ++d) acc -= s.Ri[(k * NU + c) * NU + d] * ge[d];
      kff[c] = acc;
      gi += s.Bm[i * NU + c] * acc;
    }
    G[e] = gi;
    wave_lds_fence();  // the step's four lanes share one wave: every b_k read precedes the writes
    if (i < NU) {
#pragma unroll
      for (int c = 0; c < NU; ++c)
        if (c == i) kff_out[k * NU + c] = kff[c];
    }
  }
  __syncthreads();
}

template <int NU, int kBlock>
__device__ __forceinline__ void dpp_backward(const Lds& s, int H, double* x, const double* z) {
  const int t = threadIdx.x;
  double* W = s.SV;   // [H + 1][4]: Kg_k' b_k (+ C'z_{k-1}), then p_k (backward pass)
  double* G = s.red;  // [H][4]: B kff_k
  const double* M = s.SM;
  for (int e = t; e < (H + 1) * 4; e += kBlock) {
    const int k = e >> 2, i = e & 3;
    double acc = 0.0;
    if (k < H) {
#pragma unroll
      for (int u = 0; u < NU; ++u) acc += s.Kg[(k * NU + u) * 4 + i] * x[k * NU + u];
    }
    if (z && k >= 1) acc += s.Cm[i] * z[2 * k - 2] + s.Cm[kMx + i] * z[2 * k - 1];
    W[e] = acc;
  }
  __syncthreads();
  if (t < 64) {  // backward: p_k = F_k p_{k+1} + w_k, row i of F_k
    const int i = t & 3;
    // lanes 0..3 store the state; the others write the same instruction into scratch (s.T, one
    // slot per lane), so the chain carries no branch (an exec-masked store split the loop)
    const bool keeper = t < 4;
    double p = W[H * 4 + i];  // p_H: C'z_{H-1} (0 without z)
    const int Hp = (H + 3) & ~3;  // W holds HM >= Hp steps
    StepData d[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) load_back(d[q], M, W, Hp - 1 - q, i, H);
    for (int k = Hp - 1; k >= 0; k -= 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // step k - q; its data was loaded four steps ago
        const double pn = affine4(d[q].w, d[q].f, p);
        p = d[q].in ? pn : p;      // the padding steps (k >= H) keep p_H
        *(keeper ? W + (k - q) * 4 + i : s.T + t) = p;  // p_k (w_k was read four steps ago)
        load_back(d[q], M, W, k - q - 4, i, H);
      }
    }
  }
  __syncthreads();
  dpp_backward_tail<NU, kBlock>(s, H, x, x);
}

// The forward half: x_{k+1} = F_k' x_k + B kff_k from x_0 = 0 (F_k in s.SM, B kff_k in s.red),
// du_k = kff_k - Kg_k x_k into du (kff may be du), the positions into pos.  Ends with a barrier.
template <int NU, int kBlock>
__device__ __forceinline__ void dpp_forward(const Lds& s, int H, const double* kff, double* du, double* pos,
                                   const double* c) {
  const int t = threadIdx.x;
  double* W = s.SV;   // [H + 1][4]: x_k
  const double* G = s.red;
  const double* M = s.SM;
  if (t < 64) {  // forward: x_{k+1} = F_k' x_k + B kff_k, column i of F_k
    const int i = t & 3;
    const bool keeper = t < 4;
    double xs = 0.0;
    const int Hp = (H + 3) & ~3;
    StepData d[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) load_fwd(d[q], M, G, q, i, H);
    for (int k = 0; k < Hp; k += 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        *(keeper ? W + (k + q) * 4 + i : s.T + t) = xs;  // x_k
        xs = affine4(d[q].w, d[q].f, xs);
        load_fwd(d[q], M, G, k + q + 4, i, H);
      }
    }
    if (keeper && Hp == H) W[H * 4 + i] = xs;  // x_H (with padding the loop stored it)
  }
  __syncthreads();
  // du_k = kff_k - Kg_k x_k
  for (int e = t; e < H * NU; e += kBlock) {
    const int k = e / NU, u = e - (e / NU) * NU;
    double acc = kff[e];
#pragma unroll
    for (int m = 0; m < 4; ++m) acc -= s.Kg[(k * NU + u) * 4 + m] * W[k * 4 + m];
    du[e] = acc;
  }
  if (pos) {  // p_k = c_k + C x_{k+1}
    for (int e = t; e < 2 * H; e += kBlock) {
      const int k = e >> 1, i = e & 1;
      double acc = c ? c[e] : 0.0;
#pragma unroll
      for (int m = 0; m < 4; ++m) acc += s.Cm[i * kMx + m] * W[(k + 1) * 4 + m];
      pos[e] = acc;
    }
  }
  __syncthreads();
}

template <int NU, int kBlock>
__device__ __forceinline__ void riccati_solve_dpp(const Lds& s, int H, double* x, double* pos, const double* c,
                                         const double* z) {
  dpp_backward<NU, kBlock>(s, H, x, z);
  dpp_forward<NU, kBlock>(s, H, x, x, pos, c);
}

// K x = b - Gp' z (z may be null): the DPP recurrences for NX <= 4 (z as a state source), the
// wave-serial recursion otherwise (Gp' z summed first).  With pos: the positions of the solution as
// well, pos = c + Gp x (c may be null).  Ends with a barrier.
template <int NU, int NX, int kBlock, int HMX>
__device__ __forceinline__ void newton_solve(const Lds& s, int H, int n, double* x, double* pos = nullptr,
                                    const double* c = nullptr, const double* z = nullptr) {
  if constexpr (NX <= 4) {
    riccati_solve_dpp<NU, kBlock>(s, H, x, pos, c, z);
  } else {
    if (z) {
      gpt_parts<NU, kBlock>(s, z, nullptr, nullptr, s.red, n, H);
      __syncthreads();
      for (int j = threadIdx.x; j < n; j += kBlock) x[j] -= parts_total<kBlock>(s.red, j);
      __syncthreads();
    }
    riccati_solve<NU, NX>(s, H, x);
    if (pos) {
      positions<NU, kBlock>(s, x, pos, c, H);
      __syncthreads();
    }
  }
}

// The dual residual of the inputs r_du = f + H0 u + Gp' v + (lUu - lUl) and the input part of the
// affine rhs, dua = -r_du - rU (its Gp' za part goes to the solve as a state source), for NX <= 4 on
// ONE wave, without the condensed H0: H0 u = 2 R u + 2 Gx' Q Gx u and Gp' v = Gx' C' v, so with the
// states of u from x_0 = 0 (forward: x_{k+1} = A x_k + B u_k) and the adjoint (backward:
// lambda_H = y_H, lambda_k = y_k + A' lambda_{k+1}, y_k = 2 Q x_k + C' v_{k-1}),
//   r_du_j = f_j + 2 (R u)_j + B' lambda_{j+1} (+ box).
// Phases of one wave (wave-local LDS hand-offs, no barrier): the sources B u_k for every step at
// once; the forward chain (lane i of each quad holds x_i, quad broadcasts, the source loaded four
// steps ahead as in the solves); y_k for every step at once; the backward chain; r_du for every
// input at once — two chains of H ~100-cycle steps instead of n rows of ~H + n dependent LDS terms
// (~33 k cycles at C5 on seven waves).  Progress word 1 is set once at the end.  X: 8 (H + 1)
// doubles of scratch.  Returns this lane's max |r_du|.
template <int NU>
__device__ inline double dual_residual_wave(const Lds& s, int H, int n, bool has_u, double* X) {
  const int lane = threadIdx.x & 63, i = lane & 3;
  const bool keeper = lane < 4;
  double* Src = X;                // [H + 1][4]: B u_k (at k), then y_k
  double* Xs = X + (H + 1) * 4;   // [H + 1][4]: x_k, then lambda_k
  // the other lanes' copy of each chain store (no exec-mask branch in the chain): s.dp, free from
  // the previous update to this iteration's corrector solve (s.T is the concurrent factorisation's)
  double* junk = s.dp + lane;
  for (int e = lane; e < H * 4; e += 64) {  // Src[k] = B u_k
    const int k = e >> 2, r = e & 3;
    double w = 0.0;
#pragma unroll
    for (int c = 0; c < NU; ++c) w += s.Bm[r * NU + c] * s.u[k * NU + c];
    Src[e] = w;
  }
  wave_lds_fence();
  double arow[4], acol[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    arow[m] = s.Am[i * kMx + m];
    acol[m] = s.Am[m * kMx + i];
  }
  const int Hp = (H + 3) & ~3;
  {  // forward: x_{k+1} = A x_k + B u_k, x_0 = 0
    double x = 0.0, w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = Src[(q < H ? q : 0) * 4 + i];
    for (int k = 0; k < Hp; k += 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double xn = affine4(w[q], arow, x);
        x = k + q < H ? xn : x;
        *(keeper ? Xs + (k + q + 1) * 4 + i : junk) = x;  // x_{k+q+1}
        const int kn = k + q + 4;
        w[q] = Src[(kn < H ? kn : 0) * 4 + i];
      }
    }
  }
  wave_lds_fence();
  for (int e = lane + 4; e < (H + 1) * 4; e += 64) {  // y_k = 2 Q x_k + C' v_{k-1}, k >= 1 (in place)
    const int k = e >> 2, r = e & 3;
    double y = s.Cm[r] * s.v[2 * k - 2] + s.Cm[kMx + r] * s.v[2 * k - 1];
#pragma unroll
    for (int m = 0; m < 4; ++m) y += 2.0 * s.Qm[r * kMx + m] * Xs[k * 4 + m];
    Src[e] = y;  // (Src's B u_k are no longer needed; y_k lands in Src, lambda_k in Xs)
  }
  wave_lds_fence();
  // the inputs' terms without lambda: f + 2 R u into s.rdu, the box duals' difference into s.dua;
  // the backward chain adds B'lambda_{j+1} as soon as it has lambda_{j+1}, then the box term (the
  // order of the earlier all-at-once form: a different rounding of r_du moved one degenerate batch
  // problem from one polish attempt to six)
  for (int j = lane; j < n; j += 64) {
    const int jj = j / NU, ai = j - jj * NU;
    double ru = 0.0;
#pragma unroll
    for (int c = 0; c < NU; ++c) ru += s.Rm[ai * NU + c] * s.u[jj * NU + c];
    s.rdu[j] = s.f[j] + 2.0 * ru;
    s.dua[j] = has_u ? s.bx[n + j] - s.bx[3 * n + j] : 0.0;
  }
  wave_lds_fence();
  // backward: lambda_k = y_k + A' lambda_{k+1}, lambda_{H+1} = 0; at each k the input step k - 1's
  // dual residual r_du = base + B'lambda_k and affine rhs dua = -r_du - rU (lanes c < NU), published
  // every four steps (progress word 1 = the lowest input step out), so that the pipelined backward
  // solve starts behind this chain instead of after all of it
  const bool rkeeper = lane < NU;
  const int cc = i < NU ? i : 0;
  double bcol[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) bcol[m] = s.Bm[m * NU + cc];
  double rdm = 0.0;
  {
    double lam = 0.0, y[4], base[4], box[4], ru[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kk = H - q;
      y[q] = Src[(kk >= 1 ? kk : 1) * 4 + i];
      const int jb = (kk >= 1 ? kk - 1 : 0) * NU + cc;
      base[q] = s.rdu[jb];
      box[q] = s.dua[jb];
      ru[q] = s.rU[jb];
    }
    for (int k = H; k >= H + 1 - Hp; k -= 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int kk = k - q;
        const double ln = affine4(y[q], acol, lam);
        lam = kk >= 1 ? ln : lam;
        *(keeper && kk >= 1 ? Xs + kk * 4 + i : junk) = lam;  // lambda_kk
        const double l0 = row_bcast_f64<0>(lam), l1 = row_bcast_f64<1>(lam);
        const double l2 = row_bcast_f64<2>(lam), l3 = row_bcast_f64<3>(lam);
        const double r = fma(bcol[3], l3, fma(bcol[2], l2, fma(bcol[1], l1, fma(bcol[0], l0, base[q])))) + box[q];
        const bool out = rkeeper && kk >= 1;
        const int jo = (kk - 1) * NU + i;
        *(out ? s.rdu + jo : junk) = r;
        *(out ? s.dua + jo : junk) = -r - ru[q];
        rdm = out ? fmax(rdm, fabs(r)) : rdm;
        const int kn = kk - 4;
        y[q] = Src[(kn >= 1 ? kn : 1) * 4 + i];
        const int jn = (kn >= 1 ? kn - 1 : 0) * NU + cc;
        base[q] = s.rdu[jn];
        box[q] = s.dua[jn];
        ru[q] = s.rU[jn];
      }
      const int lowest = k - 4;  // input steps >= lowest are out (k - 3 - 1)
      prog_publish(s, 1, lowest > 0 ? lowest : 0);
    }
  }
  prog_publish(s, 1, -1);  // every input step's rows are out
  return rdm;
}

// The backward recurrence of the affine solve (dpp_backward with b = dua, z = za), run by one wave
// beside the factorisation and behind it: p_k = F_k p_{k+1} + Kg_k' b_k + C'z_{k-1} into s.SV
// (p_H = C'z_{H-1}), four steps per wait on the factorisation's progress word (their rows of F_k,
// gains and sources loaded together), each block as soon as the dual-residual wave's backward chain
// has published its b_k.
// Only the chain runs here (~20 instructions a step); kff_k and the forward sources follow in
// dpp_backward_tail after the barrier, then the forward half (round 5: the follower also formed
// kff and the sources per step and, at ~760 cycles a step, was P1's last wave).  The isotropic
// factorisation writes the rows of F_k itself; otherwise they are formed here from the gains and
// stored for the later solves.  Lanes without a slot write into scratch (s.dp: free from the
// previous update to this iteration's corrector solve; the dual-residual wave scribbles there too).
template <int NU>
__device__ __forceinline__ void affine_backward_follow(const Lds& s, int H, const double* b, const double* z) {
  const int lane = threadIdx.x & 63, i = lane & 3;
  const bool keeper = lane < 4;
  double* W = s.SV;
  double* junk = s.dp + lane;
  double acol[4], Bm[4][NU];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    acol[c] = s.Am[c * kMx + i];  // A[c][i]: row i of A'
#pragma unroll
    for (int u = 0; u < NU; ++u) Bm[c][u] = s.Bm[c * NU + u];
  }
  const double c0 = s.Cm[i], c1 = s.Cm[kMx + i];
  double p = z ? c0 * z[2 * H - 2] + c1 * z[2 * H - 1] : 0.0;  // p_H = C'z_{H-1}
  *(keeper ? W + H * 4 + i : junk) = p;
  for (int k0 = H - 1; k0 >= 0; k0 -= 4) {
    prog_wait(s, 1, k0 >= 3 ? k0 - 3 : 0);  // b_k of steps k0 .. k0 - 3 (the dual-residual wave)
    prog_wait(s, 0, k0 >= 3 ? k0 - 3 : 0);  // their gains and maps (the factorisation)
    // every load of the block first, at clamped indices (steps below 0 are computed and
    // discarded), so that they are in flight together: a per-step branch on the state source
    // (k >= 1) had put a wait for each step's loads in front of the next step's
    double f[4][4], w[4], kg[4][NU], bk[4][NU], zk[4][2];
    const double* zp = z ? z : b;  // (read and not used without z)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = k0 - q >= 0 ? k0 - q : 0;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        kg[q][u] = s.Kg[(k * NU + u) * 4 + i];
        bk[q][u] = b[k * NU + u];
      }
      const int kz = k >= 1 ? 2 * k - 2 : 0;
      zk[q][0] = zp[kz];
      zk[q][1] = zp[kz + 1];
    }
    if (s.iso) {  // uniform
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = k0 - q >= 0 ? k0 - q : 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) f[q][c] = s.SM[(k * 4 + i) * 4 + c];
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = k0 - q >= 0 ? k0 - q : 0;
      double acc = 0.0;
#pragma unroll
      for (int u = 0; u < NU; ++u) acc += kg[q][u] * bk[q][u];
      const double zt = c0 * zk[q][0] + c1 * zk[q][1];
      acc += z && k >= 1 ? zt : 0.0;
      w[q] = acc;
      if (!s.iso) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          double fr = acol[c];
#pragma unroll
          for (int u = 0; u < NU; ++u) fr -= kg[q][u] * Bm[c][u];
          f[q][c] = fr;
          *(keeper && k0 - q >= 0 ? s.SM + (k * 4 + i) * 4 + c : junk) = fr;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double pn = affine4(w[q], f[q], p);
      const bool in = k0 - q >= 0;
      p = in ? pn : p;
      *(keeper && in ? W + (k0 - q) * 4 + i : junk) = p;  // p_k
    }
  }
}

struct HsRow {
  double h0, h1, g, sv, wA, lA, wB, lB;
};
struct HsLin {
  double rpA, rpB, rds, DA, DB, sig, iwA, iwB, isig;
};
struct RowDir {
  double ds, dwA, dlA, dwB, dlB;
};

__device__ __forceinline__ HsLin hs_lin(const HsRow& q, double p0, double p1) {
  HsLin l;
  l.rpA = q.h0 * p0 + q.h1 * p1 + q.g - q.sv + q.wA;  // h.p + g - s + w_hs
  l.rpB = q.wB - q.sv;                                // -s + w_s
  l.rds = kSlackHess * q.sv + kSlackLin - q.lA - q.lB;
  l.iwA = rcp(q.wA);
  l.iwB = rcp(q.wB);
  l.DA = q.lA * l.iwA;
  l.DB = q.lB * l.iwB;
  l.sig = kSlackHess + l.DA + l.DB;
  l.isig = rcp(l.sig);
  return l;
}

// Slack eliminated per row: ds = (rhs_s + D_A h.dp) / sig with rhs_s = -r_ds + rho_A + rho_B.
__device__ __forceinline__ RowDir hs_dir(const HsLin& l, double rhoA, double rhoB, double hdp) {
  RowDir d;
  d.ds = (-l.rds + rhoA + rhoB + l.DA * hdp) * l.isig;
  // gA = h.dp - ds written without the cancellation of two ~D_A-sized terms
  const double gA = (hdp * (kSlackHess + l.DB) + l.rds - rhoA - rhoB) * l.isig;
  d.dwA = -l.rpA - gA;
  d.dlA = l.DA * gA + rhoA;
  d.dwB = -l.rpB + d.ds;
  d.dlB = -l.DB * d.ds + rhoB;
  return d;
}

__device__ __forceinline__ RowDir hs_affine(const HsRow& q, const HsLin& l, double hdpa) {
  return hs_dir(l, l.DA * l.rpA - q.lA, l.DB * l.rpB - q.lB, hdpa);
}

__device__ __forceinline__ RowDir hs_corrector(const HsRow& q, const HsLin& l, double hdpa,
                                               double hdp, double sigma_mu) {
  const RowDir da = hs_affine(q, l, hdpa);
  const double rhoA = l.DA * l.rpA - q.lA + (sigma_mu - da.dwA * da.dlA) * l.iwA;
  const double rhoB = l.DB * l.rpB - q.lB + (sigma_mu - da.dwB * da.dlB) * l.iwB;
  return hs_dir(l, rhoA, rhoB, hdp);
}

__device__ __forceinline__ double hs_ratio(const HsRow& q, const RowDir& d) {
  return fmin(fmin(ratio(q.wA, d.dwA), ratio(q.lA, d.dlA)), fmin(ratio(q.wB, d.dwB), ratio(q.lB, d.dlB)));
}

// A two-sided bound lo <= y <= hi on a scalar y (an input or a position coordinate):
//   upper row  y - hi + wu = 0 (G = +1),  lower row  lo - y + wl = 0 (G = -1).
struct PairState {
  double wu, lu, wl, ll;
};
struct PairDir {
  double dwu, dlu, dwl, dll;
};
struct PairLin {
  double rpu, rpl, Du, Dl;
};
__device__ __forceinline__ PairLin pair_lin(const PairState& q, double y, double lo, double hi) {
  return {y - hi + q.wu, lo - y + q.wl, q.lu / q.wu, q.ll / q.wl};
}
__device__ __forceinline__ PairDir pair_dir(const PairState& q, const PairLin& l, double dya,
                                            double dy, double sigma_mu, bool corrector) {
  double rhou = l.Du * l.rpu - q.lu, rhol = l.Dl * l.rpl - q.ll;
  if (corrector) {
    const double dwu_a = -l.rpu - dya, dlu_a = l.Du * dya + rhou;
    const double dwl_a = -l.rpl + dya, dll_a = -l.Dl * dya + rhol;
    rhou += (sigma_mu - dwu_a * dlu_a) / q.wu;
    rhol += (sigma_mu - dwl_a * dll_a) / q.wl;
  }
  return {-l.rpu - dy, l.Du * dy + rhou, -l.rpl + dy, -l.Dl * dy + rhol};
}
__device__ __forceinline__ double pair_ratio(const PairState& q, const PairDir& d) {
  return fmin(fmin(ratio(q.wu, d.dwu), ratio(q.lu, d.dlu)), fmin(ratio(q.wl, d.dwl), ratio(q.ll, d.dll)));
}
// rho_u - rho_l of the affine step, and (base, unit) of the corrector split
__device__ __forceinline__ double pair_rho_aff(const PairState& q, const PairLin& l) {
  return (l.Du * l.rpu - q.lu) - (l.Dl * l.rpl - q.ll);
}

struct RowArrays {
  double *h0, *h1, *g, *s, *wA, *lA, *wB, *lB;
  __device__ __forceinline__ HsRow load(int64_t r) const {
    return {h0[r], h1[r], g[r], s[r], wA[r], lA[r], wB[r], lB[r]};
  }
};

__device__ __forceinline__ PairState box_state(const Lds& s, int n, int j) {
  return {s.bx[j], s.bx[n + j], s.bx[2 * n + j], s.bx[3 * n + j]};
}
__device__ __forceinline__ PairState pos_state(const Lds& s, int H, int t) {
  return {s.px[t], s.px[2 * H + t], s.px[4 * H + t], s.px[6 * H + t]};
}

// Sum kWaves per-step partials (wave 0, lane = step) in wave order.
template <int kWaves>
__device__ __forceinline__ double step_total(const double* red, int q, int lane) {
  double t = red[q * 64 + lane];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) t += red[(w * kPerStepQ + q) * 64 + lane];
  return t;
}

// ---------------------------------------------------------------------------------------------
// Clusters: one large problem (a C5 hand-off: 12 800 halfspace rows) on several workgroups.
// Every workgroup of a problem's cluster runs the whole interior-point method on its own — the
// Riccati factorisation, the solves and every decision are replicated, bitwise identical — and
// sweeps only its slice of the obstacles.  The row sums each sweep produces (per-step sums and a
// few scalars) are exchanged between the cluster's workgroups and combined in workgroup order by
// each of them, so every workgroup continues from the same totals and the solve stays
// deterministic.  Nothing else crosses workgroups: no broadcast, no leader.
// Exchange protocol (write-through payload, one counter per problem, no fences; the visibility
// rules of the MI355X guide, hand-off form "one lane signals by an agent-scope atomic add"):
//   wave 0 stores its workgroup's record with agent-scope (write-through) 8-B stores, drains them
//   (s_waitcnt vmcnt(0)), lane 0 adds 1 to the problem's counter; wave 0 polls the counter with
//   agent-scope loads until all `size` workgroups have arrived at this exchange, then every wave
//   reads the records with agent-scope loads (they bypass the CU's L1).  Records alternate
//   between two buffers: a workgroup can be at most one exchange ahead of the slowest reader.
// Every spin is bounded (MpcArgs::spin_ticks of the 100 MHz clock, default 10 ms); a workgroup
// that gives up adds kAbortBias to the counter, which releases every wait of every workgroup at
// once, and the problem ends CLUSTER_TIMEOUT (the fallback rollout) instead of hanging the launch.
// Divergence check: the protocol's liveness and the answer rest on every workgroup taking the same
// decisions (they are replicated, bitwise).  Each workgroup folds every replicated decision scalar
// (merit, step lengths, centring, polish residuals, factorisation outcomes) into a running 64-bit
// digest and publishes it, mixed with the exchange's site id and epoch, in its record; the gather
// compares every record's digest with its own.  A mismatch ends the problem at that exchange with
// CLUSTER_DIVERGED (and the abort bias releases any workgroup waiting elsewhere), instead of
// combining records from different sites or spinning until the time limit.  The counters are
// zeroed by a one-wave kernel in front of every launch; the clustered launch never has more
// workgroups than half the device's CUs, and asks for more LDS than two workgroups can share, so
// each workgroup has a CU of its own.
using gu64 = __attribute__((address_space(1))) unsigned long long;
__device__ __forceinline__ double op_apply(int op, double a, double b) {
  return op == kOpSum ? a + b : (op == kOpMax ? fmax(a, b) : fmin(a, b));
}
__device__ __forceinline__ double op_wave(int op, double v) {
  return op == kOpSum ? wave_sum_dpp(v) : (op == kOpMax ? wave_max(v) : wave_min(v));
}
__device__ __forceinline__ double op_identity(int op) {
  return op == kOpSum ? 0.0 : (op == kOpMax ? -INFINITY : INFINITY);
}
__device__ __forceinline__ void store_wt(double* p, double v) {  // write-through (sc1) 8-B store
  __hip_atomic_store((gu64*)p, static_cast<unsigned long long>(__double_as_longlong(v)),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_wt(const double* p) {  // agent-scope load (bypasses L1)
  return __longlong_as_double(static_cast<long long>(
      __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}
// 64-bit mix of a decision into a digest (xor-multiply, FNV-style); the operands are uniform
__device__ __forceinline__ uint64_t digest_mix(uint64_t d, uint64_t v) {
  d ^= v + 0x9e3779b97f4a7c15ull + (d << 6) + (d >> 2);
  return d * 0x100000001b3ull;
}

struct Cluster {
  int size, id;     // workgroups per problem, this workgroup's index in its cluster
  gu64* ctr;        // the problem's arrival counter
  double* xbuf;     // [2][size][kRec] exchange records
  double* cx;       // LDS scratch [kClusterScratch]
  uint64_t spin;    // wait bound (100 MHz ticks)
  uint64_t digest;  // running digest of every replicated decision (uniform in the workgroup)
  unsigned epoch;   // exchanges completed (the same count in every workgroup of the cluster)
  bool aborted;     // a wait gave up or the digests disagreed (uniform after that exchange)
  bool diverged;    // ... the digests disagreed
  __device__ __forceinline__ void note(double v) {
    digest = digest_mix(digest, static_cast<uint64_t>(__double_as_longlong(v)));
  }
  __device__ __forceinline__ void note_int(int64_t v) { digest = digest_mix(digest, static_cast<uint64_t>(v)); }
};

// Per-step values acc[q] (lane = step, this thread's rows) combined over the cluster with
// step_op, and NS scalars sv[i] with ops[i]; on return s.red[q * 64 + lane] holds the cluster's
// per-step totals and sv[i] the cluster's scalar totals (in every thread).  A sum counts every
// thread's value once: callers pass row contributions only (max / min may include replicated
// terms).  `site` names the call site (digest).  Contains barriers: every thread of the workgroup
// calls it.  After an abort (cl.aborted) the records it returns are not to be used.
template <int kWaves, int Q, int NS>
__device__ inline void cluster_combine(Cluster& cl, const Lds& s, const double* acc, int step_op,
                                       double* sv, const int* ops, int site) {
  static_assert(Q <= kPerStepQ && NS <= 4, "exchange layout");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double* cx = cl.cx;
#ifdef DRCVAR_MPC_STAMPS
  unsigned long long cl_t0 = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
  for (int q = 0; q < Q; ++q) s.red[(wave * kPerStepQ + q) * 64 + lane] = acc[q];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const double v = op_wave(ops[i], sv[i]);
    if (lane == 0) cx[i * kWaves + wave] = v;
  }
  __syncthreads();
  CL_STAMP(0);  // partials into LDS + barrier
  const int64_t half = static_cast<int64_t>(cl.epoch & 1u) * cl.size * kRec;
  const uint64_t mydig = digest_mix(digest_mix(cl.digest, static_cast<uint64_t>(site)), cl.epoch);
  // publish: wave q stores this workgroup's total of quantity q (waves combined in order), the
  // last wave the scalars and the digest; every storing wave drains its stores before the barrier
  // behind which one lane signals the arrival for all of them
  double* rec = cl.xbuf + half + static_cast<int64_t>(cl.id) * kRec;
  for (int q = wave; q < Q; q += kWaves) {
    double t = s.red[q * 64 + lane];
    for (int w = 1; w < kWaves; ++w) t = op_apply(step_op, t, s.red[(w * kPerStepQ + q) * 64 + lane]);
    store_wt(rec + q * 64 + lane, t);
  }
  if (wave == kWaves - 1) {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      if (lane == i) {
        double t = cx[i * kWaves];
        for (int w = 1; w < kWaves; ++w) t = op_apply(ops[i], t, cx[i * kWaves + w]);
        store_wt(rec + kRecScalars + i, t);
      }
    }
    if (lane == 8) store_wt(rec + kRecDigest, __longlong_as_double(static_cast<long long>(mydig)));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the record is out before the arrival
  CL_STAMP(1);  // combine over waves + record stores drained
  __syncthreads();
  CL_STAMP(2);  // barrier behind the drains
  if (wave == 0) {
#ifdef DRCVAR_MPC_STAMPS
    const unsigned long long arr_t = __builtin_amdgcn_s_memrealtime();
#endif
    if (lane == 0) __hip_atomic_fetch_add(cl.ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long target = (static_cast<unsigned long long>(cl.epoch) + 1ull) * cl.size;
    bool gave_up = false;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      const unsigned long long seen = __hip_atomic_load(cl.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long v =
          (static_cast<unsigned long long>(static_cast<unsigned>(
               __builtin_amdgcn_readfirstlane(static_cast<int>(seen >> 32)))) << 32) |
          static_cast<unsigned>(__builtin_amdgcn_readfirstlane(static_cast<int>(seen)));
      if (v >= target) {
        gave_up = v >= kAbortBias;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > cl.spin) {  // bounded: release everyone
        if (lane == 0) __hip_atomic_fetch_add(cl.ctr, kAbortBias, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        gave_up = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the poll
    if (lane == 0) cx[kCxGaveUp] = gave_up ? 1.0 : 0.0;
#ifdef DRCVAR_MPC_STAMPS
    if (lane == 0 && blockIdx.x < static_cast<unsigned>(cl.size) && cl.id < 32) {
      atomicAdd(&g_cl_arrive[cl.id], arr_t);
      atomicAdd(&g_cl_arrive[32 + cl.id], __builtin_amdgcn_s_memrealtime());
      atomicAdd(&g_cl_arrive[64 + cl.id], 1ull);
    }
#endif
    CL_STAMP(3);  // arrival + poll (includes waiting for the slowest workgroup)
  }
  __syncthreads();
  CL_STAMP(4);  // barrier after the poll
  // Gather: wave q sums quantity q (lane = step) over the records in workgroup order, eight
  // agent-scope loads in flight at a time — the same order in every workgroup of the cluster; the
  // last wave gathers the scalars and checks the digests (lane = record).  (16-B loads of step
  // pairs, two halves of the records per wave, measured slower: the extra live registers spilled.)
  const double* base = cl.xbuf + half;
  constexpr int kG = 8;  // agent-scope loads in flight per wave (16: no faster)
  for (int q = wave; q < Q; q += kWaves) {
    double v[kG];
    double t = op_identity(step_op);
    for (int c0 = 0; c0 < cl.size; c0 += kG) {
#pragma unroll
      for (int i = 0; i < kG; ++i)
        v[i] = c0 + i < cl.size ? load_wt(base + static_cast<int64_t>(c0 + i) * kRec + q * 64 + lane)
                                : op_identity(step_op);
#pragma unroll
      for (int i = 0; i < kG; ++i) t = op_apply(step_op, t, v[i]);
    }
    s.red[q * 64 + lane] = t;
  }
  if (wave == kWaves - 1) {
    const double* rl = base + static_cast<int64_t>(lane < cl.size ? lane : 0) * kRec;
    const uint64_t dg = static_cast<uint64_t>(__double_as_longlong(load_wt(rl + kRecDigest)));
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      double v = lane < cl.size ? load_wt(rl + kRecScalars + i) : op_identity(ops[i]);
      v = op_wave(ops[i], v);
      if (lane == 0) cx[kCxScalars + i] = v;
    }
    // (after a wait gave up the records are incomplete: no digest verdict on them)
    const bool differs = cx[kCxGaveUp] == 0.0 && __ballot(lane < cl.size && dg != mydig) != 0ull;
    if (differs && lane == 0)  // release whoever waits at another exchange
      __hip_atomic_fetch_add(cl.ctr, kAbortBias, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) cx[kCxDiverged] = differs ? 1.0 : 0.0;
  }
  __syncthreads();
  CL_STAMP(5);  // records gathered and combined
#pragma unroll
  for (int i = 0; i < NS; ++i) sv[i] = cx[kCxScalars + i];
  const bool div = cx[kCxDiverged] != 0.0;
  cl.diverged = cl.diverged || (div && !cl.aborted);
  cl.aborted = cl.aborted || div || cx[kCxGaveUp] != 0.0;
  ++cl.epoch;
}

// Row sweep of one thread (lane = halfspace step, obstacles o = wave, wave + kWaves, ...).  The
// rows of kSweep obstacles are loaded together before any is processed.  With two waves per SIMD
// in both kernel forms the other wave hides the row loads' latency, and a deeper sweep only adds
// registers: kSweep = 1 (measured against 2: H = 30 QP 0.573 -> 0.542 ms, C5 2.93 -> 2.75 ms,
// no spills on the 4-state forms).  Inside the body: q (the row), o, r (its workspace index).
constexpr int kSweep = 1;
#define ROW_SWEEP_BEGIN                                                              \
  for (int o0_ = o_lo + wave; o0_ < o_hi; o0_ += kSweep * kWaves) {                \
    HsRow qs_[kSweep];                                                               \
    _Pragma("unroll") for (int i_ = 0; i_ < kSweep; ++i_) {                          \
      const int o_ = o0_ + i_ * kWaves;                                              \
      if (o_ < o_hi) qs_[i_] = rows.load(static_cast<int64_t>(o_) * kRowStride + lane); \
    }                                                                                \
    _Pragma("unroll") for (int i_ = 0; i_ < kSweep; ++i_) {                          \
      const int o = o0_ + i_ * kWaves;                                               \
      if (o >= o_hi) break;                                                             \
      const int64_t r = static_cast<int64_t>(o) * kRowStride + lane;                 \
      (void)r;                                                                       \
      const HsRow q = qs_[i_];
#define ROW_SWEEP_END \
  }                   \
  }

// fold a replicated decision scalar into the cluster's digest (clustered form only)
#define CL_NOTE(x)                \
  do {                            \
    if constexpr (CL) cl.note(x); \
  } while (0)

// BLK threads per problem; HMX the horizon capacity of its LDS plan.  Every form targets two
// waves per SIMD (HIP's second launch bound; VGPR budget 256): 512 and 256 threads with two
// workgroups per CU, 128 threads with four.
// CL: clustered form — a.cl_size workgroups per problem (grid = problems x cl_size), each
// sweeping the obstacles [o_lo, o_hi) and exchanging row sums (cluster_combine).
template <int NU, int NX, int BLK, int HMX, bool CL = false, bool RL = false>
__global__ __launch_bounds__(BLK, (CL && BLK <= 256) ? 1 : 2) void mpc_ipm_kernel(MpcArgs a) {
  constexpr int kBlock = BLK;
  constexpr int kWaves = BLK / 64;
  static_assert(kWaves <= kMaxWaves, "LDS plan sized for kMaxWaves");
  extern __shared__ double lds_raw[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cl_size = CL ? a.cl_size : 1;
  const int64_t b = blockIdx.x / cl_size;
  const int cid = static_cast<int>(blockIdx.x - b * cl_size);
  const int n = a.n, H = a.H, K = a.K, O = a.O, nx = a.nx;
  const int o_lo = CL ? static_cast<int>((static_cast<int64_t>(O) * cid) / cl_size) : 0;
  const int o_hi = CL ? static_cast<int>((static_cast<int64_t>(O) * (cid + 1)) / cl_size) : O;
  const Lds s = carve<kWaves, NU, NX, HMX>(lds_raw, a.blob[a.off.ISO] != 0.0);
  static_assert(kWaves * kPerStepQ * 64 >= 16 * HMX, "s.red holds the isotropic factorisation's table");
  const double* H0 = a.blob + a.off.H0;
  double* ws = a.ws + a.ws_off + b * a.ws_pp;
  Cluster cl{};
  if constexpr (CL) {
    cl.size = cl_size;
    cl.id = cid;
    cl.ctr = (gu64*)(a.ws + b * kCtrlDoubles);
    cl.xbuf = ws + kRowArrays * static_cast<int64_t>(O) * kStepPad + static_cast<int64_t>(cl_size) * kBestPad;
    cl.cx = lds_raw + LdsPlan<kWaves, NU, NX, HMX>::total;
    cl.spin = a.spin_ticks;
    cl.digest = 0;
    cl.epoch = 0;
    cl.aborted = false;
    cl.diverged = false;
  }
  (void)cl;
  (void)O;
#ifdef DRCVAR_MPC_STAMPS
  unsigned long long stamp_acc[kStampSlots] = {};
  unsigned long long stamp_last = __builtin_amdgcn_s_memtime();
#endif
  // rows: [O][8 fields][64 steps] — one base, the field is an immediate offset
  // The clustered form keeps its slice of the rows in LDS when the launch found room for it
  // (the C5 hand-off: 16 obstacles x kRowStride doubles = 80 KB beside the 78 KB plan, one
  // workgroup per CU): the row sweeps then wait on LDS instead of L2 (round 5); the layout and
  // the arithmetic are the workspace's, indexed by the same r (the base is offset by o_lo).
  // (RL: a kernel form of its own, so that the row accesses compile to LDS instructions)
  double* rbase = ws;
  if constexpr (CL && RL) {
    rbase = lds_raw + (LdsPlan<kWaves, NU, NX, HMX>::total + kClusterScratch) - static_cast<int64_t>(o_lo) * kRowStride;
  }
  const RowArrays rows{rbase, rbase + kStepPad, rbase + 2 * kStepPad, rbase + 3 * kStepPad,
                       rbase + 4 * kStepPad, rbase + 5 * kStepPad, rbase + 6 * kStepPad, rbase + 7 * kStepPad};
  const int64_t pitch = static_cast<int64_t>(O) * kStepPad;
  const double* x0 = a.x0 + b * a.x0_sp;
  const double* xr = a.xr + b * a.xr_sp;

  // ------------------------------- setup -------------------------------
  for (int t = tid; t < H * 2 * NU; t += kBlock) s.Mp[t] = a.blob[a.off.Mp + t];
  // model matrices, zero-padded to the NX x NX (kMx-strided) blocks the Riccati code sweeps
  for (int t = tid; t < kMx * kMx; t += kBlock) {
    const int r = t / kMx, c = t - r * kMx;
    const bool in = r < nx && c < nx;
    s.Am[t] = in ? a.blob[a.off.A + r * nx + c] : 0.0;
    s.Qm[t] = in ? a.blob[a.off.Q + r * nx + c] : 0.0;
  }
  for (int t = tid; t < kMx * NU; t += kBlock) s.Bm[t] = t < nx * NU ? a.blob[a.off.B + t] : 0.0;
  for (int t = tid; t < NU * NU; t += kBlock) s.Rm[t] = a.blob[a.off.R + t];
  for (int t = tid; t < 2 * kMx; t += kBlock) {
    const int r = t / kMx, c = t - r * kMx;
    s.Cm[t] = c < nx ? a.blob[a.off.C + r * nx + c] : 0.0;
  }
  for (int t = tid; t < 2 * H; t += kBlock) {
    const double* ca = a.blob + a.off.CA + static_cast<int64_t>(t) * nx;
    double acc = 0.0;
    for (int q = 0; q < nx; ++q) acc += ca[q] * x0[q];
    s.c[t] = acc;
  }
  // x_ref[1..H] staged in LDS (s.xs, the output rollout's buffer, is free until then): every
  // thread of the two sums below reads all of it
  for (int e = tid; e < H * nx; e += kBlock) {
    const int t = e / nx, q = e - t * nx;
    s.xs[e] = xr[(t + 1) * a.xr_st + q];
  }
  __syncthreads();
  // f = F1 x0 - F2 xr, summed in this order on purpose: splitting the sum (as the Gp'z sums are)
  // moved the rounding of f enough to stall one degenerate test problem (generic1, H = 64) at
  // merit 1e-8 with a failing polish (degenerate active sets defeat the polish)
  // (the row of F2 is loaded 16 doubles at a time, all in flight, ahead of the chain: one thread
  // per row, so the row's ~H nx loads used to sit on the dependent chain one round trip at a time).
  // (Round 5 measured f through the dynamics on one wave for the isotropic models -- 2 Gx'Q (Phi x0
  // - xr) by the free response and its adjoint, two H-step recurrences: C5 setup 47 k -> 21 k
  // cycles but 99 k -> 90 k in all, and its rounding sent one degenerate problem of bench.py's
  // distinct batch from one polish attempt to ten; not kept.)
  for (int j = tid; j < n; j += kBlock) {
    const double* f1 = a.blob + a.off.F1 + static_cast<int64_t>(j) * nx;
    const double* f2 = a.blob + a.off.F2 + static_cast<int64_t>(j) * H * nx;
    double acc = 0.0;
    for (int q = 0; q < nx; ++q) acc += f1[q] * x0[q];
    const int len = H * nx;  // f2[t nx + q] in (t, q) order, as the nested loop summed it
    for (int e0 = 0; e0 < len; e0 += 16) {
      double fv[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) fv[e] = e0 + e < len ? f2[e0 + e] : 0.0;
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (e0 + e < len) acc -= fv[e] * s.xs[e0 + e];
    }
    s.f[j] = acc;
  }
  MPC_PHASE(17);  // setup: model, c, x_ref staging, f
  // starting inputs: the tracking optimum without rows, u = -H0^-1 f = UF1 x0 + UF2 xr (condensed
  // on the host), strictly inside the input box; the UF2 x_ref sums as interleaved partial sums
  // (threads (j, part)), so no thread carries a chain of H nx loads
  constexpr int kParts = kBlock >= 512 ? 4 : 2;
  const bool have_uf = a.blob[a.off.UFOK] != 0.0;
  if (have_uf) {
    for (int e = tid; e < n * kParts; e += kBlock) {
      const int j = e / kParts, part = e - (e / kParts) * kParts;
      const double* g2 = a.blob + a.off.UF2 + static_cast<int64_t>(j) * H * nx;
      double acc = 0.0;
      for (int t = part; t < H; t += kParts)
        for (int q = 0; q < nx; ++q) acc += g2[t * nx + q] * s.xs[t * nx + q];
      s.red[e] = acc;
    }
  }
  __syncthreads();
  for (int j = tid; j < n; j += kBlock) {
    double u0 = 0.0;
    if (have_uf) {
      const double* g1 = a.blob + a.off.UF1 + static_cast<int64_t>(j) * nx;
      for (int q = 0; q < nx; ++q) u0 += g1[q] * x0[q];
#pragma unroll
      for (int part = 0; part < kParts; ++part) u0 += s.red[j * kParts + part];
    }
    if (a.has_u) {
      const int ai = j % NU;
      const double span = a.umax[ai] - a.umin[ai];
      u0 = fmin(fmax(u0, a.umin[ai] + kStartBoxMargin * span), a.umax[ai] - kStartBoxMargin * span);
    }
    s.u[j] = u0;
  }
  __syncthreads();
  positions<NU, kBlock>(s, s.u, s.p, s.c, H);
  __syncthreads();

  // Start (round 4): every inequality on the central path of barrier parameter mu0 at the starting
  // inputs u (above).  A halfspace row with residual r = h.p + g takes the slack s > max(r, 0) that
  // minimises 50 s + 50 s^2 - mu0 log(s - r) - mu0 log(s) (start_slack), so that w_hs = s - r,
  // w_s = s, lambda = mu0 / w and the row's own stationarity 50 + 100 s = lambda_hs + lambda_s hold,
  // except that lambda_hs is capped at 25 (a row violated at u would start with lambda_hs ~ 50 +
  // 100 r: main.py's mean-metric filter at C5 size then took 20-23 iterations instead of 16-17);
  // the bound rows take lambda = mu0 / w.  Counted on the CPU restatement (scripts/micro/ipm_lab.py
  // --start central_mu=20,central_mu_few=1,u_free=1,many=64,lam_cap=25 on the problem sets of
  // scripts/micro/make_qp_set.py) against the round-3 start (u = 0, unit or (5, 1.5) duals):
  // bench-like DR-CVaR C5 problems 78 -> 64 iterations over six seeds (the degenerate C5 fixture
  // 14 -> 10), main.py's three filters at C5 size and H = 20 / 10 obstacles 180 -> 151 (C5 mean
  // 50 -> 50, C5 CVaR 42 -> 33), main.py-like problems with 3-10 obstacles 106 -> 76.
  MPC_PHASE(18);  // setup: starting inputs and their positions
  const bool many_rows = O >= kManyRowsObstacles;
  const double mu0 = many_rows ? kStartMuMany : kStartMuFew;
  double gmax = 0.0;
  if (lane < K) {
    const double p0 = s.p[2 * lane], p1 = s.p[2 * lane + 1];
    for (int o = o_lo + wave; o < o_hi; o += kWaves) {
      const double* hp = a.hs_h + b * a.h_sp + o * a.h_so + lane * a.h_sk;
      const double g = a.hs_g[b * a.g_sp + o * a.g_so + lane * a.g_sk];
      const double h0 = hp[0], h1 = hp[1];
      const int64_t r = static_cast<int64_t>(o) * kRowStride + lane;
      rows.h0[r] = h0;
      rows.h1[r] = h1;
      rows.g[r] = g;
      const double res = h0 * p0 + h1 * p1 + g;
      const double sv = start_slack(res, mu0);
      const double wA = sv - res;
      rows.s[r] = sv;
      rows.wA[r] = wA;
      rows.lA[r] = fmin(mu0 * rcp(wA), kStartDualCap);
      rows.wB[r] = sv;
      rows.lB[r] = mu0 * rcp(sv);
      gmax = fmax(gmax, fabs(g));
    }
  }
  if (a.has_u) {
    for (int j = tid; j < n; j += kBlock) {
      const int ai = j % NU;
      const double wu = fmax(a.umax[ai] - s.u[j], kStartFloorW), wl = fmax(s.u[j] - a.umin[ai], kStartFloorW);
      s.bx[j] = wu;
      s.bx[n + j] = mu0 / wu;
      s.bx[2 * n + j] = wl;
      s.bx[3 * n + j] = mu0 / wl;
      gmax = fmax(gmax, fmax(fabs(a.umin[ai]), fabs(a.umax[ai])));
    }
  }
  if (a.has_p) {
    for (int t = tid; t < 2 * H; t += kBlock) {
      const int i = t & 1;
      const double wu = fmax(a.pmax[i] - s.p[t], kStartFloorW), wl = fmax(s.p[t] - a.pmin[i], kStartFloorW);
      s.px[t] = wu;
      s.px[2 * H + t] = mu0 / wu;
      s.px[4 * H + t] = wl;
      s.px[6 * H + t] = mu0 / wl;
      gmax = fmax(gmax, fmax(fabs(a.pmin[i]), fabs(a.pmax[i])));
    }
  }
  MPC_PHASE(19);  // setup: the rows' and bounds' starting points
  double fmaxv = 0.0;
  for (int j = tid; j < n; j += kBlock) fmaxv = fmax(fmaxv, fabs(s.f[j]));
  if constexpr (CL) {  // |g| over every row of the problem: each workgroup reads all of hs_g (a
    // cluster exchange before round 4; a maximum is exact in any order, so every workgroup agrees),
    // eight loads in flight per lane (one at a time, a C5 workgroup waited for 32 in series)
    if (lane < K) {
      for (int o0 = wave; o0 < O; o0 += 8 * kWaves) {
        double gv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int o = o0 + q * kWaves;
          gv[q] = o < O ? a.hs_g[b * a.g_sp + o * a.g_so + lane * a.g_sk] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) gmax = fmax(gmax, fabs(gv[q]));
      }
    }
  }
  {
    double unused = 0.0;
    block_sum_max_max<kWaves>(unused, gmax, fmaxv, s.sc);
  }
  const double scale_d = 1.0 + gmax;
  const double scale_q = 1.0 + fmax(fmaxv, kSlackLin);
  const double m_ineq = 2.0 * O * K + (a.has_u ? 2.0 * n : 0.0) + (a.has_p ? 4.0 * H : 0.0);

  MPC_PHASE(0);
  int status = DRCVAR_MPC_STATUS_MAX_ITER;
  int it = 0, best_it = 0;
  double mu = 0.0, rp = 0.0, rd = 0.0, best_merit = kHuge;
  double* best_u = ws + kRowArrays * pitch + static_cast<int64_t>(cid) * kBestPad;  // [n] best iterate
  // P1's row part — per-step sums of the weights / duals / affine rhs, the gap and the residual
  // maxima at positions (p0, p1) — accumulated by each thread for its rows.  It runs fused with
  // the previous iteration's update pass (P5): the rows are swept once per iteration less.
  double acc[kPerStepQ], gap_rows, rpm_rows, rdm_rows;
  auto p1_clear = [&]() {
#pragma unroll
    for (int q = 0; q < kPerStepQ; ++q) acc[q] = 0.0;
    gap_rows = rpm_rows = rdm_rows = 0.0;
  };
  auto p1_row = [&](const HsRow& q, double p0, double p1) {
    const HsLin l = hs_lin(q, p0, p1);
    const double om = l.DA * (kSlackHess + l.DB) * l.isig;
    const double rhoA = l.DA * l.rpA - q.lA, rhoB = l.DB * l.rpB - q.lB;
    const double coef = rhoA - l.DA * (-l.rds + rhoA + rhoB) * l.isig;
    acc[0] += q.lA * q.h0;
    acc[1] += q.lA * q.h1;
    acc[2] += om * q.h0 * q.h0;
    acc[3] += om * q.h0 * q.h1;
    acc[4] += om * q.h1 * q.h1;
    acc[5] += coef * q.h0;
    acc[6] += coef * q.h1;
    gap_rows += q.wA * q.lA + q.wB * q.lB;
    rpm_rows = fmax(rpm_rows, fmax(fabs(l.rpA), fabs(l.rpB)));
    rdm_rows = fmax(rdm_rows, fabs(l.rds));
  };
  // Rounds: the interior-point method to tol, then the polish.  When the polish fails on a problem
  // that met tol (degenerate active sets: more binding rows than freedom), the interior-point
  // state the polish overwrote is restored and the method continues for up to kResumeIters
  // iterations towards tol * kResumeTol, then polishes once more; its iterate stands if that
  // polish fails too.  (Degenerate problems converge in u only like sqrt(mu): at merit 1e-8 the
  // answer can be 1e-5 off.)  Every decision is uniform, so a cluster takes the rounds together.
  double tol_r = a.tol;
  int it_end = a.max_iter;
  int polish_attempts = 0;
  bool polished = false;
  // saved across a failed polish: the rows' s and w_hs (fields 8, 9 of every obstacle block) and
  // the bound states bx [4 n], px [8 H] (behind the best iterate)
#define SAVED_S (rbase + 8 * kStepPad)
#define SAVED_W (rbase + 9 * kStepPad)
#define SAVED_B (ws + kRowArrays * pitch + static_cast<int64_t>(cid) * kBestPad + 128)
  it = 1;
  // one round: P1 of the current iterate, the interior-point loop, the polish; true when a resume
  // round should follow.  Inlined at both call sites (a loop around it, or an out-of-line
  // function, made the compiler spill inside the interior-point loop: C5 QP +5 % / +40 %).
  bool early = false;  // the first round left for an early polish (kEarlyPolishMerit)
  auto ipm_round = [&](const int round) __attribute__((always_inline)) -> bool {
  bool converged = false;  // this round's loop met its tolerance (the factorisation beside it stands)
  // positions of the starting (or restored) iterate and its P1 row pass
  positions<NU, kBlock>(s, s.u, s.p, s.c, H);
  __syncthreads();
  p1_clear();
  if (lane < K) {
    const double p0 = s.p[2 * lane], p1 = s.p[2 * lane + 1];
    ROW_SWEEP_BEGIN
      p1_row(q, p0, p1);
    ROW_SWEEP_END
  }
  for (; it <= it_end; ++it) {
    MPC_PHASE(15);

    // ---- P1: residuals, weights, per-step S / v / affine rhs (row sums already taken) ----
    {
      double gap = gap_rows, rpm = rpm_rows, rdm = rdm_rows;
      if constexpr (CL) {  // the cluster's row sums; the gap total enters once (thread 0)
        double sv[3] = {gap_rows, rpm_rows, rdm_rows};
        const int ops[3] = {kOpSum, kOpMax, kOpMax};
        MPC_PHASE(1);
        cluster_combine<kWaves, kPerStepQ, 3>(cl, s, acc, kOpSum, sv, ops, kSiteP1);
        MPC_PHASE(16);  // cluster exchange
        if (cl.aborted) break;  // uniform: the cluster disagreed or a wait gave up
        gap = tid == 0 ? sv[0] : 0.0;
        rpm = sv[1];
        rdm = sv[2];
      } else {
#pragma unroll
        for (int q = 0; q < kPerStepQ; ++q) s.red[(wave * kPerStepQ + q) * 64 + lane] = acc[q];
        __syncthreads();
      }
      if (wave == 0 && lane < H) {
        double tot[kPerStepQ];
#pragma unroll
        for (int q = 0; q < kPerStepQ; ++q)
          tot[q] = lane < K ? (CL ? s.red[q * 64 + lane] : step_total<kWaves>(s.red, q, lane)) : 0.0;
        if (a.has_p) {
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int t = 2 * lane + i;
            const PairState q = pos_state(s, H, t);
            const PairLin l = pair_lin(q, s.p[t], a.pmin[i], a.pmax[i]);
            tot[i] += q.lu - q.ll;                    // v
            tot[i == 0 ? 2 : 4] += l.Du + l.Dl;       // S diagonal
            tot[5 + i] += pair_rho_aff(q, l);         // affine rhs
            gap += q.wu * q.lu + q.wl * q.ll;
            rpm = fmax(rpm, fmax(fabs(l.rpu), fabs(l.rpl)));
          }
        }
        s.v[2 * lane] = tot[0];
        s.v[2 * lane + 1] = tot[1];
        s.S[lane] = tot[2];
        s.S[H + lane] = tot[3];
        s.S[2 * H + lane] = tot[4];
        s.za[2 * lane] = tot[5];
        s.za[2 * lane + 1] = tot[6];
      }
      for (int j = tid; j < n; j += kBlock) {
        if (a.has_u) {
          const int ai = j % NU;
          const PairState q = box_state(s, n, j);
          const PairLin l = pair_lin(q, s.u[j], a.umin[ai], a.umax[ai]);
          s.DU[j] = l.Du + l.Dl;
          s.rU[j] = pair_rho_aff(q, l);
          gap += q.wu * q.lu + q.wl * q.ll;
          rpm = fmax(rpm, fmax(fabs(l.rpu), fabs(l.rpl)));
        } else {
          s.DU[j] = 0.0;
          s.rU[j] = 0.0;
        }
      }
      if (tid == 0) {  // the pipelined affine solve's progress words (no step finished yet)
        *prog_word(s, 0) = H;
        *prog_word(s, 1) = H;
      }
      __syncthreads();
      // Wave 0 factorises K (it needs S and DU only) while the other waves form the dual residual
      // of the inputs r_du = H0 u + f + Gp' v + (lUu - lUl) and the input part of the affine rhs,
      // dua = -r_du - rU (its Gp' za part enters the solve as a state source).  For NX <= 4 wave 1
      // alone, by the two recurrences of dual_residual_wave (round 5); otherwise one thread per
      // input (gpt_row: the partial-sum order of gpt_parts).  The factorisation is speculative: on
      // the iteration whose merit meets the tolerance it serves the polish's active-set guess.
      // For NX <= 4 a third wave (wave 1 after its rows in the 128-thread form) runs the backward
      // half of the affine solve one step behind the factorisation (affine_backward_follow: kff
      // into s.du, the forward sources into s.red, the solve maps into s.SM), so that after it only
      // the forward half is left (round 5).  The waves hand over through the progress words.
      WAVE_SPAN_BEGIN();
      if (wave == 0) {
        riccati_factor_wave0<NU, NX, false, NX <= 4 && kPipe>(s, H);
      } else if constexpr (NX <= 4) {
        if (wave == 1) rdm = fmax(rdm, dual_residual_wave<NU>(s, H, n, a.has_u, s.xs));
        if (kPipe && wave == (kWaves >= 3 ? 2 : 1)) affine_backward_follow<NU>(s, H, s.dua, s.za);
      } else {
        // (NX > 4 keeps the affine rhs's Gp' za in these rows: handing it to the solve as for
        // the other systems made the 4-input, 8-state kernels diverge on every problem of
        // test_gpu_many_problems_every_form[generic4] — those kernels spill ~350-550 VGPRs, and
        // the same sums in newton_solve, by gpt_parts or gpt_row, with or without an extra
        // barrier, all failed, while this form passes; round 5)
        for (int j = tid - 64; j < n; j += kBlock - 64) {
          double r = s.f[j] + gpt_row<NU, kBlock>(s, s.v, H0, s.u, j, n, H);
          if (a.has_u) r += s.bx[n + j] - s.bx[3 * n + j];
          s.rdu[j] = r;
          rdm = fmax(rdm, fabs(r));
          s.dua[j] = -r - s.rU[j] - gpt_row<NU, kBlock>(s, s.za, nullptr, nullptr, j, n, H);
        }
      }
      WAVE_SPAN_END();
      block_sum_max_max<kWaves>(gap, rpm, rdm, s.sc);  // its barriers also end the factorisation
      mu = m_ineq > 0.0 ? gap / m_ineq : 0.0;
      rp = rpm;
      rd = rdm;
      if (!isfinite(gap) || !isfinite(rp) || !isfinite(rd)) {
        status = DRCVAR_MPC_STATUS_NUMERICAL;
        break;
      }
      const double merit = fmax(fmax(rp / scale_d, rd / scale_q), mu);
      CL_NOTE(merit);
      if (merit <= tol_r) {
        converged = true;
        status = DRCVAR_MPC_STATUS_OPTIMAL;
        best_merit = merit;
        break;
      }
      if (round == 0 && a.polish && merit <= (many_rows ? kEarlyPolishMeritMany : kEarlyPolishMerit)) {
        converged = true;  // (the factorisation beside this P1 serves the active-set guess)
        early = true;
        // the best iterate is this one (u, merit and iteration together): the post-loop restore
        // and a resume after a failed early polish then start from the state the rows describe
        best_merit = merit;
        best_it = it;
        for (int j = tid; j < n; j += kBlock) best_u[j] = s.u[j];
        break;
      }
      if (merit < best_merit) {  // uniform: every thread holds the same merit
        best_merit = merit;
        best_it = it;
        for (int j = tid; j < n; j += kBlock) best_u[j] = s.u[j];
      }
      if (best_merit < kPolishMerit && it - best_it >= 8) break;  // stalled at the accuracy floor
    }
    const double gap = mu * m_ineq;
    MPC_PHASE(1);

    // ---- factor K = H0 + diag(DU) + sum_k Mp' S_k Mp (Riccati; wave 0 ran the recursion above,
    // beside the affine rhs) ----
    MPC_PHASE(2);
    // A failed pivot close to the optimum hands over to the polish (the usual end of a solve
    // whose barrier weights have outgrown fp64); further out the stationary form takes over.
    // (NX <= 4: when the factorisation succeeded, the pipelined backward half of the affine solve
    // has run beside it and left the solve maps; only the forward half follows)
    const bool piped = kPipe && NX <= 4 && s.sc[62] == 0.0;  // uniform
    if (!piped && !riccati_factor_finish<NU, NX>(s, H) &&
        (best_merit <= kPolishMerit || !riccati_factor<NU, NX, true>(s, H))) {
      status = DRCVAR_MPC_STATUS_NUMERICAL;
      break;
    }
    CL_NOTE(s.Ri[0]);  // the factorisation (its first pivot's inverse)
    MPC_PHASE(3);
    if constexpr (NX <= 4) {
      if (piped) {  // the backward recurrence ran beside the factorisation: its tail, the forward half
        dpp_backward_tail<NU, kBlock>(s, H, s.dua, s.du);
        dpp_forward<NU, kBlock>(s, H, s.du, s.dua, s.dpa, nullptr);  // direction, positions
      }
      else newton_solve<NU, NX, kBlock, HMX>(s, H, n, s.dua, s.dpa, nullptr, s.za);
    } else {  // (dua holds the whole rhs, Gp' za included)
      newton_solve<NU, NX, kBlock, HMX>(s, H, n, s.dua, s.dpa);
    }
    MPC_PHASE(4);

    // ---- P2+P3: affine step length, affine gap, corrector rhs — one sweep of the rows ----
    // The corrector rhs sums do not depend on the affine step a_aff, and a row's affine gap
    // (w + a dw)(l + a dl) is a quadratic in it: the sweep keeps sum w l, sum (w dl + l dw) and
    // sum dw dl per thread and evaluates the quadratic once a_aff is known (the rows used to be
    // swept twice, before and after the block minimum).
    double amax = kHuge;
    {
      double acc[4] = {0, 0, 0, 0};
      double gq0 = 0.0, gq1 = 0.0, gq2 = 0.0;
      if (lane < K) {
        const double p0 = s.p[2 * lane], p1 = s.p[2 * lane + 1];
        const double d0 = s.dpa[2 * lane], d1 = s.dpa[2 * lane + 1];
        ROW_SWEEP_BEGIN
          const HsLin l = hs_lin(q, p0, p1);
          const RowDir d = hs_affine(q, l, q.h0 * d0 + q.h1 * d1);
          amax = fmin(amax, hs_ratio(q, d));
          gq0 += q.wA * q.lA + q.wB * q.lB;
          gq1 += (q.wA * d.dlA + q.lA * d.dwA) + (q.wB * d.dlB + q.lB * d.dwB);
          gq2 += d.dwA * d.dlA + d.dwB * d.dlB;
          const double rhoA_b = l.DA * l.rpA - q.lA - d.dwA * d.dlA * l.iwA;
          const double rhoB_b = l.DB * l.rpB - q.lB - d.dwB * d.dlB * l.iwB;
          const double cb = rhoA_b - l.DA * (-l.rds + rhoA_b + rhoB_b) * l.isig;
          const double cu = l.iwA - l.DA * (l.iwA + l.iwB) * l.isig;
          acc[0] += cb * q.h0;
          acc[1] += cb * q.h1;
          acc[2] += cu * q.h0;
          acc[3] += cu * q.h1;
        ROW_SWEEP_END
      }
      if constexpr (CL) {  // the cluster's rows: step length (min), gap quadratic, rhs sums
        double sv[4] = {amax, gq0, gq1, gq2};
        const int ops[4] = {kOpMin, kOpSum, kOpSum, kOpSum};
        MPC_PHASE(5);
        cluster_combine<kWaves, 4, 4>(cl, s, acc, kOpSum, sv, ops, kSiteP23);
        MPC_PHASE(16);  // cluster exchange
        if (cl.aborted) break;
        amax = sv[0];
        gq0 = tid == 0 ? sv[1] : 0.0;  // the quadratic enters the block sum once
        gq1 = tid == 0 ? sv[2] : 0.0;
        gq2 = tid == 0 ? sv[3] : 0.0;
      } else {
        // published by the barriers of block_min below (positions' reads of s.red ended at the
        // barrier before this sweep)
#pragma unroll
        for (int q = 0; q < 4; ++q) s.red[(wave * kPerStepQ + q) * 64 + lane] = acc[q];
      }
      if (a.has_u) {
        for (int j = tid; j < n; j += kBlock) {
          const int ai = j % NU;
          const PairState q = box_state(s, n, j);
          const PairLin l = pair_lin(q, s.u[j], a.umin[ai], a.umax[ai]);
          amax = fmin(amax, pair_ratio(q, pair_dir(q, l, 0.0, s.dua[j], 0.0, false)));
        }
      }
      if (a.has_p) {
        for (int t = tid; t < 2 * H; t += kBlock) {
          const int i = t & 1;
          const PairState q = pos_state(s, H, t);
          const PairLin l = pair_lin(q, s.p[t], a.pmin[i], a.pmax[i]);
          amax = fmin(amax, pair_ratio(q, pair_dir(q, l, 0.0, s.dpa[t], 0.0, false)));
        }
      }
      const double a_aff = fmin(1.0, block_min<kWaves>(amax, s.sc));
      double gap_aff = fma(fma(gq2, a_aff, gq1), a_aff, gq0);
      if (wave == 0 && lane < H) {
        double tot[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          tot[q] = lane < K ? (CL ? s.red[q * 64 + lane] : step_total<kWaves>(s.red, q, lane)) : 0.0;
        if (a.has_p) {
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int t = 2 * lane + i;
            const PairState q = pos_state(s, H, t);
            const PairLin l = pair_lin(q, s.p[t], a.pmin[i], a.pmax[i]);
            const PairDir d = pair_dir(q, l, 0.0, s.dpa[t], 0.0, false);
            gap_aff += (q.wu + a_aff * d.dwu) * (q.lu + a_aff * d.dlu) +
                       (q.wl + a_aff * d.dwl) * (q.ll + a_aff * d.dll);
            tot[i] += (l.Du * l.rpu - q.lu - d.dwu * d.dlu / q.wu) -
                      (l.Dl * l.rpl - q.ll - d.dwl * d.dll / q.wl);
            tot[2 + i] += 1.0 / q.wu - 1.0 / q.wl;
          }
        }
        s.za[2 * lane] = tot[0];
        s.za[2 * lane + 1] = tot[1];
        s.zu[2 * lane] = tot[2];
        s.zu[2 * lane + 1] = tot[3];
      }
      for (int j = tid; j < n; j += kBlock) {
        if (a.has_u) {
          const int ai = j % NU;
          const PairState q = box_state(s, n, j);
          const PairLin l = pair_lin(q, s.u[j], a.umin[ai], a.umax[ai]);
          const PairDir d = pair_dir(q, l, 0.0, s.dua[j], 0.0, false);
          gap_aff += (q.wu + a_aff * d.dwu) * (q.lu + a_aff * d.dlu) +
                     (q.wl + a_aff * d.dwl) * (q.ll + a_aff * d.dll);
          s.rU[j] = (l.Du * l.rpu - q.lu - d.dwu * d.dlu / q.wu) -
                    (l.Dl * l.rpl - q.ll - d.dwl * d.dll / q.wl);
          s.rUu[j] = 1.0 / q.wu - 1.0 / q.wl;
        } else {
          s.rU[j] = 0.0;
          s.rUu[j] = 0.0;
        }
      }
      gap_aff = block_sum<kWaves>(gap_aff, s.sc);  // its barriers also publish za / zu / rU / rUu
      const double ratio_g = gap > 0.0 ? gap_aff / gap : 0.0;
      const double sigma_mu = ratio_g * ratio_g * ratio_g * mu;
      CL_NOTE(a_aff);
      CL_NOTE(sigma_mu);
      s.sc[63] = sigma_mu;  // same value in every thread; kept for P4/P5
      // Gp' is linear: Gp' za + sigma_mu Gp' zu = Gp' (za + sigma_mu zu), combined in place and
      // handed to the solve as its state source
      for (int t = tid; t < 2 * H; t += kBlock) s.zu[t] = s.za[t] + sigma_mu * s.zu[t];
      for (int j = tid; j < n; j += kBlock) s.du[j] = -s.rdu[j] - (s.rU[j] + sigma_mu * s.rUu[j]);
      __syncthreads();
    }
    const double sigma_mu = s.sc[63];
    MPC_PHASE(5);
    newton_solve<NU, NX, kBlock, HMX>(s, H, n, s.du, s.dp, nullptr, s.zu);
    MPC_PHASE(4);

    // ---- P4: corrector step length ----
    amax = kHuge;
    if (lane < K) {
      const double p0 = s.p[2 * lane], p1 = s.p[2 * lane + 1];
      const double a0 = s.dpa[2 * lane], a1 = s.dpa[2 * lane + 1];
      const double d0 = s.dp[2 * lane], d1 = s.dp[2 * lane + 1];
      ROW_SWEEP_BEGIN
        const HsLin l = hs_lin(q, p0, p1);
        amax = fmin(amax, hs_ratio(q, hs_corrector(q, l, q.h0 * a0 + q.h1 * a1, q.h0 * d0 + q.h1 * d1, sigma_mu)));
      ROW_SWEEP_END
    }
    if constexpr (CL) {
      const int ops[1] = {kOpMin};
      MPC_PHASE(5);
      cluster_combine<kWaves, 0, 1>(cl, s, nullptr, kOpSum, &amax, ops, kSiteP4);
      MPC_PHASE(16);  // cluster exchange
      if (cl.aborted) break;
    }
    if (a.has_u) {
      for (int j = tid; j < n; j += kBlock) {
        const int ai = j % NU;
        const PairState q = box_state(s, n, j);
        const PairLin l = pair_lin(q, s.u[j], a.umin[ai], a.umax[ai]);
        amax = fmin(amax, pair_ratio(q, pair_dir(q, l, s.dua[j], s.du[j], sigma_mu, true)));
      }
    }
    if (a.has_p) {
      for (int t = tid; t < 2 * H; t += kBlock) {
        const int i = t & 1;
        const PairState q = pos_state(s, H, t);
        const PairLin l = pair_lin(q, s.p[t], a.pmin[i], a.pmax[i]);
        amax = fmin(amax, pair_ratio(q, pair_dir(q, l, s.dpa[t], s.dp[t], sigma_mu, true)));
      }
    }
    // fraction to the boundary: 0.995, closing to 1 - mu near the solution — a fixed 0.995 caps
    // the tail at a factor-200 reduction per iteration (measured 6e-2, 3e-4, 2e-6, 8e-9, 4e-11)
    double alpha = fmin(1.0, (1.0 - fmin(1.0 - kStepFrac, mu)) * block_min<kWaves>(amax, s.sc));
    if constexpr (CL) {
      if (a.perturb_group == cid + 1 && it == a.perturb_iter) alpha *= 1.0 - 0x1p-20;  // test hook
      cl.note(alpha);
    }

    // ---- P5: update (the halfspace rows in the fused pass below) ----
    // this lane's step: positions and directions of the iterate being updated
    double p0 = 0.0, p1 = 0.0, a0 = 0.0, a1 = 0.0, d0 = 0.0, d1 = 0.0;
    if (lane < K) {
      p0 = s.p[2 * lane];
      p1 = s.p[2 * lane + 1];
      a0 = s.dpa[2 * lane];
      a1 = s.dpa[2 * lane + 1];
      d0 = s.dp[2 * lane];
      d1 = s.dp[2 * lane + 1];
    }
    // box / position rows: every thread reads its own entries only, so no barrier is needed
    // between computing the direction and writing the update
    if (a.has_u) {
      for (int j = tid; j < n; j += kBlock) {
        const int ai = j % NU;
        const PairState q = box_state(s, n, j);
        const PairLin l = pair_lin(q, s.u[j], a.umin[ai], a.umax[ai]);
        const PairDir d = pair_dir(q, l, s.dua[j], s.du[j], sigma_mu, true);
        s.bx[j] = q.wu + alpha * d.dwu;
        s.bx[n + j] = q.lu + alpha * d.dlu;
        s.bx[2 * n + j] = q.wl + alpha * d.dwl;
        s.bx[3 * n + j] = q.ll + alpha * d.dll;
      }
    }
    if (a.has_p) {
      for (int t = tid; t < 2 * H; t += kBlock) {
        const int i = t & 1;
        const PairState q = pos_state(s, H, t);
        const PairLin l = pair_lin(q, s.p[t], a.pmin[i], a.pmax[i]);
        const PairDir d = pair_dir(q, l, s.dpa[t], s.dp[t], sigma_mu, true);
        s.px[t] = q.wu + alpha * d.dwu;
        s.px[2 * H + t] = q.lu + alpha * d.dlu;
        s.px[4 * H + t] = q.wl + alpha * d.dwl;
        s.px[6 * H + t] = q.ll + alpha * d.dll;
      }
    }
    __syncthreads();  // positions of the box loop read s.u; update it only after every reader
    for (int j = tid; j < n; j += kBlock) s.u[j] += alpha * s.du[j];
    for (int t = tid; t < 2 * H; t += kBlock) s.p[t] += alpha * s.dp[t];
    __syncthreads();
    MPC_PHASE(5);
    // fused pass: each halfspace row is updated (P5) and enters the next iteration's P1 sums
    p1_clear();
    if (lane < K) {
      const double pn0 = s.p[2 * lane], pn1 = s.p[2 * lane + 1];
      ROW_SWEEP_BEGIN
        const HsLin l = hs_lin(q, p0, p1);
        const RowDir d = hs_corrector(q, l, q.h0 * a0 + q.h1 * a1, q.h0 * d0 + q.h1 * d1, sigma_mu);
        HsRow qn = q;
        qn.sv = q.sv + alpha * d.ds;
        qn.wA = q.wA + alpha * d.dwA;
        qn.lA = q.lA + alpha * d.dlA;
        qn.wB = q.wB + alpha * d.dwB;
        qn.lB = q.lB + alpha * d.dlB;
        rows.s[r] = qn.sv;
        rows.wA[r] = qn.wA;
        rows.lA[r] = qn.lA;
        rows.wB[r] = qn.wB;
        rows.lB[r] = qn.lB;
        p1_row(qn, pn0, pn1);
      ROW_SWEEP_END
    }
    MPC_PHASE(5);
  }
  if (it > it_end) it = it_end;
  __syncthreads();
  MPC_PHASE(6);
  if (status != DRCVAR_MPC_STATUS_OPTIMAL && !(early && round == 0) && best_merit <= 1e3 * a.tol) {
    // stalled close to the optimum (or a resumed round short of its tighter tolerance): return
    // the best iterate, its slacks re-optimised below
    status = best_merit <= a.tol ? DRCVAR_MPC_STATUS_OPTIMAL : DRCVAR_MPC_STATUS_OPTIMAL_INACCURATE;
    for (int j = tid; j < n; j += kBlock) s.u[j] = best_u[j];
  }

  // ------------------------------- polish -------------------------------
  // The interior-point iterate identifies the active set; the equality-constrained QP of that
  // set is then solved by the method of multipliers (penalty kPolishRho, kPolishIters passes that
  // reuse the Hessian assembly, the Cholesky and the triangular solves), and rows whose sign
  // conditions fail are moved (primal-dual active-set step), up to kPolishAttempts times.  On
  // success the answer is exact to roundoff; otherwise the interior-point answer stands.
  const bool tried = a.polish && (best_merit <= kPolishMerit || (early && round == 0)) && !(CL && cl.aborted);
  // The active-set guess from the predictor (round 5).  On the iteration that met the tolerance
  // wave 0 has factorised the Newton matrix beside the affine rhs (s.dua), so one solve gives the
  // affine direction at the endpoint, and every complementary pair (w, lambda) is classified by
  // Tapia's indicators: active when d lambda / lambda > d w / w (its w heading to zero faster than
  // its lambda).  The endpoint's own lambda > w misreads rows whose slack is small but positive
  // (lambda_s ~ 0.1 against s ~ 5e-4 at merit 2e-8 on the bench's C5 instance): the first polish
  // attempt then fails and a second one is paid.  Counted on the CPU restatement
  // (scripts/micro/classify_lab.py, 110 problems: C5 DR-CVaR, main.py's three metrics at C5 and
  // H = 20 sizes, 64 batch seeds, few-obstacle problems) against the KKT-certified optimum: lambda > w
  // misclassifies 11 pairs in 8 problems, the indicators none.  Without a usable factorisation (a
  // stalled or resumed-from-best endpoint, a failed pivot) the endpoint rule stands.
  bool predicted = false;
  if (tried && converged) {
    bool done = false;
    if constexpr (NX <= 4 && kPipe) {
      if (s.sc[62] == 0.0) {  // uniform: the backward half ran beside the factorisation
        dpp_backward_tail<NU, kBlock>(s, H, s.dua, s.du);
        dpp_forward<NU, kBlock>(s, H, s.du, s.dua, s.dpa, nullptr);  // affine du, dp
        predicted = done = true;
      }
    }
    if (!done && riccati_factor_finish<NU, NX>(s, H)) {  // uniform
      // affine du (in place), dp; NX > 4: dua holds the whole rhs
      newton_solve<NU, NX, kBlock, HMX>(s, H, n, s.dua, s.dpa, nullptr, NX <= 4 ? s.za : nullptr);
      predicted = true;
    }
    CL_NOTE(predicted ? 1.0 : 0.0);
  }
  if (tried) {
    for (int j = tid; j < n; j += kBlock) best_u[j] = s.u[j];  // the answer if polishing fails
    // classify: flag 0 = halfspace not binding (s = 0), 1 = slack positive (s = h.p + g > 0),
    // 2 = binding with s = 0 (equality, multiplier nu in [0, 50]); rows.s <- nu, rows.wA <- flag
    if (lane < K) {
      const double p0 = s.p[2 * lane], p1 = s.p[2 * lane + 1];
      const double a0 = predicted ? s.dpa[2 * lane] : 0.0, a1 = predicted ? s.dpa[2 * lane + 1] : 0.0;
      for (int o = o_lo + wave; o < o_hi; o += kWaves) {
        const int64_t r = static_cast<int64_t>(o) * kRowStride + lane;
        const HsRow q = rows.load(r);
        bool actA = q.lA > q.wA, actB = q.lB > q.wB;
        if (predicted) {  // Tapia's indicators on the affine direction
          const RowDir d = hs_affine(q, hs_lin(q, p0, p1), q.h0 * a0 + q.h1 * a1);
          actA = d.dlA * q.wA > d.dwA * q.lA;
          actB = d.dlB * q.wB > d.dwB * q.lB;
        }
        const double flag = actA ? (actB ? 2.0 : 1.0) : 0.0;
        SAVED_S[r] = q.sv;
        SAVED_W[r] = q.wA;
        rows.s[r] = flag == 2.0 ? q.lA : 0.0;
        rows.wA[r] = flag;
      }
    }
    // bounds: bx / px <- (flag_up, nu_up, flag_lo, nu_lo)
    if (a.has_u) {
      for (int j = tid; j < n; j += kBlock) {
        const PairState q = box_state(s, n, j);
        bool up = q.lu > q.wu, lo = q.ll > q.wl;
        if (predicted) {
          const int ai = j % NU;
          const PairDir d = pair_dir(q, pair_lin(q, s.u[j], a.umin[ai], a.umax[ai]), 0.0, s.dua[j], 0.0, false);
          up = d.dlu * q.wu > d.dwu * q.lu;
          lo = d.dll * q.wl > d.dwl * q.ll;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) SAVED_B[k * n + j] = s.bx[k * n + j];
        s.bx[j] = up;
        s.bx[n + j] = up ? q.lu : 0.0;
        s.bx[2 * n + j] = lo;
        s.bx[3 * n + j] = lo ? q.ll : 0.0;
      }
    }
    if (a.has_p) {
      for (int t = tid; t < 2 * H; t += kBlock) {
        const PairState q = pos_state(s, H, t);
        bool up = q.lu > q.wu, lo = q.ll > q.wl;
        if (predicted) {
          const int i = t & 1;
          const PairDir d = pair_dir(q, pair_lin(q, s.p[t], a.pmin[i], a.pmax[i]), 0.0, s.dpa[t], 0.0, false);
          up = d.dlu * q.wu > d.dwu * q.lu;
          lo = d.dll * q.wl > d.dwl * q.ll;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) SAVED_B[4 * n + k * 2 * H + t] = s.px[k * 2 * H + t];
        s.px[t] = up;
        s.px[2 * H + t] = up ? q.lu : 0.0;
        s.px[4 * H + t] = lo;
        s.px[6 * H + t] = lo ? q.ll : 0.0;
      }
    }
    __syncthreads();
    const double tolf = 1e-9 * scale_d;
    for (int attempt = 0; attempt < kPolishAttempts && !polished && !(CL && cl.aborted); ++attempt) {
      // test hook; a loop bound computed from it instead (attempts = hook ? 0 : kPolishAttempts)
      // broke the 4-input kernels' polish (8 % polished) — a codegen effect, not a semantic one
      if (round == 0 && a.force_resume) break;
      if (round == 0 && early && attempt >= kEarlyPolishAttempts) break;  // (a break: see above)
      ++polish_attempts;
      // Hessian of the active-set problem: 100 h h' for positive slacks, rho h h' for equalities
      {
        double acc[3] = {0, 0, 0};
        if (lane < K) {
          for (int o = o_lo + wave; o < o_hi; o += kWaves) {
            const int64_t r = static_cast<int64_t>(o) * kRowStride + lane;
            const double flag = rows.wA[r];
            const double wgt = flag == 1.0 ? kSlackHess : (flag == 2.0 ? kPolishRho : 0.0);
            const double h0 = rows.h0[r], h1 = rows.h1[r];
            acc[0] += wgt * h0 * h0;
            acc[1] += wgt * h0 * h1;
            acc[2] += wgt * h1 * h1;
          }
        }
        if constexpr (CL) {
          MPC_PHASE(10);
          cluster_combine<kWaves, 3, 0>(cl, s, acc, kOpSum, nullptr, nullptr, kSitePolishHess);
          MPC_PHASE(16);  // cluster exchange
          if (cl.aborted) break;
        } else {
#pragma unroll
          for (int q = 0; q < 3; ++q) s.red[(wave * kPerStepQ + q) * 64 + lane] = acc[q];
          __syncthreads();
        }
        if (wave == 0 && lane < H) {
          double t0 = lane < K ? (CL ? s.red[lane] : step_total<kWaves>(s.red, 0, lane)) : 0.0;
          const double t1 = lane < K ? (CL ? s.red[64 + lane] : step_total<kWaves>(s.red, 1, lane)) : 0.0;
          double t2 = lane < K ? (CL ? s.red[128 + lane] : step_total<kWaves>(s.red, 2, lane)) : 0.0;
          if (a.has_p) {
            t0 += kPolishRho * (s.px[2 * lane] + s.px[4 * H + 2 * lane]);
            t2 += kPolishRho * (s.px[2 * lane + 1] + s.px[4 * H + 2 * lane + 1]);
          }
          s.S[lane] = t0;
          s.S[H + lane] = t1;
          s.S[2 * H + lane] = t2;
        }
        for (int j = tid; j < n; j += kBlock)
          s.DU[j] = a.has_u ? kPolishRho * (s.bx[j] + s.bx[2 * n + j]) : 0.0;
        __syncthreads();
      }
      MPC_PHASE(10);
      if (!riccati_factor<NU, NX>(s, H) && !riccati_factor<NU, NX, true>(s, H)) break;
      CL_NOTE(s.Ri[0]);
      MPC_PHASE(11);
      // The rhs of a pass depends on the multipliers only (the bb terms are at the free response
      // c), so the multiplier update of pass t also sums pass t + 1's rhs rows, and one exchange
      // carries both its residual maximum and those sums (`carried`): one cluster exchange per
      // pass instead of two, the same sums in the same order.
      bool carried = false;
      for (int pass = 0; pass < kPolishIters; ++pass) {
        // rhs = -f - sum_pen (50 + 100 b) a - E'(nu - rho e), per step through Gp'
        double acc[2] = {0, 0};
        if (!carried && lane < K) {
          const double c0 = s.c[2 * lane], c1 = s.c[2 * lane + 1];
          for (int o = o_lo + wave; o < o_hi; o += kWaves) {
            const int64_t r = static_cast<int64_t>(o) * kRowStride + lane;
            const double flag = rows.wA[r];
            const double h0 = rows.h0[r], h1 = rows.h1[r];
            const double bb = h0 * c0 + h1 * c1 + rows.g[r];
            const double coef = flag == 1.0 ? kSlackLin + kSlackHess * bb
                                            : (flag == 2.0 ? rows.s[r] + kPolishRho * bb : 0.0);
            acc[0] += coef * h0;
            acc[1] += coef * h1;
          }
        }
        if (!carried) {
          if constexpr (CL) {
            MPC_PHASE(12);
            cluster_combine<kWaves, 2, 0>(cl, s, acc, kOpSum, nullptr, nullptr, kSitePolishRhs);
            MPC_PHASE(16);  // cluster exchange
            if (cl.aborted) break;
          } else {
            s.red[(wave * kPerStepQ) * 64 + lane] = acc[0];
            s.red[(wave * kPerStepQ + 1) * 64 + lane] = acc[1];
            __syncthreads();
          }
        }
        if (wave == 0 && lane < H) {
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int t = 2 * lane + i;
            double z = lane < K ? (CL ? s.red[i * 64 + lane] : step_total<kWaves>(s.red, i, lane)) : 0.0;
            if (a.has_p) {
              if (s.px[t] != 0.0) z += s.px[2 * H + t] - kPolishRho * (a.pmax[i] - s.c[t]);
              if (s.px[4 * H + t] != 0.0) z -= s.px[6 * H + t] - kPolishRho * (s.c[t] - a.pmin[i]);
            }
            s.za[t] = z;
          }
        }
        // the input part of the rhs (-f and the bound terms; the per-step za is the solve's state
        // source)
        for (int j = tid; j < n; j += kBlock) {
          double r = -s.f[j];
          if (a.has_u) {
            const int ai = j % NU;
            if (s.bx[j] != 0.0) r -= s.bx[n + j] - kPolishRho * a.umax[ai];
            if (s.bx[2 * n + j] != 0.0) r += s.bx[3 * n + j] + kPolishRho * a.umin[ai];
          }
          s.du[j] = r;
        }
        __syncthreads();
        MPC_PHASE(12);
        newton_solve<NU, NX, kBlock, HMX>(s, H, n, s.du, s.p, s.c, s.za);  // u and its positions
        for (int j = tid; j < n; j += kBlock) s.u[j] = s.du[j];
        __syncthreads();
        MPC_PHASE(13);
        // multiplier updates nu += rho * (E u - e); eres = |E u - e|_inf; and the next pass's rhs
        // rows (acc, with the updated multipliers)
        double eres = 0.0;
        acc[0] = acc[1] = 0.0;
        if (lane < K) {
          const double p0 = s.p[2 * lane], p1 = s.p[2 * lane + 1];
          const double c0 = s.c[2 * lane], c1 = s.c[2 * lane + 1];
          for (int o = o_lo + wave; o < o_hi; o += kWaves) {
            const int64_t r = static_cast<int64_t>(o) * kRowStride + lane;
            const double flag = rows.wA[r];
            const double h0 = rows.h0[r], h1 = rows.h1[r], g = rows.g[r];
            double nu = rows.s[r];
            if (flag == 2.0) {
              const double e = h0 * p0 + h1 * p1 + g;
              nu += kPolishRho * e;
              rows.s[r] = nu;
              eres = fmax(eres, fabs(e));
            }
            const double bb = h0 * c0 + h1 * c1 + g;
            const double coef = flag == 1.0 ? kSlackLin + kSlackHess * bb
                                            : (flag == 2.0 ? nu + kPolishRho * bb : 0.0);
            acc[0] += coef * h0;
            acc[1] += coef * h1;
          }
        }
        if (a.has_u) {
          for (int j = tid; j < n; j += kBlock) {
            const int ai = j % NU;
            if (s.bx[j] != 0.0) {
              s.bx[n + j] += kPolishRho * (s.u[j] - a.umax[ai]);
              eres = fmax(eres, fabs(s.u[j] - a.umax[ai]));
            }
            if (s.bx[2 * n + j] != 0.0) {
              s.bx[3 * n + j] += kPolishRho * (a.umin[ai] - s.u[j]);
              eres = fmax(eres, fabs(a.umin[ai] - s.u[j]));
            }
          }
        }
        if (a.has_p) {
          for (int t = tid; t < 2 * H; t += kBlock) {
            const int i = t & 1;
            if (s.px[t] != 0.0) {
              s.px[2 * H + t] += kPolishRho * (s.p[t] - a.pmax[i]);
              eres = fmax(eres, fabs(s.p[t] - a.pmax[i]));
            }
            if (s.px[4 * H + t] != 0.0) {
              s.px[6 * H + t] += kPolishRho * (a.pmin[i] - s.p[t]);
              eres = fmax(eres, fabs(a.pmin[i] - s.p[t]));
            }
          }
        }
        // The multipliers have converged once the equalities hold to roundoff (a further pass
        // moves nu by rho * eres and u by ~eres): stop instead of running all kPolishIters.
        if constexpr (CL) {  // every workgroup's equality rows (the bound terms: replicated)
          const int ops[1] = {kOpMax};
          MPC_PHASE(12);
          cluster_combine<kWaves, 2, 1>(cl, s, acc, kOpSum, &eres, ops, kSitePolishEq);
          MPC_PHASE(16);  // cluster exchange
          if (cl.aborted) break;
        } else {
          s.red[(wave * kPerStepQ) * 64 + lane] = acc[0];  // published by the barriers below
          s.red[(wave * kPerStepQ + 1) * 64 + lane] = acc[1];
        }
        double unused_a = 0.0, unused_b = 0.0;
        block_sum_max_max<kWaves>(unused_a, eres, unused_b, s.sc);  // uniform; also the barrier
        CL_NOTE(eres);
        if (eres <= kPolishEqTol * scale_d) break;
        carried = true;
      }
      // sign conditions; violators move (primal-dual active-set step).  Rows that must become
      // equalities (a dropped row violated, a penalised row with s < 0) and equalities with a
      // negative multiplier move one per step and attempt, the most violated: moving every
      // violator at once can leave a step with more binding rows than it has freedom, after which
      // the multiplier passes diverge and the corrections thrash (degenerate problems).  Every
      // violator still counts as unresolved.
      double bad = 0.0;
      {
        double vmax = 0.0, dmax = 0.0;
        if (lane < K) {
          const double p0 = s.p[2 * lane], p1 = s.p[2 * lane + 1];
          for (int o = o_lo + wave; o < o_hi; o += kWaves) {
            const int64_t r = static_cast<int64_t>(o) * kRowStride + lane;
            const double flag = rows.wA[r];
            const double hp = rows.h0[r] * p0 + rows.h1[r] * p1 + rows.g[r];
            vmax = fmax(vmax, flag == 0.0 ? hp : (flag == 1.0 ? -hp : 0.0));
            dmax = fmax(dmax, flag == 2.0 ? -rows.s[r] : 0.0);
          }
        }
        if constexpr (CL) {  // per-step maxima over the cluster's rows
          const double vm[2] = {vmax, dmax};
          MPC_PHASE(7);
          cluster_combine<kWaves, 2, 0>(cl, s, vm, kOpMax, nullptr, nullptr, kSitePolishSign);
          MPC_PHASE(16);  // cluster exchange
        } else {
          s.red[(wave * kPerStepQ) * 64 + lane] = vmax;
          s.red[(wave * kPerStepQ + 1) * 64 + lane] = dmax;
          __syncthreads();
        }
      }
      if (lane < K) {
        double step_vmax = 0.0, step_dmax = 0.0;
        if constexpr (CL) {
          step_vmax = s.red[lane];
          step_dmax = s.red[64 + lane];
        } else {
          for (int w = 0; w < kWaves; ++w) {
            step_vmax = fmax(step_vmax, s.red[(w * kPerStepQ) * 64 + lane]);
            step_dmax = fmax(step_dmax, s.red[(w * kPerStepQ + 1) * 64 + lane]);
          }
        }
        const double p0 = s.p[2 * lane], p1 = s.p[2 * lane + 1];
        for (int o = o_lo + wave; o < o_hi; o += kWaves) {
          const int64_t r = static_cast<int64_t>(o) * kRowStride + lane;
          const double flag = rows.wA[r];
          const double hp = rows.h0[r] * p0 + rows.h1[r] * p1 + rows.g[r];
          double nf = flag, nv = rows.s[r];
          if (flag == 2.0) {
            if (nv > kSlackLin + kPolishDualTol) nf = 1.0;        // the slack is positive after all
            else if (nv < -kPolishDualTol) {                      // not binding (one per step)
              bad += 1.0;
              if (-nv >= step_dmax) nf = 0.0;
            }
            nv = nf == 2.0 ? fmin(fmax(nv, 0.0), kSlackLin) : 0.0;
            bad += nf == 1.0;
          } else {
            const double v = flag == 1.0 ? -hp : hp;              // s < 0 / dropped row violated
            if (v > tolf) {
              bad += 1.0;
              if (v >= step_vmax) {
                nf = 2.0;
                nv = 0.0;
              }
            }
          }
          rows.wA[r] = nf;
          rows.s[r] = nv;
        }
      }
      if constexpr (CL) {  // unresolved rows of the whole cluster, counted once (thread 0)
        const int ops[1] = {kOpSum};
        MPC_PHASE(7);
        cluster_combine<kWaves, 0, 1>(cl, s, nullptr, kOpSum, &bad, ops, kSitePolishBad);
        MPC_PHASE(16);  // cluster exchange
        bad = tid == 0 ? bad : 0.0;
      }
      if (a.has_u) {
        for (int j = tid; j < n; j += kBlock) {
          const int ai = j % NU;
          const double uj = s.u[j];
          for (int side = 0; side < 2; ++side) {
            double* fl = s.bx + 2 * side * n + j;
            double* nv = fl + n;
            const double viol = side == 0 ? uj - a.umax[ai] : a.umin[ai] - uj;
            if (*fl != 0.0 && *nv < -kPolishDualTol) { *fl = 0.0; *nv = 0.0; bad += 1.0; }
            else if (*fl == 0.0 && viol > tolf) { *fl = 1.0; *nv = 0.0; bad += 1.0; }
            else if (*fl != 0.0) *nv = fmax(*nv, 0.0);
          }
        }
      }
      if (a.has_p) {
        for (int t = tid; t < 2 * H; t += kBlock) {
          const int i = t & 1;
          const double pv = s.p[t];
          for (int side = 0; side < 2; ++side) {
            double* fl = s.px + 4 * side * H + t;
            double* nv = fl + 2 * H;
            const double viol = side == 0 ? pv - a.pmax[i] : a.pmin[i] - pv;
            if (*fl != 0.0 && *nv < -kPolishDualTol) { *fl = 0.0; *nv = 0.0; bad += 1.0; }
            else if (*fl == 0.0 && viol > tolf) { *fl = 1.0; *nv = 0.0; bad += 1.0; }
            else if (*fl != 0.0) *nv = fmax(*nv, 0.0);
          }
        }
      }
      bad = block_sum<kWaves>(bad, s.sc);
      CL_NOTE(bad);
      if (bad == 0.0) polished = true;
    }
    if (polished) {
      status = DRCVAR_MPC_STATUS_OPTIMAL;
    } else {
      for (int j = tid; j < n; j += kBlock) s.u[j] = best_u[j];
    }
    __syncthreads();
  }
  bool resume = round == 0 && tried && !polished && (status == DRCVAR_MPC_STATUS_OPTIMAL || early) &&
                it < a.max_iter;
  if constexpr (CL) resume = resume && !cl.aborted;
  if (!resume) return false;
  // restore what the polish overwrote (u is back already): the rows' s / w_hs and the bound states
  if (lane < K) {
    for (int o = o_lo + wave; o < o_hi; o += kWaves) {
      const int64_t r = static_cast<int64_t>(o) * kRowStride + lane;
      rows.s[r] = SAVED_S[r];
      rows.wA[r] = SAVED_W[r];
    }
  }
  for (int j = tid; j < n; j += kBlock)
#pragma unroll
    for (int k = 0; k < 4; ++k) s.bx[k * n + j] = SAVED_B[k * n + j];
  for (int t = tid; t < 2 * H; t += kBlock)
#pragma unroll
    for (int k = 0; k < 4; ++k) s.px[k * 2 * H + t] = SAVED_B[4 * n + k * 2 * H + t];
  __syncthreads();
  status = DRCVAR_MPC_STATUS_MAX_ITER;
  // after a failed early polish the method simply goes on to its tolerance; after a failed polish
  // at the tolerance, a few more iterations towards a tighter one
  tol_r = early ? a.tol : a.tol * kResumeTol;
  it_end = early ? a.max_iter : (it + kResumeIters < a.max_iter ? it + kResumeIters : a.max_iter);
  return true;
  };  // ipm_round
  if (ipm_round(0)) ipm_round(1);

  MPC_PHASE(7);
  // ------------------------------- output -------------------------------
  // A cluster that disagreed or whose wait gave up rolls the fallback inputs out, like any failed
  // solve (core/mpc_filter.py:166-178), with a status of its own.
  const int abort_status = CL && cl.diverged ? DRCVAR_MPC_STATUS_CLUSTER_DIVERGED : DRCVAR_MPC_STATUS_CLUSTER_TIMEOUT;
  if constexpr (CL) {
    if (cl.aborted) status = abort_status;
  }
  bool optimal = status == DRCVAR_MPC_STATUS_OPTIMAL || status == DRCVAR_MPC_STATUS_OPTIMAL_INACCURATE;
  // the returned inputs (the fallback's unless optimal), their positions and states
  auto rollout = [&]() __attribute__((always_inline)) {
    if (!optimal) {
      const double* uf = a.uf + b * a.uf_sp;
      for (int j = tid; j < n; j += kBlock) s.u[j] = uf[(j / NU) * a.uf_st + j % NU];
    }
    for (int q = tid; q < nx; q += kBlock) s.xs[q] = x0[q];
    __syncthreads();
    positions<NU, kBlock>(s, s.u, s.p, s.c, H);  // positions of the returned inputs (slacks below)
    // x_{t+1} = A x_t + B u_t (core/mpc_filter.py:85-86, :216-217): wave 0, lane q < nx holds x_q,
    // the state moving between lanes by readlane — no barrier per step
    if (tid < 64) {
      const int li = lane < nx ? lane : 0;
      double Arow[NX], Brow[NU];
#pragma unroll
      for (int m = 0; m < NX; ++m) Arow[m] = s.Am[li * kMx + m];  // zero-padded beyond nx
#pragma unroll
      for (int c = 0; c < NU; ++c) Brow[c] = s.Bm[li * NU + c];
      double xv = lane < nx ? x0[lane] : 0.0;
      for (int t = 0; t < H; ++t) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) acc += Arow[m] * readlane_f64(xv, m);
#pragma unroll
        for (int c = 0; c < NU; ++c) acc += Brow[c] * s.u[t * NU + c];
        xv = lane < nx ? acc : 0.0;
        if (lane < nx) s.xs[(t + 1) * nx + lane] = acc;
      }
    }
    __syncthreads();
  };
  rollout();
  // objective (core/mpc_filter.py:64-76,142-144) and the largest slack
  double obj = 0.0, smax = 0.0, obj_rows = 0.0;
  double& obj_hs = CL ? obj_rows : obj;  // the rows' terms (clustered: summed over the cluster)
  if (optimal) {
    const double* Q = a.blob + a.off.Q;
    const double* R = a.blob + a.off.R;
    for (int t = tid; t < H; t += kBlock) {
      double e[DRCVAR_MPC_MAX_STATES];
      for (int q = 0; q < nx; ++q) e[q] = s.xs[(t + 1) * nx + q] - xr[(t + 1) * a.xr_st + q];
      for (int q = 0; q < nx; ++q) {
        double row = 0.0;
        for (int r = 0; r < nx; ++r) row += Q[q * nx + r] * e[r];
        obj += e[q] * row;
      }
      for (int q = 0; q < NU; ++q) {
        double row = 0.0;
        for (int r = 0; r < NU; ++r) row += R[q * NU + r] * s.u[t * NU + r];
        obj += s.u[t * NU + q] * row;
      }
    }
    if (lane < K) {
      // the optimal slack of a halfspace for the returned inputs is max(0, h.p + g)
      const double p0 = s.p[2 * lane], p1 = s.p[2 * lane + 1];
      for (int o = o_lo + wave; o < o_hi; o += kWaves) {
        const int64_t r = static_cast<int64_t>(o) * kRowStride + lane;
        const double sv = fmax(0.0, rows.h0[r] * p0 + rows.h1[r] * p1 + rows.g[r]);
        rows.s[r] = sv;
        obj_hs += kSlackLin * sv + 0.5 * kSlackHess * sv * sv;
        smax = fmax(smax, sv);
      }
    }
  }
  if constexpr (CL) {
    if (a.stall_group == cid + 1) return;  // test hook: never arrives at the final exchange
    double sv[2] = {obj_rows, smax};
    const int ops[2] = {kOpSum, kOpMax};
    MPC_PHASE(8);
    cluster_combine<kWaves, 0, 2>(cl, s, nullptr, kOpSum, sv, ops, kSiteFinal);
    MPC_PHASE(16);  // cluster exchange
    obj += tid == 0 ? sv[0] : 0.0;
    smax = sv[1];
    if (cl.aborted && optimal) {  // this exchange gave up: the fallback after all
      status = cl.diverged ? DRCVAR_MPC_STATUS_CLUSTER_DIVERGED : DRCVAR_MPC_STATUS_CLUSTER_TIMEOUT;
      optimal = false;
      rollout();
    }
#if defined(DRCVAR_MPC_STAMPS) && defined(DRCVAR_STAMP_GROUP)  // the phase stamps of another group
    if (cid == DRCVAR_STAMP_GROUP && tid == 0 && b < kStampProblems) {
      stamp_acc[9] = it;
      for (int k = 0; k < kStampSlots; ++k) g_mpc_stamps[b * kStampSlots + k] = stamp_acc[k];
    }
#endif
    if (cid != 0) return;  // workgroup 0 writes the problem's outputs (every one holds them)
  }
  double unused = 0.0;
  block_sum_max_max<kWaves>(obj, smax, unused, s.sc);
  double* xo = a.x_out + b * (H + 1) * nx;
  for (int q = tid; q < (H + 1) * nx; q += kBlock) xo[q] = s.xs[q];
  double* uo = a.u_out + b * n;
  for (int j = tid; j < n; j += kBlock) uo[j] = s.u[j];
  if (tid == 0) {
    double* info = a.info + b * DRCVAR_MPC_INFO_WIDTH;
    info[DRCVAR_MPC_INFO_STATUS] = status;
    info[DRCVAR_MPC_INFO_ITERATIONS] = it;
    info[DRCVAR_MPC_INFO_OBJECTIVE] = optimal ? obj : NAN;
    info[DRCVAR_MPC_INFO_MU] = best_merit;
    info[DRCVAR_MPC_INFO_PRIMAL_RES] = rp;
    info[DRCVAR_MPC_INFO_DUAL_RES] = rd;
    info[DRCVAR_MPC_INFO_MAX_SLACK] = optimal ? smax : NAN;
    info[DRCVAR_MPC_INFO_USED_FALLBACK] = optimal ? 0.0 : 1.0;
    info[DRCVAR_MPC_INFO_POLISHED] = polished ? 1.0 : 0.0;
    info[DRCVAR_MPC_INFO_POLISH_ATTEMPTS] = polish_attempts;
  }
  MPC_PHASE(8);
#if defined(DRCVAR_MPC_STAMPS) && !defined(DRCVAR_STAMP_GROUP)
  if (tid == 0 && b < kStampProblems) {
    stamp_acc[9] = it;
    for (int k = 0; k < kStampSlots; ++k) g_mpc_stamps[b * kStampSlots + k] = stamp_acc[k];
  }
#endif
}

// zeroes the per-problem arrival counters of a clustered launch (in front of it, same stream)
__global__ void zero_counters_kernel(double* ws, int n_problems) {
  for (int b = threadIdx.x; b < n_problems; b += blockDim.x)
    __hip_atomic_store((gu64*)(ws + b * kCtrlDoubles), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NU, int NX, int BLK, int HMX, bool CL, bool RL>
int launch_form(const MpcArgs& args, int64_t n_problems, size_t lds_req, size_t attr_bytes, hipStream_t stream) {
  // per device and kernel form, set once; the flags are atomics because any host thread may
  // launch (a racing second caller sets the same value again, which is harmless)
  static std::atomic<bool> attr_set[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return DRCVAR_ERR_LAUNCH;
  if (!attr_set[dev].load(std::memory_order_acquire)) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&mpc_ipm_kernel<NU, NX, BLK, HMX, CL, RL>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(attr_bytes)) != hipSuccess)
      return DRCVAR_ERR_LAUNCH;
    attr_set[dev].store(true, std::memory_order_release);
  }
  // the arrival counters, zeroed in front of every launch by a one-wave kernel of agent-scope
  // (write-through) stores: a hipMemsetAsync node replayed from a hipGraph left the counters
  // unreliable from the second replay on (replays 2..5 timed out or read garbage sums; with this
  // kernel every replay reproduced the eager launch, scripts/micro/cluster_graph_diag.py)
  if constexpr (CL)
    hipLaunchKernelGGL(zero_counters_kernel, dim3(1), dim3(64), 0, stream, args.ws, static_cast<int>(n_problems));
  hipLaunchKernelGGL((mpc_ipm_kernel<NU, NX, BLK, HMX, CL, RL>),
                     dim3(static_cast<unsigned>(n_problems * (CL ? args.cl_size : 1))), dim3(BLK),
                     lds_req, stream, args);
  return DRCVAR_OK;
}

template <int NU, int NX, int BLK, int HMX = DRCVAR_MPC_MAX_HORIZON, bool CL = false>
int launch(const MpcArgs& args, int64_t n_problems, hipStream_t stream) {
  // the clustered form asks for more LDS than two workgroups can share: one workgroup per CU
  constexpr size_t plan_bytes = sizeof(double) * (LdsPlan<BLK / 64, NU, NX, HMX>::total + (CL ? kClusterScratch : 0));
  constexpr size_t lds_bytes = CL && plan_bytes < 96 * 1024 ? 96 * 1024 : plan_bytes;
  if constexpr (CL && NX <= 4) {
    // the largest obstacle slice's rows in LDS beside the plan, when they fit (the C5 hand-off:
    // 16 obstacles, 80 KB beside 78 KB): the RL form
    constexpr size_t kLdsMax = 160 * 1024;  // gfx950: LDS per workgroup
    const int64_t slice = (static_cast<int64_t>(args.O) + args.cl_size - 1) / args.cl_size;
    const size_t rows_bytes = sizeof(double) * static_cast<size_t>(slice) * kRowStride;
    if (plan_bytes + rows_bytes <= kLdsMax)
      return launch_form<NU, NX, BLK, HMX, CL, true>(args, n_problems, plan_bytes + rows_bytes, kLdsMax, stream);
  }
  return launch_form<NU, NX, BLK, HMX, CL, false>(args, n_problems, lds_bytes, lds_bytes, stream);
}

template <int NU>
int launch_nu(const MpcArgs& args, int64_t n_problems, hipStream_t stream) {
  // state dimension padded to 4 or 8 (the Riccati sweeps are unrolled over it); a launch of a
  // few problems cannot fill the chip, so each problem gets 512 threads.  Many problems with a
  // short horizon take the 128-thread form: its LDS plan (horizon <= kShortHorizon) fits four
  // workgroups per CU (three with four inputs), twice the problems in flight of the 256-thread
  // form.
  const bool few = n_problems <= kFewProblems;
  const bool short_h = args.H <= kShortHorizon;
  if (args.cl_size > 1)
    return args.nx <= 4 ? launch<NU, 4, kClusterBlock, DRCVAR_MPC_MAX_HORIZON, true>(args, n_problems, stream)
                        : launch<NU, 8, kClusterBlock, DRCVAR_MPC_MAX_HORIZON, true>(args, n_problems, stream);
  if (args.nx <= 4)
    return few ? launch<NU, 4, 512>(args, n_problems, stream)
               : short_h ? launch<NU, 4, 128, kShortHorizon>(args, n_problems, stream)
                         : launch<NU, 4, 256>(args, n_problems, stream);
  return few ? launch<NU, 8, 512>(args, n_problems, stream)
             : short_h ? launch<NU, 8, 128, kShortHorizon>(args, n_problems, stream)
                       : launch<NU, 8, 256>(args, n_problems, stream);
}

#endif  // DRCVAR_MPC_ANY_DEVICE_PART

#if DRCVAR_MPC_HOST_PART
// ------------------------------- host side -------------------------------

bool all_finite(const double* p, int64_t n) {
  for (int64_t i = 0; i < n; ++i)
    if (!std::isfinite(p[i])) return false;
  return true;
}

// Clustered launches (a few large problems): workgroups per problem.  Two obstacles per wave of
// the 512-thread form (16 per workgroup), at most kClusterMax workgroups per problem
// and never more workgroups in all than half the CUs (the workspace is sized for all of them).
// Problems with fewer than kClusterMinObstacles
// obstacles (≤ 8 rows per thread on one workgroup) stay on one workgroup: the exchanges
// (~3 per interior-point iteration) would cost more than the sweeps they split (constants
// kCluster* with the exchange layout above).
// the most workgroups a problem of this batch may use (1: not eligible for the clustered form)
int cluster_limit(int64_t n_problems, int64_t n_obstacles, int64_t cus) {
  if (n_problems < 1 || n_problems > kClusterMaxProblems || n_obstacles < kClusterMinObstacles) return 1;
  int64_t c = n_obstacles < kClusterMax ? n_obstacles : kClusterMax;
  c = c < cus / n_problems ? c : cus / n_problems;
  return c < 2 ? 1 : static_cast<int>(c);
}

// the workgroups a launch uses: kClusterObstaclesPerGroup obstacles each, or `requested` (> 0:
// drcvar_mpc_options.cluster_size, A/B runs and tests; 1 = the one-workgroup form), within the
// limit for half the device's CUs: a clustered launch's workgroups must all be resident at once,
// and half the chip leaves room for whatever else runs beside it (another stream, another process)
int cluster_size(int64_t n_problems, int64_t n_obstacles, int64_t cus, int requested) {
  const int lim = cluster_limit(n_problems, n_obstacles, cus / 2);
  if (lim == 1) return 1;
  int64_t c = (n_obstacles + kClusterObstaclesPerGroup - 1) / kClusterObstaclesPerGroup;
  if (requested > 0) c = requested;
  c = c < lim ? c : lim;
  return c < 2 ? 1 : static_cast<int>(c);
}

#endif  // DRCVAR_MPC_HOST_PART
}  // namespace

namespace drcvar_mpc_detail {
#if DRCVAR_MPC_DEVICE_PART(1)
int launch_nu1(const MpcArgs& args, int64_t n_problems, hipStream_t stream) { return launch_nu<1>(args, n_problems, stream); }
#endif
#if DRCVAR_MPC_DEVICE_PART(2)
int launch_nu2(const MpcArgs& args, int64_t n_problems, hipStream_t stream) { return launch_nu<2>(args, n_problems, stream); }
#endif
#if DRCVAR_MPC_DEVICE_PART(3)
int launch_nu3(const MpcArgs& args, int64_t n_problems, hipStream_t stream) { return launch_nu<3>(args, n_problems, stream); }
#endif
#if DRCVAR_MPC_DEVICE_PART(4)
int launch_nu4(const MpcArgs& args, int64_t n_problems, hipStream_t stream) { return launch_nu<4>(args, n_problems, stream); }
#endif
#if DRCVAR_MPC_HOST_PART
int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  static std::atomic<int> cached[64] = {};  // per device (any host thread may ask)
  if (dev >= 0 && dev < 64) {
    const int c = cached[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
  }
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (dev >= 0 && dev < 64) cached[dev].store(cus, std::memory_order_relaxed);
  return cus;
}

#endif
}  // namespace drcvar_mpc_detail

#if defined(DRCVAR_MPC_STAMPS) && DRCVAR_MPC_DEVICE_PART(2)
// diagnostic build only (not part of the ABI header): the stamps of the 2-input kernels (the
// double integrator of every benchmark), exported by the part that holds them
extern "C" {
int drcvar_diag_cluster_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_cl_stamps), sizeof(g_cl_stamps), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 8 : -1;
}
int drcvar_diag_mpc_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mpc_stamps), sizeof(g_mpc_stamps), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? kStampProblems : -1;
}
int drcvar_diag_cluster_arrivals(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_cl_arrive), sizeof(g_cl_arrive), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 96 : -1;
}
int drcvar_diag_wave_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wave_stamps), sizeof(g_wave_stamps), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 16 : -1;
}
}
#endif

#if DRCVAR_MPC_HOST_PART
extern "C" {


int drcvar_mpc_model_init(const double* A, const double* B, const double* C, const double* Q,
                          const double* R, int32_t nx, int32_t nu, int32_t ny, int32_t H,
                          const double* u_min, const double* u_max, const double* p_min,
                          const double* p_max, drcvar_mpc_model* model, double* blob) {
  if (!A || !B || !C || !Q || !R || !model) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (nx < 1 || nu < 1 || H < 1 || ny != 2) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (nx > DRCVAR_MPC_MAX_STATES || nu > DRCVAR_MPC_MAX_INPUTS || H > DRCVAR_MPC_MAX_HORIZON ||
      nu * H > DRCVAR_MPC_MAX_DECISION)
    return DRCVAR_ERR_UNSUPPORTED;
  if ((u_min == nullptr) != (u_max == nullptr) || (p_min == nullptr) != (p_max == nullptr))
    return DRCVAR_ERR_INVALID_ARGUMENT;
  if (!all_finite(A, nx * nx) || !all_finite(B, nx * nu) || !all_finite(C, ny * nx) ||
      !all_finite(Q, nx * nx) || !all_finite(R, nu * nu))
    return DRCVAR_ERR_INVALID_ARGUMENT;
  drcvar_mpc_model m{};
  m.n_states = nx;
  m.n_inputs = nu;
  m.n_outputs = ny;
  m.horizon = H;
  m.has_input_bounds = u_min != nullptr;
  m.has_position_bounds = p_min != nullptr;
  for (int i = 0; i < nu && u_min; ++i) {
    m.u_min[i] = u_min[i];
    m.u_max[i] = u_max[i];
    if (!std::isfinite(u_min[i]) || !std::isfinite(u_max[i])) return DRCVAR_ERR_INVALID_ARGUMENT;
  }
  for (int i = 0; i < 2 && p_min; ++i) {
    m.p_min[i] = p_min[i];
    m.p_max[i] = p_max[i];
    if (!std::isfinite(p_min[i]) || !std::isfinite(p_max[i])) return DRCVAR_ERR_INVALID_ARGUMENT;
  }
  const BlobLayout L = blob_layout(nx, nu, H);
  m.blob_doubles = L.total;
  *model = m;
  if (!blob) return DRCVAR_OK;

  const int n = nu * H;
  // A^i for i = 0..H, row-major nx x nx
  std::vector<double> Apow(static_cast<size_t>(H + 1) * nx * nx, 0.0);
  for (int i = 0; i < nx; ++i) Apow[i * nx + i] = 1.0;
  for (int p = 1; p <= H; ++p) {
    const double* prev = &Apow[static_cast<size_t>(p - 1) * nx * nx];
    double* cur = &Apow[static_cast<size_t>(p) * nx * nx];
    for (int i = 0; i < nx; ++i)
      for (int j = 0; j < nx; ++j) {
        double acc = 0.0;
        for (int k = 0; k < nx; ++k) acc += A[i * nx + k] * prev[k * nx + j];
        cur[i * nx + j] = acc;
      }
  }
  // AB[i] = A^i B  (nx x nu)
  std::vector<double> AB(static_cast<size_t>(H) * nx * nu, 0.0);
  for (int p = 0; p < H; ++p)
    for (int i = 0; i < nx; ++i)
      for (int j = 0; j < nu; ++j) {
        double acc = 0.0;
        for (int k = 0; k < nx; ++k) acc += Apow[(static_cast<size_t>(p) * nx + i) * nx + k] * B[k * nu + j];
        AB[(static_cast<size_t>(p) * nx + i) * nu + j] = acc;
      }
  // Gx: x_{k+1} = A^{k+1} x0 + sum_{j<=k} A^{k-j} B u_j  -> Gx [(H*nx) x n], Phi [(H*nx) x nx]
  std::vector<double> Gx(static_cast<size_t>(H) * nx * n, 0.0);
  for (int k = 0; k < H; ++k)
    for (int j = 0; j <= k; ++j)
      for (int i = 0; i < nx; ++i)
        for (int c = 0; c < nu; ++c)
          Gx[(static_cast<size_t>(k) * nx + i) * n + j * nu + c] = AB[(static_cast<size_t>(k - j) * nx + i) * nu + c];
  // QG = blockdiag(Q) Gx
  std::vector<double> QG(Gx.size(), 0.0);
  for (int k = 0; k < H; ++k)
    for (int i = 0; i < nx; ++i)
      for (int c = 0; c < n; ++c) {
        double acc = 0.0;
        for (int q = 0; q < nx; ++q) acc += Q[i * nx + q] * Gx[(static_cast<size_t>(k) * nx + q) * n + c];
        QG[(static_cast<size_t>(k) * nx + i) * n + c] = acc;
      }
  double* H0 = blob + L.H0;
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) {
      double acc = 0.0;
      for (int t = 0; t < H * nx; ++t) acc += Gx[static_cast<size_t>(t) * n + r] * QG[static_cast<size_t>(t) * n + c];
      H0[r * n + c] = 2.0 * acc;
    }
  for (int t = 0; t < H; ++t)
    for (int i = 0; i < nu; ++i)
      for (int j = 0; j < nu; ++j) H0[(t * nu + i) * n + t * nu + j] += 2.0 * R[i * nu + j];
  // F1 = 2 Gx' Qbar Phi  (n x nx),  F2 = 2 Gx' Qbar (n x H*nx)
  double* F1 = blob + L.F1;
  double* F2 = blob + L.F2;
  for (int r = 0; r < n; ++r) {
    for (int c = 0; c < nx; ++c) {
      double acc = 0.0;
      for (int k = 0; k < H; ++k)
        for (int i = 0; i < nx; ++i)
          acc += QG[(static_cast<size_t>(k) * nx + i) * n + r] * Apow[(static_cast<size_t>(k + 1) * nx + i) * nx + c];
      F1[r * nx + c] = 2.0 * acc;
    }
    for (int t = 0; t < H * nx; ++t) F2[static_cast<size_t>(r) * H * nx + t] = 2.0 * QG[static_cast<size_t>(t) * n + r];
  }
  // Mp[i] = C A^i B (2 x nu),  CA[k] = C A^{k+1} (2 x nx)
  for (int p = 0; p < H; ++p)
    for (int i = 0; i < 2; ++i) {
      for (int j = 0; j < nu; ++j) {
        double acc = 0.0;
        for (int k = 0; k < nx; ++k) acc += C[i * nx + k] * AB[(static_cast<size_t>(p) * nx + k) * nu + j];
        blob[L.Mp + (p * 2 + i) * nu + j] = acc;
      }
      for (int j = 0; j < nx; ++j) {
        double acc = 0.0;
        for (int k = 0; k < nx; ++k) acc += C[i * nx + k] * Apow[(static_cast<size_t>(p + 1) * nx + k) * nx + j];
        blob[L.CA + (p * 2 + i) * nx + j] = acc;
      }
    }
  // UF1 = -H0^-1 F1, UF2 = H0^-1 F2 by a Cholesky factorisation of H0 (SPD when R is; otherwise
  // UFOK = 0 and the kernel starts from u = 0)
  {
    std::vector<double> Lc(static_cast<size_t>(n) * n, 0.0);
    bool ok = true;
    for (int j = 0; j < n && ok; ++j) {
      double d = H0[j * n + j];
      for (int k = 0; k < j; ++k) d -= Lc[j * n + k] * Lc[j * n + k];
      if (!(d > 0.0) || !std::isfinite(d)) { ok = false; break; }
      const double ljj = std::sqrt(d);
      Lc[j * n + j] = ljj;
      for (int i = j + 1; i < n; ++i) {
        double acc = H0[i * n + j];
        for (int k = 0; k < j; ++k) acc -= Lc[i * n + k] * Lc[j * n + k];
        Lc[i * n + j] = acc / ljj;
      }
    }
    const int ncols = nx + H * nx;  // right-hand sides: the columns of F1, then of F2
    std::vector<double> col(n);
    for (int c = 0; c < ncols; ++c) {
      for (int r = 0; r < n; ++r)
        col[r] = c < nx ? -F1[r * nx + c] : F2[static_cast<size_t>(r) * H * nx + (c - nx)];
      if (ok) {
        for (int r = 0; r < n; ++r) {  // L y = col
          double acc = col[r];
          for (int k = 0; k < r; ++k) acc -= Lc[r * n + k] * col[k];
          col[r] = acc / Lc[r * n + r];
        }
        for (int r = n - 1; r >= 0; --r) {  // L' x = y
          double acc = col[r];
          for (int k = r + 1; k < n; ++k) acc -= Lc[k * n + r] * col[k];
          col[r] = acc / Lc[r * n + r];
        }
      }
      for (int r = 0; r < n; ++r) {
        const double v = ok ? col[r] : 0.0;
        if (c < nx) blob[L.UF1 + r * nx + c] = v;
        else blob[L.UF2 + static_cast<int64_t>(r) * H * nx + (c - nx)] = v;
      }
    }
    blob[L.UFOK] = ok ? 1.0 : 0.0;
  }
  // a planar isotropic model (nx = 4, nu = 2, A = [[a00 I, a01 I], [a10 I, a11 I]], B = [[b0 I],
  // [b1 I]]; the reference's double integrator) takes the register-form factorisation
  // (riccati_factor_iso); exact comparisons: any other model keeps the general form
  bool iso = nx == 4 && nu == 2;
  for (int bi = 0; bi < 2 && iso; ++bi)
    for (int bj = 0; bj < 2 && iso; ++bj) {
      const double* a = A + 2 * bi * 4 + 2 * bj;  // block (bi, bj), row stride 4
      iso = a[0] == a[5] && a[1] == 0.0 && a[4] == 0.0;
    }
  for (int bi = 0; bi < 2 && iso; ++bi) {
    const double* b = B + 2 * bi * 2;  // rows 2 bi, 2 bi + 1 (row stride 2)
    iso = b[0] == b[3] && b[1] == 0.0 && b[2] == 0.0;
  }
  blob[L.ISO] = iso ? 1.0 : 0.0;
  std::memcpy(blob + L.A, A, sizeof(double) * nx * nx);
  std::memcpy(blob + L.B, B, sizeof(double) * nx * nu);
  std::memcpy(blob + L.C, C, sizeof(double) * 2 * nx);
  std::memcpy(blob + L.Q, Q, sizeof(double) * nx * nx);
  std::memcpy(blob + L.R, R, sizeof(double) * nu * nu);
  return DRCVAR_OK;
}

int64_t drcvar_mpc_workspace_doubles(const drcvar_mpc_model* model, int64_t n_problems,
                                     int64_t n_obstacles) {
  if (!model || n_problems < 0 || n_obstacles < 0) return -1;
  const int c = cluster_limit(n_problems, n_obstacles, kClusterCUs);  // room for any cluster size
  if (c == 1) return n_problems * (kRowArrays * n_obstacles * kStepPad + kBestPad);
  // clustered: the counters first, then per problem the rows, a best iterate per workgroup and
  // the two exchange buffers
  return n_problems * (kCtrlDoubles + kRowArrays * n_obstacles * kStepPad +
                       static_cast<int64_t>(c) * (kBestPad + 2 * kRec));
}

int32_t drcvar_mpc_launch_groups_ex(const drcvar_mpc_model* model, int64_t n_problems,
                                    int64_t n_obstacles, const drcvar_mpc_options* options) {
  if (!model || n_problems < 0 || n_obstacles < 0) return -1;
  if (options && options->cluster_size < 0) return -1;
  if (cluster_limit(n_problems, n_obstacles, kClusterCUs) == 1) return 1;
  const int cus = device_cus();
  const int c = cluster_size(n_problems, n_obstacles, cus > 0 ? cus : 1, options ? options->cluster_size : 0);
  const int c_ws = cluster_limit(n_problems, n_obstacles, kClusterCUs);  // what the workspace holds
  return c < c_ws ? c : c_ws;
}

int32_t drcvar_mpc_launch_groups(const drcvar_mpc_model* model, int64_t n_problems,
                                 int64_t n_obstacles) {
  return drcvar_mpc_launch_groups_ex(model, n_problems, n_obstacles, nullptr);
}

int drcvar_mpc_filter_f64_ex(const drcvar_mpc_model* model, const double* blob, int64_t n_problems,
                             const double* hs_h, const double* hs_g, int64_t n_obstacles,
                             int64_t n_hs_steps, int64_t h_sp, int64_t h_so, int64_t h_sk,
                             int64_t g_sp, int64_t g_so, int64_t g_sk, const double* x0,
                             int64_t x0_sp, const double* x_ref, int64_t xr_sp, int64_t xr_st,
                             const double* u_fallback, int64_t uf_sp, int64_t uf_st,
                             int32_t max_iter, double tol, int32_t polish, double* x_out,
                             double* u_out, double* info_out, double* workspace,
                             int64_t workspace_doubles, const drcvar_mpc_options* options,
                             void* stream) {
  if (!model || !blob || n_problems < 0 || n_obstacles < 0 || n_hs_steps < 0)
    return DRCVAR_ERR_INVALID_ARGUMENT;
  drcvar_mpc_options opt{};
  if (options) opt = *options;
  if (opt.cluster_size < 0 || opt.spin_limit_us < 0) return DRCVAR_ERR_INVALID_ARGUMENT;
  // workgroup 0 of a cluster writes the problem's outputs after the final exchange: stalling it
  // would leave them unwritten instead of reporting CLUSTER_TIMEOUT, so the hook names groups >= 1
  if (opt.debug_stall_group == 1 || opt.debug_stall_group < 0) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (n_problems == 0) return DRCVAR_OK;
  if (!x0 || !x_ref || !u_fallback || !x_out || !u_out || !info_out) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (max_iter < 1 || !(tol > 0.0) || n_problems > 0x7fffffffLL) return DRCVAR_ERR_INVALID_ARGUMENT;
  const int nx = model->n_states, nu = model->n_inputs, H = model->horizon;
  if (nx < 1 || nx > DRCVAR_MPC_MAX_STATES || nu < 1 || nu > DRCVAR_MPC_MAX_INPUTS || H < 1 ||
      H > DRCVAR_MPC_MAX_HORIZON || nu * H > DRCVAR_MPC_MAX_DECISION || model->n_outputs != 2)
    return DRCVAR_ERR_INVALID_ARGUMENT;
  const int64_t K = n_hs_steps < H ? n_hs_steps : H;
  if (K > 0 && n_obstacles > 0 && (!hs_h || !hs_g)) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (n_obstacles > (int64_t{1} << 24)) return DRCVAR_ERR_UNSUPPORTED;
  const int64_t need = drcvar_mpc_workspace_doubles(model, n_problems, n_obstacles);
  if (!workspace || workspace_doubles < need) return DRCVAR_ERR_INVALID_ARGUMENT;

  MpcArgs args{};
  args.blob = blob;
  args.off = blob_layout(nx, nu, H);
  args.nx = nx;
  args.nu = nu;
  args.H = H;
  args.n = nu * H;
  args.K = static_cast<int>(K);
  args.O = static_cast<int>(n_obstacles);
  args.has_u = model->has_input_bounds;
  args.has_p = model->has_position_bounds;
  for (int i = 0; i < DRCVAR_MPC_MAX_INPUTS; ++i) {
    args.umin[i] = model->u_min[i];
    args.umax[i] = model->u_max[i];
  }
  for (int i = 0; i < 2; ++i) {
    args.pmin[i] = model->p_min[i];
    args.pmax[i] = model->p_max[i];
  }
  args.hs_h = hs_h;
  args.hs_g = hs_g;
  args.h_sp = h_sp;
  args.h_so = h_so;
  args.h_sk = h_sk;
  args.g_sp = g_sp;
  args.g_so = g_so;
  args.g_sk = g_sk;
  args.x0 = x0;
  args.x0_sp = x0_sp;
  args.xr = x_ref;
  args.xr_sp = xr_sp;
  args.xr_st = xr_st;
  args.uf = u_fallback;
  args.uf_sp = uf_sp;
  args.uf_st = uf_st;
  args.x_out = x_out;
  args.u_out = u_out;
  args.info = info_out;
  args.ws = workspace;
  args.ws_off = 0;
  args.ws_pp = kRowArrays * n_obstacles * kStepPad + kBestPad;
  args.cl_size = 1;
  const int c_ws = cluster_limit(n_problems, n_obstacles, kClusterCUs);
  if (c_ws > 1) {  // the workspace is laid out for c_ws; a smaller device or the cap uses fewer
    args.ws_off = kCtrlDoubles * n_problems;
    args.ws_pp = kRowArrays * n_obstacles * kStepPad + static_cast<int64_t>(c_ws) * (kBestPad + 2 * kRec);
    args.cl_size = drcvar_mpc_launch_groups_ex(model, n_problems, n_obstacles, &opt);
  }
  args.max_iter = max_iter;
  args.tol = tol;
  args.polish = polish;
  args.spin_ticks = static_cast<uint64_t>(opt.spin_limit_us > 0 ? opt.spin_limit_us : kDefaultSpinUs) * 100u;
  args.force_resume = opt.debug_force_resume != 0;
  args.perturb_group = opt.debug_perturb_group;
  args.perturb_iter = opt.debug_perturb_iteration;
  args.stall_group = opt.debug_stall_group;

  (void)hipGetLastError();
  auto st = static_cast<hipStream_t>(stream);
  int rc;
  switch (nu) {
    case 1: rc = launch_nu1(args, n_problems, st); break;
    case 2: rc = launch_nu2(args, n_problems, st); break;
    case 3: rc = launch_nu3(args, n_problems, st); break;
    default: rc = launch_nu4(args, n_problems, st); break;
  }
  if (rc != DRCVAR_OK) return rc;
  return hipGetLastError() == hipSuccess ? DRCVAR_OK : DRCVAR_ERR_LAUNCH;
}

int drcvar_mpc_filter_f64(const drcvar_mpc_model* model, const double* blob, int64_t n_problems,
                          const double* hs_h, const double* hs_g, int64_t n_obstacles,
                          int64_t n_hs_steps, int64_t h_sp, int64_t h_so, int64_t h_sk,
                          int64_t g_sp, int64_t g_so, int64_t g_sk, const double* x0,
                          int64_t x0_sp, const double* x_ref, int64_t xr_sp, int64_t xr_st,
                          const double* u_fallback, int64_t uf_sp, int64_t uf_st, int32_t max_iter,
                          double tol, int32_t polish, double* x_out, double* u_out, double* info_out,
                          double* workspace, int64_t workspace_doubles, void* stream) {
  return drcvar_mpc_filter_f64_ex(model, blob, n_problems, hs_h, hs_g, n_obstacles, n_hs_steps,
                                  h_sp, h_so, h_sk, g_sp, g_so, g_sk, x0, x0_sp, x_ref, xr_sp,
                                  xr_st, u_fallback, uf_sp, uf_st, max_iter, tol, polish, x_out,
                                  u_out, info_out, workspace, workspace_doubles, nullptr, stream);
}

}  // extern "C"

#endif  // DRCVAR_MPC_HOST_PART
