/*
 * drcvar_mpc.h — C ABI of the MI355X (gfx950) MPC safety-filter QP (the halfspace hand-off).
 *
 * The reference consumes the safe halfspaces in core/mpc_filter.py:40-178
 * (MPCSafetyFilter.filter_trajectory): it builds a CVXPY problem over states, inputs and one slack
 * per halfspace and calls the default QP solver, falling back to a shifted previous solution
 * (_fallback, :180-219) when the solve does not succeed.  These entry points replace that call:
 *
 *   drcvar_mpc_model_init     replaces the per-call problem construction of :60-144 — the part that
 *                             depends only on (A, B, C, Q, R, horizon, bounds) is condensed once on
 *                             the host (prediction matrices, Hessian) into a blob of doubles the
 *                             caller uploads to the device;
 *   drcvar_mpc_filter_f64     replaces problem.solve() (:151) + the status handling of :154-178 +
 *                             the fallback rollout of :180-219, for a batch of independent
 *                             problems, one workgroup per problem, entirely on the device.
 *
 * Problem (identical to the reference's, core/mpc_filter.py):
 *   min  sum_t (x_{t+1}-xr_{t+1})'Q(x_{t+1}-xr_{t+1}) + u_t'R u_t + sum 50 s + 50 s^2
 *   s.t. x_0 = x0, x_{t+1} = A x_t + B u_t, u_min <= u_t <= u_max, p_min <= C x_t <= p_max,
 *        h . C x_{k+1} + g <= s, s >= 0 for every halfspace (h, g) of step k < min(K, horizon).
 * Solved in the input space (states eliminated) by a primal-dual Mehrotra interior-point method;
 * the halfspace rows enter the Newton system only through per-step 2x2 reductions, and each Newton
 * system is solved by a Riccati recursion over the horizon (no dense Hessian is factored).
 *
 * Conventions as in drcvar_halfspace.h: device pointers unless noted, caller-owned buffers, no
 * allocation or synchronisation inside drcvar_mpc_filter_f64, strides in doubles, DRCVAR_* codes.
 */
#ifndef DRCVAR_MPC_H
#define DRCVAR_MPC_H

#include <stdint.h>

#include "drcvar_halfspace.h"

#ifdef __cplusplus
extern "C" {
#endif

/* limits of the single-workgroup solver (per-step Riccati factors and input vectors live in LDS) */
#define DRCVAR_MPC_MAX_STATES 8
#define DRCVAR_MPC_MAX_INPUTS 4
#define DRCVAR_MPC_MAX_HORIZON 64
#define DRCVAR_MPC_MAX_DECISION 120 /* n_inputs * horizon */

/* info record, DRCVAR_MPC_INFO_WIDTH doubles per problem */
#define DRCVAR_MPC_INFO_WIDTH 10
#define DRCVAR_MPC_INFO_STATUS 0        /* DRCVAR_MPC_STATUS_* */
#define DRCVAR_MPC_INFO_ITERATIONS 1
#define DRCVAR_MPC_INFO_OBJECTIVE 2     /* reference objective at the returned trajectory (optimal only) */
#define DRCVAR_MPC_INFO_MU 3            /* merit of the returned iterate (see tol) */
#define DRCVAR_MPC_INFO_PRIMAL_RES 4    /* max-norm primal residual of the last iterate */
#define DRCVAR_MPC_INFO_DUAL_RES 5      /* max-norm dual residual of the last iterate */
#define DRCVAR_MPC_INFO_MAX_SLACK 6     /* largest halfspace slack s (0 = every halfspace satisfied) */
#define DRCVAR_MPC_INFO_USED_FALLBACK 7 /* 1 when the fallback inputs were rolled out (:180-219) */
#define DRCVAR_MPC_INFO_POLISHED 8      /* 1 when the active-set polish succeeded (exact optimum) */
#define DRCVAR_MPC_INFO_POLISH_ATTEMPTS 9

#define DRCVAR_MPC_STATUS_OPTIMAL 0
#define DRCVAR_MPC_STATUS_MAX_ITER 1  /* not converged (e.g. infeasible input/position boxes) */
#define DRCVAR_MPC_STATUS_NUMERICAL 2 /* non-positive pivot or non-finite iterate */
#define DRCVAR_MPC_STATUS_OPTIMAL_INACCURATE 3 /* stalled with merit <= 1e3*tol; best iterate
                                                  returned (accepted, like mpc_filter.py:154) */
/* clustered launches only (drcvar_mpc_launch_groups > 1); both roll the fallback inputs out */
#define DRCVAR_MPC_STATUS_CLUSTER_TIMEOUT 4  /* a workgroup of the problem's cluster did not reach an
                                                exchange within the spin limit (e.g. it could not be
                                                made resident beside other work on the device) */
#define DRCVAR_MPC_STATUS_CLUSTER_DIVERGED 5 /* the cluster's workgroups disagreed on a replicated
                                                decision (their published state digests differ) */

/*
 * Per-call options (NULL = every field 0 = the defaults).  No environment variable is read by the
 * library: what is not set here is the default, and a hipGraph capture freezes what was passed.
 *   cluster_size      0 = automatic; 1 = one workgroup per problem; c > 1 = clusters of c
 *                     workgroups where the batch is eligible (capped like the automatic size)
 *   spin_limit_us     0 = 10000: a cluster exchange that waits longer ends the problem with
 *                     DRCVAR_MPC_STATUS_CLUSTER_TIMEOUT (fallback rollout) instead of hanging
 *   debug_*           test hooks (tests/test_mpc_cluster.py), 0 = off:
 *     debug_force_resume        the first polish gives up at once (exercises the resume round)
 *     debug_perturb_group       g + 1: workgroup g of every cluster scales its step length by
 *                               (1 - 2^-20) at interior-point iteration debug_perturb_iteration
 *                               (must end with DRCVAR_MPC_STATUS_CLUSTER_DIVERGED)
 *     debug_stall_group         g + 1: workgroup g (g >= 1) of every cluster leaves before the
 *                               final exchange (must end with DRCVAR_MPC_STATUS_CLUSTER_TIMEOUT);
 *                               g = 0 is rejected (workgroup 0 writes the outputs)
 */
typedef struct drcvar_mpc_options {
  int32_t cluster_size;
  int32_t spin_limit_us;
  int32_t debug_force_resume;
  int32_t debug_perturb_group;
  int32_t debug_perturb_iteration;
  int32_t debug_stall_group;
  int32_t reserved[2];
} drcvar_mpc_options;

/* Host-side description of a condensed model (filled by drcvar_mpc_model_init). */
typedef struct drcvar_mpc_model {
  int32_t n_states, n_inputs, n_outputs, horizon;
  int32_t has_input_bounds, has_position_bounds;
  double u_min[DRCVAR_MPC_MAX_INPUTS], u_max[DRCVAR_MPC_MAX_INPUTS];
  double p_min[2], p_max[2];
  int64_t blob_doubles; /* size of the device blob */
} drcvar_mpc_model;

/*
 * Condense (A, B, C, Q, R, horizon) — HOST pointers, row-major, A [nx,nx], B [nx,nu], C [ny,nx],
 * Q [nx,nx], R [nu,nu] — into `model` and, when `blob` is not NULL, into the host buffer `blob`
 * (model->blob_doubles doubles; call once with blob = NULL to size it).  The caller copies the blob
 * to device memory and passes that pointer to drcvar_mpc_filter_f64.  Bounds may be NULL (no
 * constraint, core/mpc_filter.py:89,96); u_min/u_max hold n_inputs values, p_min/p_max n_outputs
 * (the reference truncates longer bound vectors to C's rows, :103-110).  n_outputs must be 2
 * (halfspaces are planar).  Pure host function (no device needed).
 */
int drcvar_mpc_model_init(const double* A, const double* B, const double* C, const double* Q,
                          const double* R, int32_t n_states, int32_t n_inputs, int32_t n_outputs,
                          int32_t horizon, const double* u_min, const double* u_max,
                          const double* p_min, const double* p_max, drcvar_mpc_model* model,
                          double* blob);

/* Doubles of device workspace drcvar_mpc_filter_f64 needs for this batch (clustered shapes, see
 * drcvar_mpc_launch_groups, also hold per-problem arrival counters at the workspace's start and
 * exchange buffers; the launch zeroes the counters itself). */
int64_t drcvar_mpc_workspace_doubles(const drcvar_mpc_model* model, int64_t n_problems,
                                     int64_t n_obstacles);

/*
 * Workgroups per problem the next drcvar_mpc_filter_f64 launch of this batch shape uses on the
 * current device: 1 (one workgroup per problem), or a cluster of c > 1 workgroups that split the
 * problem's halfspace rows (batches of at most 8 problems with >= 64 obstacles: one workgroup per
 * 16 obstacles, c <= 32 and c * n_problems <= half the device's CUs, so that a clustered launch
 * stays resident beside other work).  The _ex form applies options->cluster_size.
 * Host query (reads the device's CU count).  -1 on invalid arguments.
 */
int32_t drcvar_mpc_launch_groups(const drcvar_mpc_model* model, int64_t n_problems,
                                 int64_t n_obstacles);
int32_t drcvar_mpc_launch_groups_ex(const drcvar_mpc_model* model, int64_t n_problems,
                                    int64_t n_obstacles, const drcvar_mpc_options* options);

/*
 * Solve n_problems independent safety-filter QPs.
 *   model, blob             from drcvar_mpc_model_init (model: host struct; blob: device copy)
 *   hs_h, hs_g              halfspace directions / offsets: problem b, obstacle o, halfspace step k
 *                           at hs_h + b*h_sp + o*h_so + k*h_sk (h[1] at +1) and hs_g + b*g_sp +
 *                           o*g_so + k*g_sk.  Step k constrains x_{k+1} (mpc_filter.py:117-121);
 *                           steps k >= horizon are ignored.  For the [O, T, 8] record of
 *                           drcvar_safe_halfspaces_f64: dr_cvar = (rec+3, rec+7), cvar = (rec+3,
 *                           rec+5), mean = (rec+0, rec+2) with strides (T*8, 8).
 *   x0 [B, nx]              initial states (row stride x0_sp)
 *   x_ref [B, horizon+1, nx] reference states (strides xr_sp, xr_st; column stride 1)
 *   u_fallback [B, horizon, nu] inputs rolled out when a problem is not solved (the caller builds
 *                           them as _fallback does: shifted last optimum, else u_ref)
 *   x_out [B, horizon+1, nx], u_out [B, horizon, nu], info_out [B, DRCVAR_MPC_INFO_WIDTH]: dense
 *   workspace               drcvar_mpc_workspace_doubles() doubles: scratch of the solver, whose
 *                           contents at exit are unspecified.  Per problem it reserves ten
 *                           [n_obstacles, 64] row arrays (h0, h1, g, s, w_hs, lambda_hs, w_s,
 *                           lambda_s and two saved across a failed polish), then per workgroup the
 *                           best iterate and the saved bound states.  The row arrays are used
 *                           only by the forms that keep their rows in global memory: the clustered
 *                           rows-in-LDS form (a cluster whose obstacle slice fits in LDS, e.g. the
 *                           C5 hand-off) keeps its row slice in LDS and never writes them back, so
 *                           no caller may read slacks or duals from the workspace
 *   max_iter, tol           interior-point limits (e.g. 60, 1e-7); converged when
 *                           max(|r_primal|/(1+|d|), |r_dual|/(1+|q|), mean complementarity) <= tol
 *   polish                  nonzero: finish with the active-set polish (method of multipliers on
 *                           the equality QP of the identified active set, with active-set
 *                           corrections) — exact to roundoff when it succeeds, as OSQP's polish;
 *                           when it fails on a problem that met tol, the interior-point method
 *                           resumes for up to 8 iterations towards tol * 1e-3 and polishes again;
 *                           a first round stalled at merit <= 1e-3 polishes early (two corrections)
 *                           and, when that fails, resumes towards tol
 */
int drcvar_mpc_filter_f64(const drcvar_mpc_model* model, const double* blob, int64_t n_problems,
                          const double* hs_h, const double* hs_g, int64_t n_obstacles,
                          int64_t n_hs_steps, int64_t h_sp, int64_t h_so, int64_t h_sk,
                          int64_t g_sp, int64_t g_so, int64_t g_sk, const double* x0,
                          int64_t x0_sp, const double* x_ref, int64_t xr_sp, int64_t xr_st,
                          const double* u_fallback, int64_t uf_sp, int64_t uf_st, int32_t max_iter,
                          double tol, int32_t polish, double* x_out, double* u_out,
                          double* info_out, double* workspace, int64_t workspace_doubles,
                          void* stream);
/* drcvar_mpc_filter_f64 with per-call options (NULL = defaults; see drcvar_mpc_options) */
int drcvar_mpc_filter_f64_ex(const drcvar_mpc_model* model, const double* blob, int64_t n_problems,
                             const double* hs_h, const double* hs_g, int64_t n_obstacles,
                             int64_t n_hs_steps, int64_t h_sp, int64_t h_so, int64_t h_sk,
                             int64_t g_sp, int64_t g_so, int64_t g_sk, const double* x0,
                             int64_t x0_sp, const double* x_ref, int64_t xr_sp, int64_t xr_st,
                             const double* u_fallback, int64_t uf_sp, int64_t uf_st,
                             int32_t max_iter, double tol, int32_t polish, double* x_out,
                             double* u_out, double* info_out, double* workspace,
                             int64_t workspace_doubles, const drcvar_mpc_options* options,
                             void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DRCVAR_MPC_H */
