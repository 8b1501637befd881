/*
 * drcvar_halfspace.h — C ABI of the MI355X (gfx950) safe-halfspace engine.
 *
 * The reference computes every safe halfspace in Python, one (obstacle, horizon step) at a time,
 * with two CVXPY/ECOS LP solves per unit.  These entry points replace that whole loop with one
 * kernel launch over a batch of units; the Python host layer
 * (dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/) keeps the reference's call
 * surface on top of them.
 *
 *   drcvar_safe_halfspaces_f64   replaces  core/halfspaces.py:196-248  compute_safe_halfspaces
 *                                 (mean, CVaR and DR-CVaR halfspaces for every obstacle), batched
 *                                 over the horizon loop of simulation/environment.py:60-106
 *                                 (compute_safe_halfspaces_for_trajectory); per unit it covers
 *                                 core/halfspaces.py:70-106 (MeanSafeHalfspace.create),
 *                                 :112-149 (CVaRSafeHalfspace.create), :155-194
 *                                 (DRCVaRSafeHalfspace.create) and core/geometry.py:35-53.
 *   drcvar_offsets_given_h_f64   replaces  core/risk_metrics.py:305-338  cvar_halfspace and
 *                                 core/risk_metrics.py:267-303  dr_cvar_halfspace (caller supplies
 *                                 the direction h; the LPs of :84-177 and :179-265 are evaluated in
 *                                 closed form).
 *
 * Conventions
 *  - All pointers are DEVICE pointers (hipMalloc / torch CUDA tensors) except where noted; the
 *    caller owns every buffer.  No allocation, no host synchronisation inside a call; work is
 *    enqueued on `stream` (a hipStream_t passed as void*, NULL = the default stream) and the call
 *    returns immediately, so a call may be captured into a hipGraph.
 *  - Strides are in units of double.  The two coordinates of one sample are adjacent (stride 1).
 *  - Thread-safe: no global mutable state.
 *  - Output record: 8 doubles per unit, unit u = o * n_steps + t, laid out as DRCVAR_COL_*.
 *  - Errors are returned as DRCVAR_* codes; drcvar_strerror() gives a static message.  Numerical
 *    "solver failure" is not an error: like the reference (core/risk_metrics.py:173-177,261-265,
 *    298-303,334-338) the offsets become the sentinel 100.0 (g_dr_tilde = 100 - R_c*|h|) when the
 *    samples of a unit are not all finite, when alpha > 1 (both LPs unbounded) or, for DR-CVaR
 *    only, when epsilon < 0 (DR LP unbounded).
 */
#ifndef DRCVAR_HALFSPACE_H
#define DRCVAR_HALFSPACE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DRCVAR_ABI_VERSION 3 /* 2: MPC options / cluster statuses, per-unit status outputs;
                                3: the peer-push exchange (drcvar_exchange.h) */

/* return codes */
#define DRCVAR_OK 0
#define DRCVAR_ERR_INVALID_ARGUMENT 1 /* null pointer, negative size, n_samples < 1, alpha <= 0, ... */
#define DRCVAR_ERR_UNSUPPORTED 2      /* n_samples above DRCVAR_MAX_SAMPLES_STREAM, or an explicit
                                         geometry that does not exist / cover n_samples */
#define DRCVAR_ERR_LAUNCH 3           /* the HIP runtime refused the launch */

/* largest n_samples a single unit may hold (samples are kept on chip, in registers) */
#define DRCVAR_MAX_SAMPLES 16384
/* larger units run a streaming kernel (samples re-read from memory instead of held on chip;
   ~4 reads of the unit's samples instead of 1) up to this many samples */
#define DRCVAR_MAX_SAMPLES_STREAM 2147483647

/* output record columns */
#define DRCVAR_COL_MEAN_H0 0    /* MeanSafeHalfspace.h[0]   (direction from the origin, halfspaces.py:88) */
#define DRCVAR_COL_MEAN_H1 1    /* MeanSafeHalfspace.h[1] */
#define DRCVAR_COL_G_MEAN 2     /* MeanSafeHalfspace.g_tilde (halfspaces.py:94) */
#define DRCVAR_COL_H0 3         /* CVaR / DR-CVaR direction h[0] (halfspaces.py:130,174) */
#define DRCVAR_COL_H1 4         /* h[1] */
#define DRCVAR_COL_G_CVAR 5     /* CVaRSafeHalfspace.g_tilde = cvar_halfspace() (risk_metrics.py:305) */
#define DRCVAR_COL_G_DR_STAR 6  /* g_star of dr_cvar_halfspace() (risk_metrics.py:267) */
#define DRCVAR_COL_G_DR_TILDE 7 /* DRCVaRSafeHalfspace.g_tilde = g_star - R_c*|h| (risk_metrics.py:299) */
#define DRCVAR_OUT_WIDTH 8

/* per-unit status word (optional int32 output of the _v2 entry points), a bit set: which of the
   reference's solver-failure branches the unit took (core/risk_metrics.py:173-177, 261-265,
   298-303, 334-338), so callers need not infer failure from the sentinel's value */
#define DRCVAR_UNIT_OK 0
#define DRCVAR_UNIT_NONFINITE 1    /* a sample is not finite, or the sample sums overflow: every
                                      offset is the sentinel (both LPs fail) */
#define DRCVAR_UNIT_UNBOUNDED 2    /* alpha * N > N: both LPs unbounded, every offset the sentinel */
#define DRCVAR_UNIT_DR_UNBOUNDED 4 /* epsilon < 0: the DR-CVaR LP unbounded (g_star = 100,
                                      g_dr_tilde = 100 - R_c|h|); the CVaR offset stands */

int drcvar_abi_version(void);
const char* drcvar_strerror(int code);

/*
 * Mean, CVaR and DR-CVaR safe halfspaces for n_obstacles x n_steps units of n_samples 2-D samples.
 *   samples  sample i of obstacle o at step t is (samples[o*stride_obstacle + t*stride_step +
 *            i*stride_sample], ... + 1).  The packed [O, T, N, 2] layout (strides T*N*2, N*2, 2) is
 *            the fast path; the reference's per-obstacle [N, S+1, 2] trajectories stacked as
 *            [O, N, S+1, 2] are accepted directly with strides (N*(S+1)*2, 2, (S+1)*2).
 *   ego_ref_pos  ego reference position at step t is (ego_ref_pos[t*ego_stride_step], ... + 1)
 *            (environment.py:92: C @ x_ref[t]).
 *   robot_radius, obstacle_radius, alpha, delta, epsilon: as compute_safe_halfspaces().
 *   out      [n_obstacles * n_steps, DRCVAR_OUT_WIDTH] doubles, contiguous.
 */
int drcvar_safe_halfspaces_f64(const double* samples, int64_t n_obstacles, int64_t n_steps,
                               int64_t n_samples, int64_t stride_obstacle, int64_t stride_step,
                               int64_t stride_sample, const double* ego_ref_pos,
                               int64_t ego_stride_step, double robot_radius,
                               double obstacle_radius, double alpha, double delta, double epsilon,
                               double* out, void* stream);

/*
 * drcvar_safe_halfspaces_f64 with an explicit launch geometry (threads per unit and samples held
 * per thread; both 0 = automatic, the plan drcvar_launch_plan reports).  For tuning: returns
 * DRCVAR_ERR_UNSUPPORTED when no compiled geometry matches or threads * samples < n_samples.
 */
int drcvar_safe_halfspaces_f64_ex(const double* samples, int64_t n_obstacles, int64_t n_steps,
                                  int64_t n_samples, int64_t stride_obstacle, int64_t stride_step,
                                  int64_t stride_sample, const double* ego_ref_pos,
                                  int64_t ego_stride_step, double robot_radius,
                                  double obstacle_radius, double alpha, double delta,
                                  double epsilon, double* out, void* stream,
                                  int32_t threads_per_unit, int32_t samples_per_thread);

/*
 * drcvar_safe_halfspaces_f64_ex that also writes the per-unit status word (DRCVAR_UNIT_*) into
 * status[n_obstacles * n_steps] (int32, device; NULL = not written).  Same cost: one 4-B store
 * per unit.
 */
int drcvar_safe_halfspaces_f64_v2(const double* samples, int64_t n_obstacles, int64_t n_steps,
                                  int64_t n_samples, int64_t stride_obstacle, int64_t stride_step,
                                  int64_t stride_sample, const double* ego_ref_pos,
                                  int64_t ego_stride_step, double robot_radius,
                                  double obstacle_radius, double alpha, double delta,
                                  double epsilon, double* out, int32_t* status, void* stream,
                                  int32_t threads_per_unit, int32_t samples_per_thread);

/*
 * cvar_halfspace / dr_cvar_halfspace for n_units units with a caller-supplied direction
 * h[u] = (h[u*h_stride_unit], h[u*h_stride_unit + 1]) (not necessarily unit length; the combined
 * radius is scaled by |h| exactly as risk_metrics.py:293 / :234 do).  The output record has the
 * same layout; columns DRCVAR_COL_H0/H1 echo h, columns 0..2 hold the mean halfspace.
 */
int drcvar_offsets_given_h_f64(const double* samples, int64_t n_units, int64_t n_samples,
                               int64_t stride_unit, int64_t stride_sample, const double* h,
                               int64_t h_stride_unit, double robot_radius, double obstacle_radius,
                               double alpha, double delta, double epsilon, double* out,
                               void* stream);
/* the same with the per-unit status word (status[n_units], NULL = not written) */
int drcvar_offsets_given_h_f64_v2(const double* samples, int64_t n_units, int64_t n_samples,
                                  int64_t stride_unit, int64_t stride_sample, const double* h,
                                  int64_t h_stride_unit, double robot_radius,
                                  double obstacle_radius, double alpha, double delta,
                                  double epsilon, double* out, int32_t* status, void* stream);

/*
 * Host-only query (no device access): the launch geometry chosen for n_samples — threads per
 * workgroup, samples held per thread (0 = the streaming kernel, n_samples > DRCVAR_MAX_SAMPLES)
 * and histogram bins.  Returns DRCVAR_OK or an error code.
 */
int drcvar_launch_plan(int64_t n_samples, int32_t* threads_per_unit, int32_t* samples_per_thread,
                       int32_t* bins);

#ifdef __cplusplus
}
#endif

#endif /* DRCVAR_HALFSPACE_H */
