/*
 * drcvar_sampling.h — C ABI of the MI355X (gfx950) obstacle-sample generator.
 *
 * The reference draws every obstacle's Monte Carlo sample trajectories on the host
 * (simulation/obstacles.py:43-77 generate_obstacle_sample_trajectories: per step, n_samples draws
 * of N(0, noise_cov) added to the nominal position; step 0 noise-free, :63) and the caller ships
 * them to the solver.  This entry point generates the same distribution directly in device memory,
 * in the layout drcvar_safe_halfspaces_f64 consumes, so a GPU pipeline never stages samples
 * through the host.
 *
 *   drcvar_sample_trajectories_f64   replaces simulation/obstacles.py:43-77 (and the per-obstacle
 *                                    loop of generate_obstacle_scenarios, :150-163) for a batch
 *                                    of obstacles.
 *   drcvar_sample_units_f64          the same draws for a contiguous block of (obstacle, step)
 *                                    units of a global batch (one rank's shard).
 *
 * Random numbers: Philox4x32-10 (counter-based; key = seed, counter = (unit * ceil(N/2) + pair,
 * stream)), one call per PAIR of samples of a unit -> two (32-bit uniform, 32-bit turn) pairs ->
 * Box-Muller -> z ~ N(0, I2); sample = nominal + L z with L the lower Cholesky factor of noise_cov
 * (for L = l I, l > 0 — the reference's default — the kernel folds l^2 into the log of Box-Muller
 * and adds l z directly: the same values to a few ulp).
 * Tail: the radius uniform is 32-bit (u = (2x + 1) 2^-33 >= 2^-33), so |z| <= sqrt(66 ln 2) = 6.76
 * and the far tail is quantised in steps of 2^-32 in u; the reference's 53-bit draws exceed 6.76 sd
 * with probability 2^-33 per sample (~0.0075 samples per 128 M-sample C5 refill).  Below the cap the
 * Rayleigh tail frequencies are kept (tests/test_sampling.py::test_device_sampler_radius_tail).
 * Same distribution as the reference's
 * np.random.multivariate_normal, not the same stream (numpy's MT19937 is sequential; the host
 * mirror in simulation/obstacles.py reproduces that stream exactly).  Output is a pure function
 * of (seed, stream_offset, indices): deterministic and independent of the launch geometry.
 *
 * Conventions as in drcvar_halfspace.h (device pointers, caller-owned buffers, strides in doubles,
 * async on `stream`, DRCVAR_* return codes).
 */
#ifndef DRCVAR_SAMPLING_H
#define DRCVAR_SAMPLING_H

#include <stdint.h>

#include "drcvar_halfspace.h"

#ifdef __cplusplus
extern "C" {
#endif

/*
 * nominal      [n_obstacles, n_steps, 2] nominal positions (strides nom_so, nom_st; coords adjacent)
 * l00,l10,l11  lower Cholesky factor of the 2x2 noise covariance (reference default diag(0.01, 0.01)
 *              -> 0.1, 0, 0.1; simulation/obstacles.py:134)
 * seed         Philox key; stream_offset selects an independent stream (e.g. per rank)
 * zero_first_step  nonzero: step 0 is the nominal position for every sample (obstacles.py:63)
 * out          [n_obstacles, n_steps, n_samples, 2] with strides (so, st, sn), coords adjacent
 */
int drcvar_sample_trajectories_f64(const double* nominal, int64_t n_obstacles, int64_t n_steps,
                                   int64_t nom_so, int64_t nom_st, int64_t n_samples, double l00,
                                   double l10, double l11, uint64_t seed, uint64_t stream_offset,
                                   int32_t zero_first_step, double* out, int64_t so, int64_t st,
                                   int64_t sn, void* stream);

/*
 * Units [unit_begin, unit_begin + unit_count) of the global [n_obstacles, n_steps] grid (unit
 * u = o * n_steps + t), written flat: unit u at out + (u - unit_begin) * su, sample i at + i * sn.
 * Every sample is the one drcvar_sample_trajectories_f64 draws for the whole grid (same Philox
 * counter u * n_samples + i), so a rank can draw its shard of a global batch without the rest
 * (per-rank sampling of contiguous unit blocks).  nominal is the GLOBAL
 * [n_obstacles, n_steps, 2] path.
 */
int drcvar_sample_units_f64(const double* nominal, int64_t n_obstacles, int64_t n_steps,
                            int64_t nom_so, int64_t nom_st, int64_t unit_begin, int64_t unit_count,
                            int64_t n_samples, double l00, double l10, double l11, uint64_t seed,
                            uint64_t stream_offset, int32_t zero_first_step, double* out,
                            int64_t su, int64_t sn, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DRCVAR_SAMPLING_H */
