"""CPU ORACLE — test infrastructure only, never the product path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker.  The shipped path (the HIP kernel behind
``include/drcvar_halfspace.h``) never calls into ``oracle/``.

NumPy float64 restatement of the reference's safe-halfspace hot path:

* ``core/geometry.py:35-53``          compute_separating_vector (unit vector, ``[1,0]`` fallback
                                       when the norm is below 1e-10)
* ``core/halfspaces.py:70-106``       MeanSafeHalfspace.create (direction from the ORIGIN)
* ``core/halfspaces.py:112-149``      CVaRSafeHalfspace.create  -> ``cvar_halfspace``
* ``core/halfspaces.py:155-194``      DRCVaRSafeHalfspace.create -> ``dr_cvar_halfspace``
* ``core/risk_metrics.py:179-265``    CVaROptimizer LP  (rows :198-213)
* ``core/risk_metrics.py:84-177``     DRCVaROptimizer LP (rows :105-125)
* ``core/risk_metrics.py:267-338``    wrappers, ``g_tilde = g_star - r``, sentinel 100.0

The LPs are solved in closed form.  With ``d_i = h . xi_i``, ``k = alpha*N``, ``m = floor(k)`` and
``d_(1) <= ... <= d_(N)``::

    L        = ( sum_{j<=m} d_(j) + (k - m) * d_(m+1) ) / k     (lower-tail mean, Rockafellar-Uryasev)
    g_cvar   = R_c*|h| - delta - L
    g_star   = R_c*|h| - delta + epsilon/alpha - L               (lambda* = 1/alpha, risk_metrics.py:122)
    g_tilde  = g_star - R_c*|h|

Derivation: the CVaR rows (:202-213) say ``tau + 1/(alpha N) sum (l_i - tau)_+ <= delta`` for the loss
``l_i = r - g - d_i``; minimising over tau gives ``CVaR_alpha(l) = r - g - L <= delta``.  The DR rows
(:113-119, a=b=(-1/alpha,0), c=(1-1/alpha,1)) give ``eta_i >= tau + (l_i - tau)_+/alpha`` and the budget
row (:110) adds ``lambda*epsilon`` with lambda pinned to its lower bound 1/alpha (:122).  The closed form
is cross-checked against an LP restatement solved by HiGHS (``oracle/lp_highs.py``) in
``tests/test_oracle.py`` and pinned to the golden vectors in ``tests/golden/``.

LP edge cases mirrored as "solver failure" (``risk_metrics.py:173-177,261-265`` -> sentinels
``:298-303,334-338``): ``alpha > 1`` makes both LPs unbounded (tau -> -inf), ``epsilon < 0`` makes the DR
LP unbounded (lambda -> +inf); non-finite samples make the solver fail.  Sentinel: ``g_cvar = 100``,
``g_star = 100``, ``g_tilde = 100 - R_c*|h|``.
"""
from __future__ import annotations

import numpy as np

SENTINEL = 100.0
OUT_WIDTH = 8
# Column order of the [.., 8] output record (same as include/drcvar_halfspace.h).
COLS = ("mean_h0", "mean_h1", "g_mean", "h0", "h1", "g_cvar", "g_dr_star", "g_dr_tilde")


def separating_vector(ego_pos, obstacle_pos):
    """Vectorised ``core/geometry.py:35-53``: ``(obs - ego)/|obs - ego|``, ``[1, 0]`` if |.| < 1e-10."""
    diff = np.asarray(obstacle_pos, dtype=np.float64) - np.asarray(ego_pos, dtype=np.float64)
    norm = np.sqrt(diff[..., 0] * diff[..., 0] + diff[..., 1] * diff[..., 1])
    degenerate = norm < 1e-10
    with np.errstate(invalid="ignore", divide="ignore"):
        h = diff / norm[..., None]
    h[degenerate] = (1.0, 0.0)
    return h


def lower_tail_mean(d, alpha):
    """Exact ``L`` of the module docstring for each row of ``d`` ([..., N]); NaN where alpha*N > N."""
    d = np.asarray(d, dtype=np.float64)
    n = d.shape[-1]
    k = alpha * n
    if not (k <= n):
        return np.full(d.shape[:-1], np.nan)
    m = int(np.floor(k))
    idx = min(m, n - 1)
    part = np.partition(d, idx, axis=-1)
    tau = part[..., idx]
    s_m = part[..., :m].sum(axis=-1)
    return (s_m + (k - m) * tau) / k


def offsets_given_h(samples, h, alpha, delta, epsilon, robot_radius, obstacle_radius):
    """``cvar_halfspace`` / ``dr_cvar_halfspace`` for a caller-supplied ``h`` (risk_metrics.py:267-338).

    samples [..., N, 2], h [..., 2] -> (g_cvar, g_star, g_tilde), each [...].
    """
    samples = np.asarray(samples, dtype=np.float64)
    h = np.asarray(h, dtype=np.float64)
    rc = robot_radius + obstacle_radius
    hn = np.sqrt(h[..., 0] * h[..., 0] + h[..., 1] * h[..., 1])
    r = rc * hn
    d = h[..., None, 0] * samples[..., 0] + h[..., None, 1] * samples[..., 1]
    finite = np.isfinite(samples).all(axis=(-1, -2))
    L = lower_tail_mean(np.where(finite[..., None], d, 0.0), alpha)
    n = samples.shape[-2]
    ok = finite & (alpha * n <= n)                              # k = alpha N <= N, else unbounded
    g_cvar = np.where(ok, r - delta - L, SENTINEL)
    ok_dr = ok & (epsilon >= 0.0)
    g_star = np.where(ok_dr, r - delta + epsilon / alpha - L, SENTINEL)
    g_tilde = g_star - r
    return g_cvar, g_star, g_tilde


def safe_halfspaces(samples, ego, robot_radius, obstacle_radius, alpha, delta, epsilon):
    """Batched ``compute_safe_halfspaces`` over every (obstacle, step) unit.

    samples [O, T, N, 2] f64, ego [T, 2] f64 -> out [O, T, 8] f64 with columns ``COLS``.
    Mirrors ``simulation/environment.py:82-104`` (loop over t) x ``core/halfspaces.py:225-246``
    (loop over obstacles).
    """
    if alpha <= 0.0:
        raise ValueError("alpha must be > 0")
    samples = np.asarray(samples, dtype=np.float64)
    ego = np.asarray(ego, dtype=np.float64)
    O, T, N, _ = samples.shape
    if N < 1:
        raise ValueError("need at least one sample per unit")
    rc = robot_radius + obstacle_radius
    mu = samples.mean(axis=-2)                                  # halfspaces.py:84 / :130 / :174
    out = np.empty((O, T, OUT_WIDTH), dtype=np.float64)
    hm = separating_vector(np.zeros(2), mu)                     # halfspaces.py:88 (origin!)
    hm_norm = np.sqrt(hm[..., 0] ** 2 + hm[..., 1] ** 2)
    out[..., 0:2] = hm
    out[..., 2] = -((hm[..., 0] * mu[..., 0] + hm[..., 1] * mu[..., 1]) - rc * hm_norm)  # :94
    h = separating_vector(ego[None, :, :], mu)                  # halfspaces.py:130,174
    out[..., 3:5] = h
    g_cvar, g_star, g_tilde = offsets_given_h(samples, h, alpha, delta, epsilon,
                                              robot_radius, obstacle_radius)
    out[..., 5] = g_cvar
    out[..., 6] = g_star
    out[..., 7] = g_tilde
    return out
