"""CPU ORACLE — test infrastructure only, never the product path.

LP restatement of the reference's two optimisers, solved with HiGHS (``scipy.optimize.linprog``) in
place of CVXPY 1.2.1 + ECOS 2.0.14 (``environment.yml:31,33``; neither is installed in this image).
The rows are written out exactly as the reference builds them, so this is the reference's own
mathematical problem — only the interior-point solver is swapped.  It is the "algorithm class"
CPU baseline (one LP per halfspace) and the independent check on ``oracle/closed_form.py``.

CVaR (``core/risk_metrics.py:182-213``), variables ``x = [g, tau, aux_1..aux_N]``::

    min g   s.t.  aux >= 0                                           (:202)
                  aux_i >= -h.xi_i - g + r - tau                     (:206-209)
                  tau + 1/(alpha N) * sum(aux) <= delta              (:212-213)

DR-CVaR (``core/risk_metrics.py:87-125``), variables ``x = [g, tau, lambda, eta_1..eta_N]``::

    min g   s.t.  lambda*epsilon + (1/N) sum(eta) <= delta           (:110)
                  a_k h.xi_i + b_k (g - r) + c_k tau <= eta_i        (:113-119)
                  a = b = (-1/alpha, 0), c = (1 - 1/alpha, 1)        (:105-107)
                  lambda >= 0 (:97), lambda >= 1/alpha               (:122)

Status handling mirrors ``:173-177`` / ``:261-265``: anything but optimal -> sentinel 100.0, and the
DR wrapper returns ``(100.0, 100.0 - r)`` (``:298-303``).
"""
from __future__ import annotations

import numpy as np
from scipy import sparse
from scipy.optimize import linprog

SENTINEL = 100.0


def _h_xi(h, samples):
    h = np.asarray(h, dtype=np.float64)
    samples = np.asarray(samples, dtype=np.float64)
    return samples @ h                                           # risk_metrics.py:145 / :233


def cvar_lp(h_xi, r, alpha, delta):
    """The CVaR LP of :182-213 on its parameters (``h_xi_param`` = h.xi_i, ``r_param``).
    Returns ``(solved, g)``."""
    hxi = np.asarray(h_xi, dtype=np.float64).reshape(-1)
    n = hxi.shape[0]
    nv = 2 + n
    c = np.zeros(nv)
    c[0] = 1.0
    # -g - tau - aux_i <= h.xi_i - r
    rows = sparse.hstack([
        sparse.csr_matrix(-np.ones((n, 1))),
        sparse.csr_matrix(-np.ones((n, 1))),
        -sparse.identity(n, format="csr"),
    ])
    budget = np.zeros((1, nv))
    budget[0, 1] = 1.0
    budget[0, 2:] = 1.0 / (alpha * n)
    A = sparse.vstack([rows, sparse.csr_matrix(budget)]).tocsc()
    b = np.concatenate([hxi - r, [delta]])
    bounds = [(None, None), (None, None)] + [(0.0, None)] * n
    res = linprog(c, A_ub=A, b_ub=b, bounds=bounds, method="highs")
    if res.status != 0:
        return False, SENTINEL
    return True, float(res.x[0])


def dr_cvar_lp(h_xi, r, alpha, delta, epsilon):
    """The DR-CVaR LP of :87-125 on its parameters (``h_xi_param``, ``r_param``).
    Returns ``(solved, g*)``."""
    hxi = np.asarray(h_xi, dtype=np.float64).reshape(-1)
    n = hxi.shape[0]
    a_k = (-1.0 / alpha, 0.0)
    b_k = (-1.0 / alpha, 0.0)
    c_k = (1.0 - 1.0 / alpha, 1.0)
    nv = 3 + n                                                   # g, tau, lambda, eta
    c = np.zeros(nv)
    c[0] = 1.0
    blocks = []
    rhs = []
    for k in range(2):
        # b_k g + c_k tau - eta_i <= -a_k hxi_i + b_k r
        blk = sparse.hstack([
            sparse.csr_matrix(np.full((n, 1), b_k[k])),
            sparse.csr_matrix(np.full((n, 1), c_k[k])),
            sparse.csr_matrix((n, 1)),
            -sparse.identity(n, format="csr"),
        ])
        blocks.append(blk)
        rhs.append(-a_k[k] * hxi + b_k[k] * r)
    budget = np.zeros((1, nv))
    budget[0, 2] = epsilon
    budget[0, 3:] = 1.0 / n
    A = sparse.vstack(blocks + [sparse.csr_matrix(budget)]).tocsc()
    b = np.concatenate(rhs + [[delta]])
    bounds = [(None, None), (None, None), (max(0.0, 1.0 / alpha), None)] + [(None, None)] * n
    res = linprog(c, A_ub=A, b_ub=b, bounds=bounds, method="highs")
    if res.status != 0:
        return False, SENTINEL
    return True, float(res.x[0])


def solve_cvar_lp(samples, h, alpha, delta, robot_radius, obstacle_radius):
    """``cvar_halfspace`` (risk_metrics.py:305-338) with the LP of :182-213. Returns g."""
    r = (robot_radius + obstacle_radius) * np.linalg.norm(h)    # :329 and :234
    return cvar_lp(_h_xi(h, samples), r, alpha, delta)[1]


def solve_dr_cvar_lp(samples, h, alpha, delta, epsilon, robot_radius, obstacle_radius):
    """``dr_cvar_halfspace`` (risk_metrics.py:267-303) with the LP of :87-125. Returns (g*, g~)."""
    r = (robot_radius + obstacle_radius) * np.linalg.norm(h)    # :293
    ok, g_star = dr_cvar_lp(_h_xi(h, samples), r, alpha, delta, epsilon)
    if not ok:
        return SENTINEL, SENTINEL - r
    return g_star, g_star - r
