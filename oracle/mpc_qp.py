"""CPU ORACLE — test infrastructure only, never the product path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker.  The shipped MPC hand-off (``csrc/drcvar_mpc.hip`` behind
``include/drcvar_mpc.h``) never calls into ``oracle/``.

Restatement of the safety-filter QP that ``MPCSafetyFilter.filter_trajectory``
(``core/mpc_filter.py:40-178``) hands to CVXPY, written in the reference's own *full-space* form —
states, inputs and one slack per halfspace are all variables, the dynamics are equality rows —
and solved by a sparse primal-dual (Mehrotra) interior-point method (NumPy/SciPy float64)::

    min  sum_{t=0}^{H-1} (x_{t+1}-xr_{t+1})' Q (x_{t+1}-xr_{t+1}) + u_t' R u_t      (:67-76)
         + sum_{t=1}^{H} sum_j 50 s_tj + 50 s_tj^2                                    (:142-144)
    s.t. x_0 = x0                                                                      (:82)
         x_{t+1} = A x_t + B u_t                                                       (:85-86)
         u_min <= u_t <= u_max                    (if input_constraints)               (:89-93)
         p_min <= C x_t <= p_max, t = 1..H        (if position_constraints; bounds
                                                   truncated to C's rows)              (:96-113)
         h_tj . C x_t + g_tj <= s_tj,  s_tj >= 0  for the halfspaces of
                                                   safe_halfspaces[t-1], t-1 < len     (:117-140)

``quad_form(v, Q)`` is ``v'Qv`` (no 1/2).  The reference solves with CVXPY 1.2.1's default QP solver
(OSQP; ``environment.yml:31``), which is not installed here, so parity against OSQP's iterates is
unpinned; what IS pinned is the mathematical answer: the objective is strictly convex in
(x, u, s) (R > 0, the slack Hessian is 100), so the optimum is unique, and this module returns it
with a KKT certificate (:func:`kkt_residuals`) that the tests check to ~1e-9.  The GPU kernel uses
a different (condensed, input-space) formulation, so the two are independent computations of the
same unique point.

Failure handling mirrors ``:170-178`` + ``_fallback`` (``:180-219``): a problem the IPM does not
solve (infeasible input/position boxes) takes the fallback trajectory.
"""
from __future__ import annotations

import numpy as np
from scipy import sparse
from scipy.sparse import linalg as splinalg

SLACK_LINEAR = 50.0      # core/mpc_filter.py:143
SLACK_QUADRATIC = 50.0   # core/mpc_filter.py:144
_TRACE = False


def _bounds(bounds, dim):
    """(min, max) pair truncated to ``dim`` entries, as ``core/mpc_filter.py:103-110`` does."""
    if bounds is None:
        return None
    lo, hi = bounds
    lo = np.asarray(lo, dtype=np.float64).reshape(-1)[:dim]
    hi = np.asarray(hi, dtype=np.float64).reshape(-1)[:dim]
    return lo, hi


def build_qp(A, B, C, Q, R, horizon, x0, x_ref, rows, input_constraints=None,
             position_constraints=None):
    """Assemble the full-space QP (sparse matrices).

    ``rows``: list over halfspace steps k (k = t-1) of arrays ``[O_k, 3]`` = (h0, h1, g); step k
    constrains ``x_{k+1}`` (``core/mpc_filter.py:117-121``); steps k >= horizon are ignored.
    Returns dict(P, q, E, e, G, d, layout).
    """
    A, B, C, Q, R = (np.asarray(m, dtype=np.float64) for m in (A, B, C, Q, R))
    nx, nu, ny, H = A.shape[0], B.shape[1], C.shape[0], int(horizon)
    x0 = np.asarray(x0, dtype=np.float64).reshape(nx)
    x_ref = np.asarray(x_ref, dtype=np.float64)
    hs = []
    for k in range(min(len(rows), H)):
        for h0, h1, g in np.asarray(rows[k], dtype=np.float64).reshape(-1, 3):
            hs.append((k + 1, h0, h1, g))
    M = len(hs)
    nX, nU = H * nx, H * nu
    nz = nX + nU + M
    ix = lambda t: (t - 1) * nx                                     # x_t, t = 1..H
    iu = lambda t: nX + t * nu                                      # u_t, t = 0..H-1
    P = sparse.lil_matrix((nz, nz))
    q = np.zeros(nz)
    for t in range(H):
        P[ix(t + 1):ix(t + 1) + nx, ix(t + 1):ix(t + 1) + nx] = 2.0 * Q
        q[ix(t + 1):ix(t + 1) + nx] = -2.0 * Q @ x_ref[t + 1]
        P[iu(t):iu(t) + nu, iu(t):iu(t) + nu] = 2.0 * R
    P = P.tocsr() + sparse.diags(np.r_[np.zeros(nX + nU), np.full(M, 2.0 * SLACK_QUADRATIC)])
    q[nX + nU:] = SLACK_LINEAR
    E = sparse.lil_matrix((nX, nz))
    e = np.zeros(nX)
    for t in range(H):
        r0 = t * nx
        E[r0:r0 + nx, ix(t + 1):ix(t + 1) + nx] = np.eye(nx)
        E[r0:r0 + nx, iu(t):iu(t) + nu] = -B
        if t == 0:
            e[r0:r0 + nx] = A @ x0
        else:
            E[r0:r0 + nx, ix(t):ix(t) + nx] = -A
    Gr, Gc, Gv, d = [], [], [], []

    def add_row(cols, vals, rhs):
        r = len(d)
        Gr.extend([r] * len(cols))
        Gc.extend(cols)
        Gv.extend(vals)
        d.append(rhs)

    ib = _bounds(input_constraints, nu)
    if ib is not None:
        for t in range(H):
            for i in range(nu):
                add_row([iu(t) + i], [1.0], ib[1][i])
                add_row([iu(t) + i], [-1.0], -ib[0][i])
    pb = _bounds(position_constraints, ny)
    if pb is not None:
        for t in range(1, H + 1):
            for i in range(ny):
                cols = list(range(ix(t), ix(t) + nx))
                add_row(cols, list(C[i]), pb[1][i])
                add_row(cols, list(-C[i]), -pb[0][i])
    for r, (t, h0, h1, g) in enumerate(hs):
        cols = list(range(ix(t), ix(t) + nx)) + [nX + nU + r]
        add_row(cols, list(h0 * C[0] + h1 * C[1]) + [-1.0], -g)
        add_row([nX + nU + r], [-1.0], 0.0)
    G = sparse.csr_matrix((Gv, (Gr, Gc)), shape=(len(d), nz))
    d = np.array(d, dtype=np.float64)
    return {"P": P.tocsr(), "q": q, "E": E.tocsr(), "e": e, "G": G, "d": d,
            "layout": {"nx": nx, "nu": nu, "H": H, "M": M, "nX": nX, "nU": nU}}


def solve_qp(P, q, E, e, G, d, tol=1e-11, max_iter=80, n_diag_tail=0):
    """Sparse Mehrotra predictor-corrector IPM for ``min 1/2 z'Pz + q'z, Ez = e, Gz <= d``.

    Each Newton system is the KKT matrix ``[[P + G'DG, E'], [E, 0]]`` factorised by SuperLU.  When
    the last ``n_diag_tail`` variables have a diagonal block in ``P + G'DG`` and no equality rows
    (the halfspace slacks), they are eliminated exactly first (block Gaussian elimination); without
    that, lambda/w spanning ~1e14 near the optimum costs the factorisation most of its accuracy.
    Merit = max(|r_primal|/(1+|d|), |r_dual|/(1+|q|), mean complementarity).  Converged ('optimal')
    when merit <= tol.  Near the optimum lambda/w spans ~1e14 and the full KKT factorisation loses
    accuracy, so the best iterate is kept: if the loop ends unconverged but the best merit is
    <= 1e3*tol the status is 'optimal_inaccurate' (accepted by the reference, mpc_filter.py:154).
    Returns (z, lam, nu, info).
    """
    nz, m, me = P.shape[0], G.shape[0], E.shape[0]
    z = np.zeros(nz)
    nu = np.zeros(me)
    w = np.maximum(d - G @ z, 1.0)
    lam = np.ones(m)
    scale_d = 1.0 + max(np.abs(d).max(initial=0.0), np.abs(e).max(initial=0.0))
    scale_q = 1.0 + np.abs(q).max(initial=0.0)
    GT = G.T.tocsr()
    ny_ = nz - n_diag_tail
    G = G.tocsr()
    Gy, Gs = G[:, :ny_].tocsr(), G[:, ny_:].tocsr()
    GyT, GsT = Gy.T.tocsr(), Gs.T.tocsr()
    Ey = E.tocsr()[:, :ny_]
    if E.tocsr()[:, ny_:].nnz:
        raise ValueError("eliminated variables must not appear in equality rows")
    P = P.tocsr()
    P_yy = P[:ny_, :ny_]
    if n_diag_tail:
        P_ss_block = P[ny_:, ny_:]
        p_ss = P_ss_block.diagonal()
        if (P_ss_block - sparse.diags(p_ss)).count_nonzero() or P[:ny_, ny_:].count_nonzero():
            raise ValueError("the eliminated block of P must be diagonal and uncoupled")
        Gs2T = Gs.multiply(Gs).T.tocsr()
        if np.any(np.diff(Gs.indptr) > 1):
            raise ValueError("each inequality row may touch at most one eliminated variable")
        slack_of_row = np.full(G.shape[0], -1)
        Gs_row_coef = np.zeros(G.shape[0])
        rows_with = np.repeat(np.arange(G.shape[0]), np.diff(Gs.indptr))
        slack_of_row[rows_with] = Gs.indices
        Gs_row_coef[rows_with] = Gs.data
        has_y = np.diff(Gy.indptr) > 0
        per_slack = np.bincount(slack_of_row[has_y & (slack_of_row >= 0)], minlength=n_diag_tail)
        if np.any(per_slack > 1):
            raise ValueError("each eliminated variable may couple to at most one row with a y part")
    status = "max_iter"
    best = (np.inf, z, lam, nu)
    best_it = 0
    it = 0
    for it in range(1, max_iter + 1):
        r_d = P @ z + q + GT @ lam + E.T @ nu
        r_p = G @ z + w - d
        r_e = E @ z - e
        mu = (w @ lam) / m if m else 0.0
        merit = max(max(np.abs(r_p).max(initial=0.0), np.abs(r_e).max(initial=0.0)) / scale_d,
                    np.abs(r_d).max() / scale_q, mu)
        if _TRACE:
            print(it, merit, np.abs(r_d).max(), np.abs(r_p).max(initial=0.0), mu)
        if merit < best[0]:
            best = (merit, z, lam, nu)
            best_it = it
        if merit <= tol:
            status = "optimal"
            break
        if best[0] < 1e-6 and it - best_it >= 8:   # stalled at the factorisation's accuracy floor
            break
        D = lam / w
        ny_ = nz - n_diag_tail
        if n_diag_tail:
            # slack block: k_ss = P_ss + sum_i D_i g_is^2 (diagonal); a row with both a y part and
            # a slack contributes omega_i g_iy g_iy' with omega_i = D_i (k_ss - D_i g_is^2) / k_ss,
            # formed without the cancellation of D_i - D_i^2 g_is^2 / k_ss
            kss = p_ss + Gs2T @ D
            gs_row = Gs_row_coef                    # g_is of the (single) slack of row i, or 0
            r_of = slack_of_row
            rest = kss[r_of] - D * gs_row * gs_row
            omega = np.where(r_of >= 0, D * rest / kss[np.maximum(r_of, 0)], D)
            omega = np.where(has_y, omega, 0.0)
        else:
            omega = D
        Ky = (P_yy + GyT @ sparse.diags(omega) @ Gy).tocsc()
        lu = splinalg.splu(sparse.bmat([[Ky, Ey.T], [Ey, None]], format="csc"))

        def direction(r_c):
            rho = D * r_p + r_c / w
            rz = -r_d - GT @ rho
            ry = rz[:ny_]
            if n_diag_tail:
                t = rz[ny_:] / kss
                ry = ry - GyT @ (D * (Gs @ t))
            sol = lu.solve(np.concatenate([ry, -r_e]))
            dz = np.empty(nz)
            dz[:ny_] = sol[:ny_]
            if n_diag_tail:
                dz[ny_:] = (rz[ny_:] - GsT @ (D * (Gy @ dz[:ny_]))) / kss
            dnu = sol[ny_:]
            gdz = G @ dz
            return dz, dnu, -r_p - gdz, D * gdz + rho

        def step_to_boundary(dw, dlam):
            a = 1.0
            for x, dx in ((w, dw), (lam, dlam)):
                neg = dx < 0
                if neg.any():
                    a = min(a, np.min(-x[neg] / dx[neg]))
            return a

        dz, dnu, dw, dlam = direction(-w * lam)
        a_aff = step_to_boundary(dw, dlam)
        mu_aff = ((w + a_aff * dw) @ (lam + a_aff * dlam)) / m if m else 0.0
        sigma = (mu_aff / mu) ** 3 if mu > 0 else 0.0
        dz, dnu, dw, dlam = direction(-w * lam - dw * dlam + sigma * mu)
        a = min(1.0, 0.995 * step_to_boundary(dw, dlam))
        z = z + a * dz
        nu = nu + a * dnu
        w = w + a * dw
        lam = lam + a * dlam
    if status != "optimal":
        merit, z, lam, nu = best
        if merit <= 1e3 * tol:
            status = "optimal_inaccurate"
    polished = False
    if best[0] <= 1e-4:
        w = d - G @ z
        # guesses for the active set: lambda > w; then the ambiguous rows (both small, no strict
        # complementarity) forced active, then forced inactive
        amb = np.maximum(w, lam) < 1e-2 * max(1.0, np.sqrt(best[0]) * 1e3)
        for act in (lam > w, (lam > w) | amb, (lam > w) & ~amb):
            res = _polish(P, q, E, e, G, d, act)
            if res is not None:
                z, lam, nu = res
                polished = True
                status = "optimal"
                break
        if not polished:  # degenerate instances: primal-dual active-set steps from the IPM's guess
            res = _polish_steps(P, q, E, e, G, d, lam > w)
            if res is not None:
                z, lam, nu = res
                polished = True
                status = "optimal"
    return z, lam, nu, {"status": status, "iterations": it, "merit": float(best[0]),
                        "polished": polished}


def _polish(P, q, E, e, G, d, active, feas_tol=1e-9):
    """Solve the equality-constrained QP of the guessed active set exactly (the step OSQP calls
    polishing): ``[[P, E', Ga'], [E, 0, 0], [Ga, 0, 0]] (z, nu, lam_a) = (-q, e, d_a)``.  Accepted
    only when the result is primal feasible and dual feasible; otherwise None."""
    Ga = G[active]
    nz, me, ma = P.shape[0], E.shape[0], Ga.shape[0]
    K = sparse.bmat([[P, E.T, Ga.T], [E, None, None], [Ga, None, None]], format="csc")
    try:
        sol = splinalg.spsolve(K, np.concatenate([-q, e, d[active]]))
    except RuntimeError:
        return None
    if not np.all(np.isfinite(sol)):
        return None
    z, nu, lam_a = sol[:nz], sol[nz:nz + me], sol[nz + me:]
    if np.any(G @ z - d > feas_tol * (1.0 + np.abs(d).max(initial=0.0))) or np.any(lam_a < -feas_tol):
        return None
    lam = np.zeros(G.shape[0])
    lam[active] = np.maximum(lam_a, 0.0)
    return z, lam, nu


def _polish_steps(P, q, E, e, G, d, active, max_steps=40, feas_tol=1e-9):
    """Active-set refinement when the guessed sets fail: solve the equality QP of the set, then
    add the most violated inactive row or drop the active row with the most negative multiplier,
    one row per step (a degenerate problem — more binding rows at a step than inputs — makes
    moving every violated row at once cycle).  Returns (z, lam, nu) of the first set whose
    solution is primal and dual feasible, else None."""
    active = np.array(active, dtype=bool)
    nz, me = P.shape[0], E.shape[0]
    scale = 1.0 + np.abs(d).max(initial=0.0)
    for _ in range(max_steps):
        Ga = G[active]
        K = sparse.bmat([[P, E.T, Ga.T], [E, None, None], [Ga, None, None]], format="csc")
        try:
            sol = splinalg.spsolve(K, np.concatenate([-q, e, d[active]]))
        except RuntimeError:
            return None
        if not np.all(np.isfinite(sol)):
            return None
        z, nu, lam_a = sol[:nz], sol[nz:nz + me], sol[nz + me:]
        viol = G @ z - d
        viol[active] = -np.inf
        worst_p = int(np.argmax(viol)) if viol.size else -1
        worst_d = int(np.argmin(lam_a)) if lam_a.size else -1
        p_bad = worst_p >= 0 and viol[worst_p] > feas_tol * scale
        d_bad = worst_d >= 0 and lam_a[worst_d] < -feas_tol
        if not p_bad and not d_bad:
            lam = np.zeros(G.shape[0])
            lam[active] = np.maximum(lam_a, 0.0)
            return z, lam, nu
        if p_bad:
            active[worst_p] = True
        else:
            active[np.flatnonzero(active)[worst_d]] = False
    return None


def kkt_residuals(qp, z, lam, nu):
    """Max-norm KKT residuals (stationarity, equality, inequality, complementarity, dual sign)."""
    P, q, E, e, G, d = (qp[k] for k in ("P", "q", "E", "e", "G", "d"))
    slack = d - G @ z
    return {
        "stationarity": float(np.abs(P @ z + q + G.T @ lam + E.T @ nu).max()),
        "equality": float(np.abs(E @ z - e).max(initial=0.0)),
        "inequality": float(max(0.0, -slack.min(initial=0.0))),
        "complementarity": float(np.abs(slack * lam).max(initial=0.0)),
        "dual_sign": float(max(0.0, -lam.min(initial=0.0))),
    }


def objective(Q, R, x, u, x_ref, slacks):
    """The reference objective (``core/mpc_filter.py:64-76,142-144``) at a trajectory."""
    val = 0.0
    for t in range(u.shape[0]):
        err = x[t + 1] - x_ref[t + 1]
        val += err @ Q @ err + u[t] @ R @ u[t]
    return val + float(np.sum(SLACK_LINEAR * slacks + SLACK_QUADRATIC * slacks ** 2))


def filter_trajectory(A, B, C, Q, R, horizon, x0, x_ref, u_ref, rows, input_constraints=None,
                      position_constraints=None, last_optimal_u=None, tol=1e-11):
    """Oracle ``MPCSafetyFilter.filter_trajectory`` -> (x [H+1,nx], u [H,nu], info).

    ``info`` carries the multipliers and the KKT residuals of the full-space problem.
    """
    A, B = np.asarray(A, dtype=np.float64), np.asarray(B, dtype=np.float64)
    qp = build_qp(A, B, C, Q, R, horizon, x0, x_ref, rows, input_constraints, position_constraints)
    L = qp["layout"]
    z, lam, nu, info = solve_qp(qp["P"], qp["q"], qp["E"], qp["e"], qp["G"], qp["d"], tol=tol,
                                n_diag_tail=L["M"])
    H, nx, nu_ = L["H"], L["nx"], L["nu"]
    x0 = np.asarray(x0, dtype=np.float64).reshape(nx)
    if info["status"] in ("optimal", "optimal_inaccurate"):   # core/mpc_filter.py:154
        x = np.vstack([x0, z[:L["nX"]].reshape(H, nx)])
        u = z[L["nX"]:L["nX"] + L["nU"]].reshape(H, nu_)
        s = z[L["nX"] + L["nU"]:]
        info.update(kkt=kkt_residuals(qp, z, lam, nu), slacks=s,
                    objective=objective(np.asarray(Q, float), np.asarray(R, float), x, u,
                                        np.asarray(x_ref, float), s))
        return x, u, info
    u = fallback_inputs(H, nu_, np.asarray(u_ref, dtype=np.float64), last_optimal_u)
    x = rollout(A, B, x0, u)
    info["used_fallback"] = True
    return x, u, info


def fallback_inputs(H, nu, u_ref, last_optimal_u):
    """``_fallback`` input sequence (``core/mpc_filter.py:197-210``)."""
    if last_optimal_u is None:
        return np.array(u_ref, dtype=np.float64, copy=True)
    u = np.zeros((H, nu))
    remaining = min(H - 1, len(last_optimal_u) - 1)
    u[:remaining] = last_optimal_u[1:remaining + 1]
    if remaining < H:
        u[remaining:] = u_ref[remaining:]
    return u


def rollout(A, B, x0, u):
    """``x_{t+1} = A x_t + B u_t`` from ``x0`` (``core/mpc_filter.py:212-217``)."""
    x = np.zeros((u.shape[0] + 1, A.shape[0]))
    x[0] = x0
    for t in range(u.shape[0]):
        x[t + 1] = A @ x[t] + B @ u[t]
    return x
