"""``core/risk_metrics.py`` surface, evaluated by the HIP engine instead of CVXPY/ECOS.

Reference: ``core/risk_metrics.py`` — ``DRCVaROptimizer`` (:84-177), ``CVaROptimizer`` (:179-265),
``dr_cvar_halfspace`` (:267-303), ``cvar_halfspace`` (:305-338), ``save_timing_info`` (:16-33).

The optimiser classes keep their names and ``solve(h, samples, combined_radius) -> (solved, g, info)``
contract, but there is no LP to build: the GPU kernel evaluates the LP optimum in closed form
(derivation in DESIGN.md §2).  Behaviour kept on purpose:

* module-level optimiser singletons keyed on ``n_samples`` only (:12-13, :289, :325) — like the
  reference, ``dr_cvar_halfspace`` / ``cvar_halfspace`` keep the alpha/delta/epsilon of the first
  call for a given N, and so do the batched ``compute_safe_halfspaces`` and
  ``SafetyFilteringEnvironment`` paths (:func:`singleton_params`); call :func:`reset_optimizers`
  to drop them;
* ``tmp/timing_info_{drcvar,cvar}.json`` side channel with ``setup_time`` / ``solve_time`` seconds
  (:16-33), which ``core/halfspaces.py`` and ``evaluation/timing_analysis.py`` read back;
* solver-failure sentinels (:173-177, :261-265, :298-303, :334-338): ``g = 100.0`` and
  ``g_tilde = 100.0 - R_c|h|`` when the samples are not finite (or their sums overflow) or the LP
  is unbounded (alpha > 1; epsilon < 0 for DR-CVaR).  Failure is what the kernel reports in its
  per-unit status word (``_native.UNIT_*``), never inferred from the sentinel's value.

``RiskMetric`` is the batched evaluator named by the build's north star (no such class exists in
the reference): one object per metric, ``evaluate(samples [O,T,N,2], ego [T,2])`` on device tensors.
"""
from __future__ import annotations

import json
import os
import time

import numpy as np
import torch

from .. import _native, engine
from ..engine import RiskParams

# For storing optimizer instances (reference :12-13)
drcvar_optimizer = None
cvar_optimizer = None

#: write tmp/timing_info_*.json after every per-unit solve, as the reference does (:16-33)
WRITE_TIMING_FILES = True


def save_timing_info(key, setup_time, solve_time):
    """Write ``tmp/timing_info_{key}.json`` (cwd-relative) with setup/solve seconds (:16-33)."""
    os.makedirs("tmp", exist_ok=True)
    with open(f"tmp/timing_info_{key}.json", "w") as f:
        json.dump({"setup_time": setup_time, "solve_time": solve_time}, f)


def device() -> torch.device:
    """The HIP device the engine runs on (the current torch device); raises if there is none."""
    if not torch.cuda.is_available():
        raise _native.NativeLibraryError(
            "no HIP device is visible: the DR-CVaR engine runs only on the GPU (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


_CVAR_FAILED = _native.UNIT_NONFINITE | _native.UNIT_UNBOUNDED
_DR_FAILED = _CVAR_FAILED | _native.UNIT_DR_UNBOUNDED


def failure_status(bits: int, dr: bool) -> str | None:
    """The LP status name the reference would print for a unit's status bits, or None if solved
    (ECOS reports an unbounded LP as dual infeasible and non-finite data as an error)."""
    if bits & _native.UNIT_NONFINITE:
        return "solver_error"
    if bits & _native.UNIT_UNBOUNDED or (dr and bits & _native.UNIT_DR_UNBOUNDED):
        return "unbounded"
    return None


def _stage_unit(h, samples, dev):
    s = torch.as_tensor(np.ascontiguousarray(samples, dtype=np.float64)).to(dev)
    hh = torch.as_tensor(np.ascontiguousarray(np.asarray(h, dtype=np.float64).reshape(1, 2))).to(dev)
    return s.reshape(1, -1, 2), hh


class _UnitOptimizer:
    """Shared machinery of the two optimiser classes: one unit through ``offsets_given_h``."""

    key = ""

    def __init__(self, alpha, epsilon, delta, max_samples):
        self.alpha = alpha
        self.epsilon = epsilon
        self.delta = delta
        self.n_samples = max_samples
        RiskParams(0.0, 0.0, alpha, delta, epsilon).validate()

    def _run(self, h, samples, rc):
        setup_start = time.time()
        dev = device()
        s, hh = _stage_unit(h, samples, dev)
        setup_time = time.time() - setup_start
        solve_start = time.time()
        st = torch.empty(1, dtype=torch.int32, device=dev)
        out = engine.offsets_given_h(s, hh, RiskParams(rc, 0.0, self.alpha, self.delta, self.epsilon),
                                     status=st)
        rec = out[0].cpu().numpy()
        bits = int(st[0])
        solve_time = time.time() - solve_start
        info = {"setup_time": setup_time, "solve_time": solve_time,
                "solve_call_time": setup_time + solve_time}
        if WRITE_TIMING_FILES:
            save_timing_info(self.key, setup_time, solve_time)
        return rec, bits, info


class DRCVaROptimizer(_UnitOptimizer):
    """``DRCVaROptimizer`` (:84-177): ``solve(h, samples, combined_radius)`` -> (solved, g*, info),
    where ``combined_radius`` is already ``R_c*|h|`` (:293)."""

    key = "drcvar"

    def __init__(self, alpha, epsilon, delta, max_samples):
        super().__init__(alpha, epsilon, delta, max_samples)

    def solve(self, h, samples, combined_radius):
        # kernel with zero radius gives g*(r=0); the LP optimum is affine in r with slope 1 (:113-119)
        rec, bits, info = self._run(h, samples, 0.0)
        failed = failure_status(bits, dr=True)
        if failed:                                                   # :173-177
            print(f"Warning: DR-CVaR optimization failed with status: {failed}")
            return False, 100.0, info
        return True, float(combined_radius) + float(rec[_native.COL_G_DR_STAR]), info


class CVaROptimizer(_UnitOptimizer):
    """``CVaROptimizer`` (:179-265): ``solve(h, samples, combined_radius)`` -> (solved, g, info),
    where ``combined_radius`` is ``R_c`` and the LP uses ``R_c*|h|`` (:234)."""

    key = "cvar"

    def __init__(self, alpha, delta, max_samples):
        super().__init__(alpha, 0.0, delta, max_samples)

    def solve(self, h, samples, combined_radius):
        rec, bits, info = self._run(h, samples, float(combined_radius))
        failed = failure_status(bits, dr=False)
        if failed:                                                   # :261-265
            print(f"Warning: CVaR optimization failed with status: {failed}")
            return False, 100.0, info
        return True, float(rec[_native.COL_G_CVAR]), info


def dr_cvar_halfspace(samples, h, alpha, delta, epsilon, robot_radius, obstacle_radius):
    """DR-CVaR offset for one unit with direction ``h`` (:267-303). Returns ``(g_star, g_tilde)``."""
    global drcvar_optimizer
    if drcvar_optimizer is None or drcvar_optimizer.n_samples != len(samples):
        drcvar_optimizer = DRCVaROptimizer(alpha, epsilon, delta, len(samples))
    combined_radius = (robot_radius + obstacle_radius) * np.linalg.norm(h)
    solved, g_star, _ = drcvar_optimizer.solve(h, samples, combined_radius)
    if solved:
        return g_star, g_star - combined_radius
    return 100.0, 100.0 - combined_radius


def cvar_halfspace(samples, h, alpha, delta, robot_radius, obstacle_radius):
    """CVaR offset for one unit with direction ``h`` (:305-338). Returns ``g``."""
    global cvar_optimizer
    if cvar_optimizer is None or cvar_optimizer.n_samples != len(samples):
        cvar_optimizer = CVaROptimizer(alpha, delta, len(samples))
    combined_radius = robot_radius + obstacle_radius
    solved, g_value, _ = cvar_optimizer.solve(h, samples, combined_radius)
    return g_value if solved else 100.0


def plan_singletons(sample_counts, alpha, delta, epsilon):
    """The parameters the reference's optimiser singletons solve each call with — without
    touching them.

    The reference reaches its LPs only through ``cvar_halfspace`` / ``dr_cvar_halfspace``, whose
    module singletons are keyed on N alone (:289, :325): a call whose N matches the live singleton
    keeps the alpha/delta(/epsilon) the singleton was built with, any other N rebuilds it with the
    call's values — CVaR and DR-CVaR independently.  ``sample_counts`` lists N for every solve in
    the reference's call order (per ``compute_safe_halfspaces`` call: obstacles in order; per
    ``compute_safe_halfspaces_for_trajectory``: steps outer, obstacles inner).  Returns
    ``(keys, final)``: per call ``((alpha_cvar, delta_cvar), (alpha_dr, delta_dr, epsilon_dr))``,
    and the singletons as those calls leave them (hand to :func:`commit_singletons` once the
    evaluation has succeeded).
    """
    dr, cv = drcvar_optimizer, cvar_optimizer
    keys = []
    for n in sample_counts:
        n = int(n)
        if dr is None or dr.n_samples != n:
            dr = DRCVaROptimizer(alpha, epsilon, delta, n)
        if cv is None or cv.n_samples != n:
            cv = CVaROptimizer(alpha, delta, n)
        keys.append(((cv.alpha, cv.delta), (dr.alpha, dr.delta, dr.epsilon)))
    return keys, (dr, cv)


def commit_singletons(final) -> None:
    """Leave the singletons as :func:`plan_singletons` computed (after the launches succeeded)."""
    global drcvar_optimizer, cvar_optimizer
    drcvar_optimizer, cvar_optimizer = final


def singleton_params(sample_counts, alpha, delta, epsilon):
    """:func:`plan_singletons` + :func:`commit_singletons`: the per-call parameters, with the
    singletons updated exactly as the reference's calls would leave them."""
    keys, final = plan_singletons(sample_counts, alpha, delta, epsilon)
    commit_singletons(final)
    return keys


def reset_optimizers() -> None:
    """Drop the cached optimiser singletons (the reference has no equivalent)."""
    global drcvar_optimizer, cvar_optimizer
    drcvar_optimizer = None
    cvar_optimizer = None


class RiskMetric:
    """Batched safe-halfspace evaluator for one risk metric ('mean', 'cvar' or 'dr_cvar').

    ``evaluate(samples, ego)`` takes device tensors ``[O, T, N, 2]`` / ``[T, 2]`` (float64) and
    returns ``(h [O, T, 2], g [O, T])`` — the ``get_constraint_params()`` pair
    (``core/halfspaces.py:56-64``) of every unit, computed by one kernel launch.
    ``evaluate_all`` returns the full ``[O, T, 8]`` record (all three metrics at once).
    """

    _COLS = {"mean": (0, 1, 2), "cvar": (3, 4, 5), "dr_cvar": (3, 4, 7)}

    def __init__(self, kind="dr_cvar", alpha=0.2, delta=0.1, epsilon=0.15, robot_radius=0.3,
                 obstacle_radius=0.3):
        if kind not in self._COLS:
            raise ValueError(f"kind must be one of {sorted(self._COLS)}, got {kind!r}")
        self.kind = kind
        self.params = RiskParams(robot_radius, obstacle_radius, alpha, delta, epsilon)
        self.params.validate()

    def evaluate_all(self, samples: torch.Tensor, ego: torch.Tensor, out=None, stream=None):
        return engine.safe_halfspaces(samples, ego, self.params, out=out, stream=stream)

    def evaluate(self, samples: torch.Tensor, ego: torch.Tensor, stream=None):
        rec = self.evaluate_all(samples, ego, stream=stream)
        c0, c1, cg = self._COLS[self.kind]
        return rec[..., c0:c1 + 1], rec[..., cg]
