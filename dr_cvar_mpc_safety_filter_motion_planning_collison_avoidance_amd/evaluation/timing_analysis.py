"""``evaluation/timing_analysis.py`` counterpart: the reference's timing harness on the HIP engine.

Reference: ``analyze_dr_cvar_computation_time`` (``evaluation/timing_analysis.py:13-132``),
``plot_timing_results`` (``:134-226``), ``create_comparison_table`` (``:228-275``).

:func:`analyze_dr_cvar_computation_time` keeps the reference's protocol: for every sample size and
run it draws the same per-element normal samples in the same order (``:63-68``, so a seeded run
reproduces the reference's inputs), times one ``DRCVaRSafeHalfspace.create`` and one
``CVaRSafeHalfspace.create`` call (``:73-77``, ``:100-104``), reads the setup / solve split back from
``tmp/timing_info_{drcvar,cvar}.json`` (``:84-93``, ``:111-119``) and writes the same
``timing_comparison.csv`` columns (``:256-266``).  Per call these numbers are dominated by the
host<->device round trip of one unit; :func:`analyze_batched_computation_time` adds what the engine
is for — every size evaluated as a device-resident batch, timed with HIP events — and writes
``timing_batched.csv``.
"""
from __future__ import annotations

import json
import os
import time

import numpy as np
import torch

from .. import engine
from ..core import risk_metrics
from ..core.halfspaces import CVaRSafeHalfspace, DRCVaRSafeHalfspace
from ..engine import RiskParams

# config/parameters.py:11-16,29
ALPHA, DELTA, EPSILON, ROBOT_RADIUS, OBSTACLE_RADIUS = 0.2, 0.1, 0.15, 0.3, 0.3
COLUMNS = ["Samples", "DR-CVaR Setup", "DR-CVaR Solve", "DR-CVaR Call", "CVaR Setup", "CVaR Solve",
           "CVaR Call"]                                          # timing_analysis.py:259-265


def draw_samples(n_samples):
    """One run's obstacle samples, drawn element by element as the reference does (:63-68)."""
    mean_pos = np.array([0.5, 0.0])
    scale = np.array([0.1, 0.1])
    samples = np.zeros((n_samples, 2))
    for i in range(n_samples):
        samples[i, 0] = np.random.normal(mean_pos[0], scale[0])
        samples[i, 1] = np.random.normal(mean_pos[1], scale[1])
    return samples


def _read_ms(path):
    try:
        with open(path) as f:
            info = json.load(f)
        return info.get("setup_time", 0) * 1000, info.get("solve_time", 0) * 1000
    except (OSError, ValueError):
        return 0.0, 0.0


def analyze_dr_cvar_computation_time(sample_sizes=(10, 50, 100, 500, 1000, 1500), n_runs=50,
                                     save_dir=None, keep_halfspaces=False):
    """Per-call timing of the create() factories (reference protocol, :13-132).

    Returns the reference's ``timing_data`` dict (ms); with ``keep_halfspaces`` also a list of
    ``(n_samples, samples, dr_halfspace, cvar_halfspace)`` per run.
    """
    sample_sizes = list(sample_sizes)
    if save_dir and not os.path.exists(save_dir):
        os.makedirs(save_dir)
    timing_data = {key: {n: [] for n in sample_sizes}
                   for key in ("setup_times", "solve_times", "call_times", "cvar_setup_times",
                               "cvar_solve_times", "cvar_call_times")}
    os.makedirs("tmp", exist_ok=True)                             # :44-49
    for key in ("drcvar", "cvar"):
        if os.path.exists(f"tmp/timing_info_{key}.json"):
            os.remove(f"tmp/timing_info_{key}.json")
    kept = []
    ego_ref_pos = np.array([0.0, 0.0])
    for n_samples in sample_sizes:
        print(f"Testing with {n_samples} samples...")
        for run in range(n_runs):
            if run % 10 == 0 and run > 0:
                print(f"  Run {run}/{n_runs}")
            samples = draw_samples(n_samples)
            t0 = time.time()
            dr = DRCVaRSafeHalfspace.create(samples, ego_ref_pos, ALPHA, DELTA, EPSILON,
                                            ROBOT_RADIUS, OBSTACLE_RADIUS)
            call_ms = (time.time() - t0) * 1000
            setup_ms, solve_ms = _read_ms("tmp/timing_info_drcvar.json")
            timing_data["setup_times"][n_samples].append(setup_ms)
            timing_data["solve_times"][n_samples].append(solve_ms)
            timing_data["call_times"][n_samples].append(call_ms)
            t0 = time.time()
            cv = CVaRSafeHalfspace.create(samples, ego_ref_pos, ALPHA, DELTA, ROBOT_RADIUS,
                                          OBSTACLE_RADIUS)
            call_ms = (time.time() - t0) * 1000
            setup_ms, solve_ms = _read_ms("tmp/timing_info_cvar.json")
            timing_data["cvar_setup_times"][n_samples].append(setup_ms)
            timing_data["cvar_solve_times"][n_samples].append(solve_ms)
            timing_data["cvar_call_times"][n_samples].append(call_ms)
            if keep_halfspaces:
                kept.append((n_samples, samples, dr, cv))
    plot_timing_results(timing_data, sample_sizes, save_dir)
    create_comparison_table(timing_data, sample_sizes, save_dir)
    return (timing_data, kept) if keep_halfspaces else timing_data


def plot_timing_results(timing_data, sample_sizes, save_dir=None):
    """Box plots of setup / solve / call time per sample size (:134-226), outliers above the
    reference's thresholds (2 / 100 / 400 ms) filtered in the first figure.  Skipped silently when
    matplotlib is not importable or nothing is to be saved."""
    if not save_dir:
        return
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        return
    keys = ("setup_times", "solve_times", "call_times")
    limits = (2.0, 100.0, 400.0)
    for name, filtered in (("dr_cvar_computation_time.png", True),
                           ("dr_cvar_computation_time_with_outliers.png", False)):
        fig, axs = plt.subplots(3, 1, figsize=(10, 12))
        for ax, key, lim, title in zip(axs, keys, limits, ("Setup Time", "Solve Time", "Call Time")):
            data = [np.asarray(timing_data[key][n]) for n in sample_sizes]
            if filtered:
                data = [d[d < lim] for d in data]
                title = f"{title} (outliers > {lim:g}ms removed)"
            else:
                title = f"{title} (with outliers)"
            ax.boxplot(data, tick_labels=sample_sizes)
            ax.set_title(title)
            ax.set_ylabel("Time (ms)")
        axs[2].set_xlabel("Number Samples")
        fig.tight_layout()
        fig.savefig(os.path.join(save_dir, name))
        plt.close(fig)


def create_comparison_table(timing_data, sample_sizes, save_dir=None):
    """Mean times per sample size with the reference's columns (:228-275)."""
    import pandas as pd
    rows = []
    for n in sample_sizes:
        rows.append([n] + [float(np.mean(timing_data[k][n])) for k in (
            "setup_times", "solve_times", "call_times", "cvar_setup_times", "cvar_solve_times",
            "cvar_call_times")])
    df = pd.DataFrame(rows, columns=COLUMNS)
    print("\nTiming Comparison (times in ms):")
    print(df.to_string(index=False))
    if save_dir:
        df.to_csv(os.path.join(save_dir, "timing_comparison.csv"), index=False)
    return df


def analyze_batched_computation_time(sample_sizes=(10, 50, 100, 500, 1000, 1500), n_units=4096,
                                     reps=20, save_dir=None, seed=0):
    """Device-resident batches: ``n_units`` units of each size in ONE launch, HIP-event timed.

    Units follow the same distribution as :func:`draw_samples` (mean (0.5, 0), sigma 0.1, ego at
    the origin).  Returns a DataFrame with the per-halfspace time of a batched launch (both
    metrics come out of the same launch) and writes ``timing_batched.csv``.
    """
    import pandas as pd
    dev = risk_metrics.device()
    params = RiskParams(ROBOT_RADIUS, OBSTACLE_RADIUS, ALPHA, DELTA, EPSILON)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    rows = []
    for n in sample_sizes:
        samples = torch.randn((n_units, 1, n, 2), dtype=torch.float64, device=dev, generator=gen) * 0.1
        samples[..., 0] += 0.5
        ego = torch.zeros((1, 2), dtype=torch.float64, device=dev)
        launch, out = engine.prepare_safe_halfspaces(samples, ego, params)
        launch()
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            launch()
        b.record()
        torch.cuda.synchronize(dev)
        ms = a.elapsed_time(b) / reps
        rows.append([n, n_units, ms, ms * 1000.0 / n_units, n_units / (ms * 1e-3)])
        del samples, out
    df = pd.DataFrame(rows, columns=["Samples", "Units", "Launch ms", "Per-halfspace us",
                                     "Halfspaces/s"])
    print("\nBatched device timing:")
    print(df.to_string(index=False))
    if save_dir:
        os.makedirs(save_dir, exist_ok=True)
        df.to_csv(os.path.join(save_dir, "timing_batched.csv"), index=False)
    return df


__all__ = ["analyze_dr_cvar_computation_time", "analyze_batched_computation_time",
           "plot_timing_results", "create_comparison_table", "draw_samples"]
