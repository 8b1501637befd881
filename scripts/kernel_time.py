#!/usr/bin/env python3
"""Record the kernel time of the metric line's kernel from profiles of bench.py's own command, so
that bench.py's `roofline` carries a frac that follows from committed evidence:

  busy   a `rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE --kernel-trace` pass: per dispatch of the
         kernel, its window (End - Start) times GRBM_GUI_ACTIVE / GRBM_COUNT — the time the GPU was
         busy inside the window (both counters are summed over the same XCDs, so the clock cancels);
  trace  a plain `rocprofv3 --kernel-trace` run: the mean dispatch window (the profiler's completion
         handling stretches back-to-back graph dispatches, so this is an upper bound).

The entry is keyed by the halfspace unit's source key (_native.source_key): bench.py uses it only
while the kernel sources still match and the command is the one profiled.

    python scripts/kernel_time.py c3 --pmc-dir <dir> --trace <kernel_trace.csv> \\
        --kernel 'safe_halfspace_kernel<256, 4, 9, 1, false>' --command '...' --store <profiles/...>
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def busy_times(pmc_dir, kernel):
    win, cnt = {}, {}
    for f in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel not in r.get("Kernel_Name", ""):
                continue
            d = r["Dispatch_Id"]
            win[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            cnt.setdefault(d, {})[r["Counter_Name"]] = cnt.get(d, {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = []
    for d, w in win.items():
        c = cnt[d]
        if c.get("GRBM_COUNT"):
            out.append((w, w * c["GRBM_GUI_ACTIVE"] / c["GRBM_COUNT"], c["GRBM_GUI_ACTIVE"] / c["GRBM_COUNT"]))
    return out


def trace_times(trace, kernel):
    return [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            for r in csv.DictReader(open(trace)) if kernel in r.get("Kernel_Name", "")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload")
    ap.add_argument("--pmc-dir", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--command", required=True)
    ap.add_argument("--pmc-file", required=True, help="committed copy of the counter CSV")
    ap.add_argument("--trace-file", required=True, help="committed copy of the trace / stats")
    a = ap.parse_args()
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native
    b = busy_times(a.pmc_dir, a.kernel)
    t = trace_times(a.trace, a.kernel)
    if not b or not t:
        raise SystemExit(f"no dispatch of {a.kernel!r}")
    entry = {
        "kernel": a.kernel, "command": a.command, "source_key": _native.source_key(),
        "busy": {"file": a.pmc_file, "dispatches": len(b), "mean_ns": statistics.fmean(x[1] for x in b),
                 "median_ns": statistics.median(x[1] for x in b), "window_mean_ns": statistics.fmean(x[0] for x in b),
                 "gui_active_over_count_mean": statistics.fmean(x[2] for x in b),
                 "method": ("per dispatch of a --pmc pass (dispatches serialised, none overlapped by the "
                            "profiler's completion handling of graph replays): (End - Start) x "
                            "GRBM_GUI_ACTIVE / GRBM_COUNT; a ratio of 1 makes it the dispatch window")},
        "trace": {"file": a.trace_file, "dispatches": len(t), "mean_ns": statistics.fmean(t),
                  "median_ns": statistics.median(t), "min_ns": min(t),
                  "method": "rocprofv3 --kernel-trace dispatch windows (stretched by the profiler)"}}
    path = os.path.join(REPO, "profiles", "kernel_time.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    data[a.workload] = entry
    with open(path, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(a.workload, json.dumps(entry))


if __name__ == "__main__":
    main()
