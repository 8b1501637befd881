#!/usr/bin/env python3
"""Record the rocprofv3 kernel-trace time of the metric line's kernel so that bench.py's `roofline`
can carry a frac that follows from a committed profile.

Reads a `--kernel-trace` CSV (one row per dispatch: Kernel_Name, Start_Timestamp, End_Timestamp) of
`bench.py` run with the given command, keeps the dispatches of the kernel whose name contains
`--kernel`, and stores mean / median / min durations under the workload in
profiles/rocprof_kernel_time.json:

    python scripts/rocprof_kernel_time.py c3 <kernel_trace.csv> --kernel 'safe_halfspace_kernel<256, 4, 9, 1, false>' \
        --command 'python3 bench.py --gpus 1 --steps 20 --warmup 5' --file profiles/r04/...csv
"""
import argparse
import csv
import json
import os
import statistics

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def durations(trace, kernel):
    out = []
    for r in csv.DictReader(open(trace)):
        if kernel in r.get("Kernel_Name", ""):
            out.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload")
    ap.add_argument("trace")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--command", required=True)
    ap.add_argument("--file", help="committed path of the trace / stats (defaults to the trace)")
    a = ap.parse_args()
    d = durations(a.trace, a.kernel)
    if not d:
        raise SystemExit(f"no dispatch of {a.kernel!r} in {a.trace}")
    path = os.path.join(REPO, "profiles", "rocprof_kernel_time.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    entry = {"kernel": a.kernel, "command": a.command, "file": a.file or os.path.relpath(a.trace, REPO),
             "dispatches": len(d), "mean_ns": statistics.fmean(d), "median_ns": statistics.median(d),
             "min_ns": min(d), "max_ns": max(d)}
    data[a.workload] = entry
    with open(path, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(a.workload, json.dumps(entry))


if __name__ == "__main__":
    main()
