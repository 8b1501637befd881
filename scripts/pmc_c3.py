#!/usr/bin/env python3
"""Summarise scripts/gpu_c3_pmc.sh: mean counters per dispatch of the C3 halfspace kernel
(safe_halfspace_kernel<256, 4, 9, 1, false>) and the wave-time split they imply.

    python3 scripts/pmc_c3.py gpurun_out/c3pmc   ->  profiles/r02/c3_latency_pmc.json
"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "safe_halfspace_kernel<256, 4, 9, 1, false>"


def main():
    d = sys.argv[1]
    per = {}  # counter -> {dispatch: value}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL not in r.get("Kernel_Name", ""):
                continue
            key = (f, r["Dispatch_Id"])
            c = per.setdefault(r["Counter_Name"], {})
            c[key] = c.get(key, 0.0) + float(r["Counter_Value"])
    mean = {k: sum(v.values()) / len(v) for k, v in per.items() if v}
    out = {"kernel": KERNEL + " (C3: 10 obstacles x 20 steps x 1000 samples, 200 workgroups)",
           "dispatches": {k: len(v) for k, v in per.items()},
           "counters_mean_per_dispatch": mean}
    wc = mean.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if k in mean:
                out[f"{k}_per_wave_cycle"] = mean[k] / wc
    if mean.get("SQ_WAVES"):
        out["wave_cycles_per_wave"] = (wc or 0.0) / mean["SQ_WAVES"]
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"):
            if k in mean:
                out[f"{k}_per_wave"] = mean[k] / mean["SQ_WAVES"]
    path = os.path.join(REPO, "profiles", "r02", "c3_latency_pmc.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
