#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch of the
safe-halfspace kernel, with the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB)
reports half the bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is exact
for 16-B-per-lane stores.  Writes/updates profiles/pmc_traffic.json.

    python scripts/pmc_traffic.py <workload> <fetch_dir> <write_dir>
"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter_mean(d, name):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "safe_halfspace_kernel" not in r.get("Kernel_Name", ""):
                continue
            if r.get("Counter_Name") != name:
                continue
            key = r.get("Dispatch_Id")
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        return None, 0
    return sum(vals.values()) / len(vals), len(vals)


def main():
    workload, fetch_dir, write_dir = sys.argv[1:4]
    fetch_kb, nf = counter_mean(fetch_dir, "FETCH_SIZE")
    write_kb, nw = counter_mean(write_dir, "WRITE_SIZE")
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    entry = {"fetch_size_kb_raw": fetch_kb, "write_size_kb_raw": write_kb,
             "dispatches": [nf, nw],
             "correction": "FETCH_SIZE x 2 (gfx950 half-count on wide streaming reads), WRITE_SIZE x 1; KB = 1024 B"}
    if fetch_kb is not None and write_kb is not None:
        entry["hbm_bytes_per_launch"] = fetch_kb * 1024 * 2 + write_kb * 1024
    data[workload] = entry
    with open(path, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(workload, json.dumps(entry))


if __name__ == "__main__":
    main()
