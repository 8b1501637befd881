#!/usr/bin/env python3
"""Summarise the counter passes of scripts/gpu_sampler_pmc.sh over sample_kernel (the device
sampler refilling a 256 x 50 x 10000 batch, 128 M samples, 2.05 GB per launch):
    python3 scripts/pmc_sampler.py gpurun_out/spmc > profiles/r02/sampler_pmc.json
Counters are rocprofv3 totals per dispatch (summed over the XCDs); GRBM_GUI_ACTIVE / 8 is the
dispatch's duration in shader cycles; SQ_ACTIVE_INST_VALU counts quad-cycles per wave."""
import collections
import csv
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/spmc"
vals = collections.defaultdict(list)
for p in ("valu", "f64", "fetch", "write"):
    for r in csv.DictReader(open(os.path.join(d, p, "run_counter_collection.csv"))):
        if "sample_kernel" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
samples = 256 * 50 * 10000
simds = 256 * 4
cycles = m["GRBM_GUI_ACTIVE"] / 8
valu_cycles = m["SQ_ACTIVE_INST_VALU"] * 4
f64 = sum(m[k] for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                         "SQ_INSTS_VALU_TRANS_F64"))
slots = samples / 64  # per-sample wave-instruction slots (64 samples share one wave instruction)
out = {
    "kernel": "sample_kernel (csrc/drcvar_sampling.hip), 128 M samples per dispatch",
    "dispatches": len(vals["SQ_WAVES"]),
    "counters_mean_per_dispatch": m,
    "dispatch_cycles": cycles,
    "valu_busy_frac": valu_cycles / (simds * cycles),
    "valu_insts_per_sample": m["SQ_INSTS_VALU"] / slots,
    "f64_insts_per_sample": f64 / slots,
    "other_valu_insts_per_sample": (m["SQ_INSTS_VALU"] - f64) / slots,
    "cycles_per_valu_inst": valu_cycles / m["SQ_INSTS_VALU"],
    "hbm_write_bytes": m["WRITE_SIZE"] * 1024,
    "hbm_fetch_bytes": m["FETCH_SIZE"] * 1024,
    "algorithmic_write_bytes": samples * 16,
    "bound": "valu",
}
json.dump(out, sys.stdout, indent=1)
print()
