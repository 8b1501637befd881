#!/usr/bin/env python3
"""Per-kernel VGPR / scratch usage from a device assembly file (hipcc --cuda-device-only -S):
    python3 scripts/isa_resources.py /tmp/mpc.s"""
import re
import sys

txt = open(sys.argv[1]).read()
for block in re.split(r"\n\s+- \.", txt.split("amdhsa.kernels:")[-1])[1:]:
    name = re.search(r"\.name:\s+(\S+)", block)
    vg = re.search(r"\.vgpr_count:\s+(\d+)", block)
    sc = re.search(r"\.private_segment_fixed_size:\s+(\d+)", block)
    lds = re.search(r"\.group_segment_fixed_size:\s+(\d+)", block)
    if name:
        print(f"{name.group(1)[:90]:90s} vgpr {vg.group(1) if vg else '?':>4s} scratch "
              f"{sc.group(1) if sc else '?':>4s} lds {lds.group(1) if lds else '?'}")
