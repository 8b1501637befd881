#!/usr/bin/env python3
"""Write-bandwidth floor next to the sampler: torch fill_ and copy_ on the C5-sized 2.05 GB
buffer, then the sampler refill with the product library and with DRCVAR_DIAG_LIB variants."""
import ctypes, os, subprocess, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import diaglib  # noqa: E402
diaglib.apply()  # DRCVAR_DIAG_LIB: a variant build (diagnostics)
dev = torch.device("cuda", 0)
out = torch.empty((256, 50, 10000, 2), dtype=torch.float64, device=dev)
src = torch.empty_like(out)
def t(fn, reps=10):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps
n = out.numel() * 8
ms = t(lambda: out.fill_(1.0)); print(f"fill_  {ms:.3f} ms {n / ms / 1e9:.2f} TB/s", flush=True)
ms = t(lambda: out.copy_(src)); print(f"copy_  {ms:.3f} ms {2 * n / ms / 1e9:.2f} TB/s (read+write)", flush=True)
