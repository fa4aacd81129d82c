"""Standalone K=256 SYRK (n=7680) timed alone vs in a steady back-to-back stream of 30 launches
(clock under sustained fp64 MFMA load).   python scripts/syrk_steady.py"""
import sys
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import torch
from gpu_util import handle
from ipm355 import _lib as L
h = handle()
n, k = 7680, 256
X = torch.rand(k, n, dtype=torch.float64, device="cuda")
H = torch.zeros(n, n, dtype=torch.float64, device="cuda")
def run(reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        h.lib.ipm_syrk(h.ptr, n, k, L.dptr(X), n, None, 1.0, 0.0, L.dptr(H), n)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps
for _ in range(3):
    print(f"single: {run(1)*1e3:.1f} us", flush=True)
    torch.cuda._sleep(100000000) if hasattr(torch.cuda, "_sleep") else None
    torch.cuda.synchronize()
print(f"steady x30: {run(30)*1e3:.1f} us per launch", flush=True)
print(f"steady x100: {run(100)*1e3:.1f} us per launch", flush=True)
