"""K=256 SYRK n=7680 steady state: beta=0 (no C read) vs the Cholesky-update form C -= X^T X
(accumulators start from the C tile).   python scripts/syrk_cinit.py"""
import sys
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import torch
from gpu_util import handle
from ipm355 import _lib as L
h = handle()
n, k = 7680, 256
X = torch.rand(k, n, dtype=torch.float64, device="cuda")
H = torch.zeros(n, n, dtype=torch.float64, device="cuda")
def run(reps, alpha, beta):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        h.lib.ipm_syrk(h.ptr, n, k, L.dptr(X), n, None, alpha, beta, L.dptr(H), n)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps
run(20, 1.0, 0.0)
for _ in range(2):
    print(f"beta=0:            {run(50, 1.0, 0.0)*1e3:.1f} us", flush=True)
    print(f"C -= X^T X (cinit): {run(50, -1.0, 1.0)*1e3:.1f} us", flush=True)
