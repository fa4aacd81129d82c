"""Determinism check of the fused Cholesky (a race detector): factor the SAME matrix `reps` times
and compare every factor bitwise with the first (the kernel is deterministic by construction:
fixed reduction orders, ticketed roles).  Reports mismatching runs and where they differ.
   python scripts/race_check.py n ncols lda reps     (ncols < n: the bordered phase-1 shape)"""
import ctypes, sys
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import torch
from gpu_util import handle
from ipm355 import _lib as L
n, ncols, lda, reps = (int(v) for v in sys.argv[1:5])
h = handle()
torch.manual_seed(0)
M = torch.rand(n, n, dtype=torch.float64, device="cuda") - 0.5
A = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
buf0 = torch.zeros(n, lda, dtype=torch.float64, device="cuda")
buf0[:, :n] = A
ref = None
bad = 0
for r in range(reps):
    H = buf0.clone()
    info = ctypes.c_int(-7)
    rc = h.lib.ipm_potrf_partial(h.ptr, n, ncols, L.dptr(H), lda, ctypes.byref(info))
    torch.cuda.synchronize()
    Lf = torch.tril(H[:, :n].T)[:, :ncols]   # column-major buffer: H[j, i] = L(i, j)
    if ref is None:
        ref = Lf.clone()
        print(f"n={n} ncols={ncols} lda={lda}: rc={rc} info={info.value}", flush=True)
        continue
    d = (Lf != ref)
    if bool(d.any()):
        bad += 1
        idx = d.nonzero()
        i0, j0 = int(idx[0, 0]), int(idx[0, 1])
        cols = torch.unique(idx[:, 1] // 128).tolist()
        print(f"  run {r}: {int(d.sum())} elements differ; first (row {i0}, col {j0}) "
              f"{float(Lf[i0, j0])!r} vs {float(ref[i0, j0])!r}; 128-column blocks {cols[:12]}; info={info.value}",
              flush=True)
print(f"n={n} ncols={ncols} lda={lda}: {bad} of {reps - 1} runs differ from the first", flush=True)
