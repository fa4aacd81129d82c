"""POTRF wall time at n (median of reps, HIP events on the library's stream) + error vs torch.
Env knobs of the library (IPM_*) are read at load, so run one configuration per process."""
import ctypes, os, sys
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import torch
from gpu_util import handle
from ipm355 import _lib as L
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
lda = int(sys.argv[3]) if len(sys.argv) > 3 else n   # leading dimension (the solver's ldh: n rounded up to even)
h = handle()
torch.manual_seed(0)
M = torch.rand(n, n, dtype=torch.float64, device="cuda")
A = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
Lref = torch.linalg.cholesky(A)
ts = []
for r in range(reps + 1):
    Hb = torch.zeros(n, lda, dtype=torch.float64, device="cuda")
    Hb[:, :n] = A
    Hc = Hb[:, :n]
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    info = ctypes.c_int(0)
    s.record()
    h.lib.ipm_potrf(h.ptr, n, L.dptr(Hb), lda, ctypes.byref(info))
    e.record(); torch.cuda.synchronize()
    if r: ts.append(s.elapsed_time(e))
err = ((torch.tril(Hc.T) - Lref).norm() / Lref.norm()).item()
ts.sort()
knobs = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("IPM_"))
print(f"potrf n={n} lda={lda} [{knobs or 'default'}]: median {ts[len(ts)//2]:.3f} ms min {ts[0]:.3f} ms "
      f"{n**3/3/ts[len(ts)//2]/1e9:.1f} TF/s info={info.value} relerr={err:.1e}", flush=True)
