"""Kernel micro-bench on the GPU box: KKT SYRK, POTRF, single-RHS POTRS at the headline size,
timed with HIP events on the library's stream (the legacy default stream == torch's), checked
against torch (rocSOLVER/hipBLAS comparators, timing only)."""
import ctypes
import sys
import time

sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gpu_util import handle  # noqa: E402
from ipm355 import _lib as L  # noqa: E402

h = handle()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
m = n // 4
torch.manual_seed(0)
dev = "cuda"


def timed(fn, reps=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return min(ts), sum(ts) / len(ts)


X = torch.rand(m, n, dtype=torch.float64, device=dev) * 4 - 2
w = torch.rand(m, dtype=torch.float64, device=dev) + 0.1
H = torch.zeros(n, n, dtype=torch.float64, device=dev)
syrk = lambda: h.lib.ipm_syrk(h.ptr, n, m, L.dptr(X), n, L.dptr(w), 1.0, 0.0, L.dptr(H), n)
tmin, tavg = timed(syrk)
fl = m * n * (n + 1)
print(f"syrk n={n} k={m}: {tmin:.3f} ms (avg {tavg:.3f})  {fl / tmin / 1e9:.1f} TF/s", flush=True)
ref = (X.T * w) @ X
err = (torch.tril(H.T) - torch.tril(ref)).abs().max().item() / ref.abs().max().item()
print(f"   max rel err vs torch {err:.1e}", flush=True)

A = ref + n * torch.eye(n, dtype=torch.float64, device=dev)
Hc = A.clone()
info = ctypes.c_int(0)
potrf = lambda: (Hc.copy_(A), h.lib.ipm_potrf(h.ptr, n, L.dptr(Hc), n, ctypes.byref(info)))
# time the factorisation alone: copy outside the events
ts = []
for r in range(4):
    Hc.copy_(A)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h.lib.ipm_potrf(h.ptr, n, L.dptr(Hc), n, ctypes.byref(info))
    ts.append((time.perf_counter() - t0) * 1e3)
t = min(ts[1:])
print(f"potrf n={n}: {t:.3f} ms  {n ** 3 / 3 / t / 1e9:.1f} TF/s info={info.value}", flush=True)
Lr = torch.linalg.cholesky(A)
print(f"   rel err vs torch {(torch.linalg.norm(torch.tril(Hc.T) - Lr) / torch.linalg.norm(Lr)).item():.1e}", flush=True)
t0 = time.perf_counter(); torch.linalg.cholesky(A); torch.cuda.synchronize()
print(f"   rocSOLVER comparator {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)

b = torch.randn(n, dtype=torch.float64, device=dev)
x = b.clone()
potrs = lambda: (x.copy_(b), h.lib.ipm_potrs(h.ptr, n, 1, L.dptr(Hc), n, L.dptr(x), 1))
tmin, tavg = timed(potrs, 10)
print(f"potrs n={n} nrhs=1: {tmin:.3f} ms (avg {tavg:.3f})  {8 * n * n / tmin / 1e6:.0f} GB/s algorithmic (L read twice)", flush=True)
xr = torch.cholesky_solve(b[:, None], Lr)[:, 0]
print(f"   rel err vs torch {(torch.linalg.norm(x - xr) / torch.linalg.norm(xr)).item():.1e}", flush=True)
