import sys, time, ctypes
sys.path[:0]=['/root/repo/interiorpoint-gpu_amd','/root/repo/tests']
import numpy as np, torch
from gpu_util import dev, potrf, colmajor_lower, handle
for n in [2048, 4096, 8192]:
    torch.manual_seed(0)
    M = torch.randn(n, n, dtype=torch.float64, device="cuda")
    A = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
    H = A.clone()
    rc, info = potrf(H, n, n); torch.cuda.synchronize()
    ts=[]
    for r in range(3):
        H.copy_(A); torch.cuda.synchronize(); t0=time.perf_counter(); rc, info = potrf(H, n, n); ts.append(time.perf_counter()-t0)
    Lr = torch.linalg.cholesky(A)
    Lg = torch.tril(H.T)
    err = (torch.linalg.norm(Lg - Lr) / torch.linalg.norm(Lr)).item()
    t=min(ts); print(f"potrf n={n}: {t*1e3:.2f} ms  {n**3/3/t/1e12:.2f} TF/s  rc={rc} info={info} rel-err vs torch {err:.1e}", flush=True)
    # torch (rocSOLVER) reference timing for comparison only
    torch.cuda.synchronize(); t0=time.perf_counter(); torch.linalg.cholesky(A); torch.cuda.synchronize(); t1=time.perf_counter()
    print(f"   rocSOLVER (torch) comparator: {(t1-t0)*1e3:.2f} ms", flush=True)
