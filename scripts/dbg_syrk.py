import ctypes, sys
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import torch
from gpu_util import handle
from ipm355 import _lib as L
h = handle()
torch.manual_seed(0)
for (n, k, ld, beta, alpha) in [(7680, 256, 8192, 1.0, -1.0), (7680, 256, 7680, 1.0, -1.0), (7680, 256, 8192, 0.0, 1.0), (4096, 256, 4096, 1.0, -1.0), (1024, 256, 1024, 1.0, -1.0)]:
    X = torch.rand(k, ld, dtype=torch.float64, device="cuda")
    H0 = torch.rand(n, ld, dtype=torch.float64, device="cuda")
    H = H0.clone()
    h.lib.ipm_syrk(h.ptr, n, k, L.dptr(X), ld, None, alpha, beta, L.dptr(H), ld)
    torch.cuda.synchronize()
    Xs = X[:, :n]
    ref = alpha * Xs.T @ Xs + beta * H0[:, :n].T
    got = H[:, :n].T
    d = torch.tril(got - ref).abs().max().item()
    print(n, k, ld, beta, alpha, "maxdiff", d, "untouched upper ok:", torch.equal(torch.triu(H[:, :n].T, 1), torch.triu(H0[:, :n].T, 1)), flush=True)
for n in [1024, 2048, 4096, 8192]:
    M = torch.rand(n, n, dtype=torch.float64, device="cuda")
    A = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
    Hc = A.clone()
    info = ctypes.c_int(0)
    rc = h.lib.ipm_potrf(h.ptr, n, L.dptr(Hc), n, ctypes.byref(info))
    Lr = torch.linalg.cholesky(A)
    print("potrf", n, rc, info.value, (torch.tril(Hc.T) - Lr).abs().max().item(), flush=True)
