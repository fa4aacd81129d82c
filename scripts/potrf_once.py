"""Two potrf calls at n (for kernel-trace timelines)."""
import ctypes, sys
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import torch
from gpu_util import handle
from ipm355 import _lib as L
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
h = handle()
torch.manual_seed(0)
M = torch.rand(n, n, dtype=torch.float64, device="cuda")
A = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
for r in range(2):
    Hc = A.clone(); torch.cuda.synchronize()
    info = ctypes.c_int(0)
    h.lib.ipm_potrf(h.ptr, n, L.dptr(Hc), n, ctypes.byref(info))
    torch.cuda.synchronize()
print("info", info.value)
