"""Factor a seeded SPD matrix with the library's ipm_potrf and save the lower factor (bitwise
comparisons between library builds: IPM355_LIB=... python scripts/potrf_dump.py n out.npy)."""
import ctypes, sys
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import numpy as np
import torch
from gpu_util import handle
from ipm355 import _lib as L
n, out = int(sys.argv[1]), sys.argv[2]
h = handle()
g = torch.Generator(device="cuda").manual_seed(1)
M = torch.rand(n, n, dtype=torch.float64, device="cuda", generator=g)
A = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
info = ctypes.c_int(0)
h.lib.ipm_potrf(h.ptr, n, L.dptr(A), n, ctypes.byref(info))
torch.cuda.synchronize()
np.save(out, torch.tril(A.T).cpu().numpy())
print(f"n={n} info={info.value}", flush=True)
