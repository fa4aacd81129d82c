"""Raw role timeline of ONE fused Cholesky launch (block b) from the diagnostic library, saved
for offline analysis (scripts/role_trace.py prints the summary of the same data).
   IPM355_LIB=<trace lib> IPM_TRACE_BLOCK=b python scripts/role_dump.py n out.npz
Saves rows (role, start, end, wake-or-cu-key) in s_memrealtime ticks (100 MHz) and the launch's
kernel time (HIP events over the whole factorization)."""
import ctypes, os, sys
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import numpy as np
import torch
from gpu_util import handle
from ipm355 import _lib as L
n = int(sys.argv[1])
out = sys.argv[2]
h = handle()
torch.manual_seed(0)
M = torch.rand(n, n, dtype=torch.float64, device="cuda")
A = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
ms = []
for _ in range(3):
    Hc = A.clone(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    info = ctypes.c_int(0)
    e0.record()
    h.lib.ipm_potrf(h.ptr, n, L.dptr(Hc), n, ctypes.byref(info))
    e1.record()
    torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1))
buf = (ctypes.c_ulonglong * (4 * 8192))()
h.lib.ipm_debug_role_trace(buf, 8192)
a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4).astype(np.int64)
a = a[a[:, 1] > 0]
np.savez(out, a=a, ms=np.array(ms), n=n, block=int(os.environ.get("IPM_TRACE_BLOCK", "-1")))
print(f"block {os.environ.get('IPM_TRACE_BLOCK')}: {len(a)} workgroups, span {(a[:, 2].max() - a[:, 1].min()) / 100:.1f} us,"
      f" factorization {min(ms):.3f} ms")
