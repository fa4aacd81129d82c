"""Times one device LU factorisation + solve (the Cholesky fallback, Q9 / np_solve) at n = 2048, 8192
(HIP events around ipm_getrf), against one fused Cholesky of the same SPD matrix."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "interiorpoint-gpu_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

from gpu_util import handle  # noqa: E402
from ipm355 import _lib as L  # noqa: E402

h = handle()
out = []
for n in [int(a) for a in sys.argv[1:]] or [2048, 8192]:
    g = torch.Generator(device="cuda").manual_seed(n)
    M = torch.rand((n, n), dtype=torch.float64, device="cuda", generator=g) - 0.5
    A = M.T @ M + n * torch.eye(n, dtype=torch.float64, device="cuda")
    piv = torch.empty(n, dtype=torch.int64, device="cuda")
    info = ctypes.c_int(0)
    res = {"n": n}
    for name, fn in (("getrf", lambda H: h.lib.ipm_getrf(h.ptr, n, L.dptr(H), n, L.dptr(piv), ctypes.byref(info))),
                     ("potrf", lambda H: h.lib.ipm_potrf(h.ptr, n, L.dptr(H), n, ctypes.byref(info)))):
        ts = []
        for rep in range(3):
            H = A.clone()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert fn(H) == 0
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        res[name + "_ms"] = min(ts)
    flops = 2 * n ** 3 / 3
    res["getrf_tflops"] = flops / (res["getrf_ms"] * 1e-3) / 1e12
    print(json.dumps(res), flush=True)
