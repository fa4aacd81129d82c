"""Device LU (ipm_getrf / ipm_getrs) against LAPACK (numpy.linalg.solve) on ill-conditioned
symmetric matrices: backward error ||A x - b|| / (||A|| ||x||) of both, forward error vs each other.
    python scripts/lu_accuracy.py"""
import ctypes
import sys

import numpy as np
import torch

sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
from gpu_util import handle  # noqa: E402
from ipm355 import _lib as L  # noqa: E402

h = handle()
for n, cond in ((80, 1e8), (80, 1e12), (80, 1e15), (300, 1e12), (1000, 1e12)):
    rng = np.random.default_rng(n)
    Q, _ = np.linalg.qr(rng.normal(size=(n, n)))
    ev = np.logspace(0, -np.log10(cond), n)
    A = (Q * ev) @ Q.T
    A = 0.5 * (A + A.T)
    b = rng.normal(size=n)
    x_np = np.linalg.solve(A, b)
    Ad = torch.as_tensor(A.T.copy(), device="cuda")
    piv = torch.empty(n, dtype=torch.int64, device="cuda")
    info = ctypes.c_int(0)
    assert h.lib.ipm_getrf(h.ptr, n, L.dptr(Ad), n, L.dptr(piv), ctypes.byref(info)) == 0
    Bd = torch.as_tensor(b.copy()[:, None], device="cuda")
    assert h.lib.ipm_getrs(h.ptr, n, 1, L.dptr(Ad), n, L.dptr(piv), L.dptr(Bd), 1) == 0
    x_d = Bd.cpu().numpy()[:, 0]
    be = lambda x: np.linalg.norm(A @ x - b) / (np.linalg.norm(A, 2) * np.linalg.norm(x))
    print(f"n={n} cond={cond:.0e}: backward err LAPACK {be(x_np):.1e} device {be(x_d):.1e}; "
          f"|x_d - x_np|/|x_np| {np.linalg.norm(x_d - x_np) / np.linalg.norm(x_np):.1e}", flush=True)
