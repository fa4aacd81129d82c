"""Helpers for the -m gpu tests (device tensors + C-ABI calls)."""
import ctypes

import numpy as np


def handle():
    from ipm355 import _lib
    return _lib.Handle.get(0)


def dev(a):
    import torch
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device="cuda")


def host(t):
    return t.detach().cpu().numpy()


def colmajor_lower(Hmem, n):
    """device buffer laid out column-major with ld = Hmem.shape[1] -> dense lower-tri matrix"""
    M = host(Hmem).T[:n, :n]
    return np.tril(M)


def syrk(X, w, n, ldh=None, beta=0.0, H0=None, alpha=1.0):
    import torch
    from ipm355 import _lib as L
    h = handle()
    k = X.shape[0]
    ldh = ldh or n
    Xd = dev(X)
    wd = dev(w) if w is not None else None
    H = dev(H0) if H0 is not None else torch.zeros((n, ldh), dtype=torch.float64, device="cuda")
    h.check(h.lib.ipm_syrk(h.ptr, n, k, L.dptr(Xd), X.shape[1], L.dptr(wd), alpha, beta, L.dptr(H), ldh), h.ptr)
    return H


def potrf(Hmem, n, ldh, ncols=None):
    from ipm355 import _lib as L
    h = handle()
    info = ctypes.c_int(-7)
    if ncols is None:
        rc = h.lib.ipm_potrf(h.ptr, n, L.dptr(Hmem), ldh, ctypes.byref(info))
    else:
        rc = h.lib.ipm_potrf_partial(h.ptr, n, ncols, L.dptr(Hmem), ldh, ctypes.byref(info))
    return rc, info.value


def potrs(Lmem, n, ldl, B):
    from ipm355 import _lib as L
    h = handle()
    Bd = dev(B.reshape(n, -1))
    h.check(h.lib.ipm_potrs(h.ptr, n, Bd.shape[1], L.dptr(Lmem), ldl, L.dptr(Bd), Bd.shape[1]), h.ptr)
    return host(Bd)
