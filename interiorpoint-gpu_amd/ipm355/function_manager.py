"""Barrier oracles (the reference's L1 seam), backed by the HIP engine.

Mirrors the protocol of FunctionManager.py:94-195 -- update_x(x, update_slacks),
update_t, objective, newton_objective, gradient, hessian, inv_hessian and the
``slacks`` attribute -- for FunctionManagerLP (:197-356), FunctionManagerPhase1
(:359-616), FunctionManagerQP (:619-831), FunctionManagerSOCP (:834-1162) and
FunctionManagerSOCPPhase1 (:1165-1460).  Every value is computed on the device
(ipm_fm_* in include/ipm355.h); stale-slack semantics (update_slacks=False keeps
the previous slacks, Q2) are kept by the engine's slack state.  Results come
back as NumPy arrays, as the reference returns with use_gpu=False.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .device import ConeData, DeviceProblem, expand_bound


def _host(t):
    return t.detach().cpu().numpy()


class _DeviceBarrier:
    diag = False

    def _init_state(self, prob: DeviceProblem, x0, t):
        import torch
        self.prob = prob
        self.t = t
        self._x = torch.zeros(prob.N, dtype=torch.float64, device=prob.dev)
        self.is_constrained = True

    # -- protocol ---------------------------------------------------------------------
    def _set_x(self, x):
        import torch
        xt = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x, dtype=np.float64))
        xt = xt.to(device=self.prob.dev, dtype=torch.float64).reshape(-1)
        if xt.numel() == self.prob.N:
            self._x.copy_(xt)
        elif xt.numel() == self.prob.n and self.prob.phase1:
            self._x[: self.prob.n].copy_(xt)
        else:
            raise ValueError("Provided x does not have the right dimensions!")

    def update_x(self, x, update_slacks=True):
        self._set_x(x)
        self.prob.fm_update_x(self._x, update_slacks)

    def update_t(self, t):
        self.t = t

    @property
    def x(self):
        return _host(self._x[: self.prob.n])

    @property
    def slacks(self):
        return _host(self.prob.fm_slacks())

    def objective(self, x=None):
        if x is not None:
            self.update_x(x)
        return self.prob.fm_objective()

    def newton_objective(self, x=None, t=None):
        if x is not None:
            self.update_x(x)
        if t is not None:
            self.update_t(t)
        return self.prob.fm_newton_objective(self.t)

    def gradient(self, x=None, t=None):
        if x is not None:
            self.update_x(x)
        if t is not None:
            self.update_t(t)
        return _host(self.prob.fm_gradient(self.t))

    def hessian(self, x=None, t=None):
        if x is not None:
            self.update_x(x)
        if t is not None:
            self.update_t(t)
        return _host(self.prob.fm_hessian(self.t, diag=self.diag))

    def inv_hessian(self, x=None):
        if not self.diag:
            raise ValueError("Hessian is not diagonal, cannot use inv hessian function!")
        return 1 / self.hessian(x)


class FunctionManagerLP(_DeviceBarrier):
    """FunctionManager.py:197-356.  try_diag and no C and bounded -> diagonal Hessian."""

    def __init__(self, c=None, A=None, b=None, C=None, d=None, x0=None, lower_bound=None, upper_bound=None,
                 t=1, use_gpu=True, n=None, try_diag=True, solve_method=None, device=0, _prob=None):
        n = len(x0) if x0 is not None else n
        if c is None:
            c = np.ones(n)
        self.try_diag = try_diag
        self.diag = C is None and try_diag and (lower_bound is not None or upper_bound is not None)
        if solve_method is None:
            solve_method = L.SOLVE_DIAGONAL if self.diag else L.SOLVE_CHOLESKY
        prob = _prob or DeviceProblem("LP", n, solve_method=solve_method, c=c, C=C, d=d,
                                      lb=expand_bound(lower_bound, n), ub=expand_bound(upper_bound, n),
                                      A=A, b=b, device=device)
        self._init_state(prob, x0, t)
        if x0 is not None:
            self.update_x(x0)


class FunctionManagerQP(_DeviceBarrier):
    """FunctionManager.py:619-831."""

    def __init__(self, P=None, q=None, A=None, b=None, C=None, d=None, x0=None, lower_bound=None,
                 upper_bound=None, t=1, use_gpu=True, n=None, solve_method=L.SOLVE_CHOLESKY, device=0,
                 _prob=None):
        n = len(x0) if x0 is not None else n
        prob = _prob or DeviceProblem("QP", n, solve_method=solve_method, P=P, q=q, C=C, d=d,
                                      lb=expand_bound(lower_bound, n), ub=expand_bound(upper_bound, n),
                                      A=A, b=b, device=device)
        self._init_state(prob, x0, t)
        if x0 is not None:
            self.update_x(x0)


class FunctionManagerPhase1(_DeviceBarrier):
    """FunctionManager.py:359-616: x~ = (x, s), s0 = -min(slacks) + 1 (:390-393)."""

    def __init__(self, c=None, A=None, b=None, C=None, d=None, x0=None, lower_bound=None, upper_bound=None,
                 t=1, use_gpu=True, n=None, try_diag=False, suppress_print=True, device=0, _prob=None):
        n = len(x0)
        prob = _prob or DeviceProblem("LP", n, phase1=True, C=C, d=d, lb=expand_bound(lower_bound, n),
                                      ub=expand_bound(upper_bound, n), device=device)
        self._init_state(prob, x0, t)
        self._start(x0, suppress_print)

    def _start(self, x0, suppress_print=True):
        self.update_x(np.append(np.asarray(x0, dtype=np.float64), 0.0))
        self.s = -float(self.prob.fm_slacks().min().item()) + 1
        self.update_x(np.append(np.asarray(x0, dtype=np.float64), self.s))
        if not suppress_print:
            print(f"Starting slack of {np.round(self.s, 4)}")

    def update_x(self, x, update_slacks=True):
        super().update_x(x, update_slacks)
        if len(x) == self.prob.N:
            self.s = float(x[-1]) if not hasattr(x, "device") else float(x[-1].item())


class FunctionManagerSOCP(_DeviceBarrier):
    """FunctionManager.py:834-1162 (stacked-cone form: no per-cone n x n caches)."""

    def __init__(self, P=None, q=None, A=None, b=None, c=None, d=None, F=None, g=None, lower_bound=None,
                 upper_bound=None, x0=None, t=1, use_gpu=True, n=None, solve_method=L.SOLVE_CHOLESKY,
                 device=0, _prob=None, _cones=None):
        n = len(x0) if x0 is not None else n
        if _prob is None:
            import torch
            dev = torch.device("cuda", device)
            cones = _cones or ConeData(A, b, c, d, n, dev)
            _prob = DeviceProblem("SOCP", n, solve_method=solve_method, P=P, q=q, cones=cones,
                                  lb=expand_bound(lower_bound, n), ub=expand_bound(upper_bound, n),
                                  A=F, b=g, device=device)
        self._init_state(_prob, x0, t)
        if x0 is not None:
            self.update_x(x0)


class FunctionManagerSOCPPhase1(FunctionManagerPhase1):
    """FunctionManager.py:1165-1460."""

    def __init__(self, A=None, b=None, c=None, d=None, x0=None, lower_bound=None, upper_bound=None, t=1,
                 use_gpu=True, n=None, suppress_print=True, device=0, _prob=None, _cones=None):
        import torch
        n = len(x0)
        if _prob is None:
            dev = torch.device("cuda", device)
            cones = _cones or ConeData(A, b, c, d, n, dev)
            _prob = DeviceProblem("SOCP", n, phase1=True, cones=cones, lb=expand_bound(lower_bound, n),
                                  ub=expand_bound(upper_bound, n), device=device)
        self._init_state(_prob, x0, t)
        self._start(x0, suppress_print)
