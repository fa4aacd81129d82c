"""Phase-1 feasibility solver (PhaseOneSolver.py:6-154) on the HIP engine.

min s  s.t.  slacks(x) + s > 0, variables x~ = (x, s) held on the device; the
inner solver is the same native Newton loop (Cholesky, bordered (n+1) KKT).
"""
from __future__ import annotations

import numpy as np

from .function_manager import FunctionManagerPhase1, FunctionManagerSOCPPhase1
from .newton import NewtonSolverCholesky


class PhaseOneSolver:
    def __init__(self, C=None, d=None, lower_bound=0, upper_bound=None, x0=None, max_outer_iters=50,
                 max_inner_iters=20, epsilon=1e-8, inner_epsilon=1e-5, linear_solve_method="cholesky",
                 max_cg_iters=50, alpha=0.2, beta=0.6, mu=15, t0=1, suppress_print=False, use_gpu=True,
                 track_loss=False, n=None, tol=0.1, socp=False, socp_params=None, use_psd_condition=False,
                 update_slacks_every=0, device=0, _cones=None):
        import torch
        self.C, self.d = C, d
        self.lb, self.ub = lower_bound, upper_bound
        self.n = n
        self.max_outer_iters, self.max_inner_iters = max_outer_iters, max_inner_iters
        self.epsilon, self.inner_epsilon = epsilon, inner_epsilon
        self.alpha, self.beta, self.mu = alpha, beta, mu
        self.suppress_print = suppress_print
        self.tol, self.t0 = tol, t0
        self.update_slacks_every = update_slacks_every
        if not socp:
            self.phase1_fm = FunctionManagerPhase1(C=C, d=d, x0=x0, lower_bound=lower_bound,
                                                   upper_bound=upper_bound, t=t0, n=n,
                                                   suppress_print=suppress_print, device=device)
        else:
            A, b, c, dd = socp_params
            self.phase1_fm = FunctionManagerSOCPPhase1(A=A, b=b, c=c, d=dd, x0=x0, lower_bound=lower_bound,
                                                       upper_bound=upper_bound, t=t0, n=n,
                                                       suppress_print=suppress_print, device=device,
                                                       _cones=_cones)
        prob = self.phase1_fm.prob
        self.x = torch.as_tensor(np.append(np.asarray(x0, dtype=np.float64), self.phase1_fm.s),
                                 device=prob.dev)
        self.phase1_ns = NewtonSolverCholesky(function_manager=self.phase1_fm, max_iters=max_inner_iters,
                                              epsilon=inner_epsilon, suppress_print=suppress_print,
                                              max_cg_iters=max_cg_iters, alpha=alpha, beta=beta, mu=mu,
                                              phase1_flag=True, phase1_tol=tol,
                                              use_psd_condition=use_psd_condition,
                                              update_slacks_every=update_slacks_every)
        self.outer_iters = 0
        self.inner_iters = []
        self._budget = None

    def solve(self, x0=None):
        """PhaseOneSolver.py:112-154; returns (x[:-1] (device view), s)."""
        if x0 is not None:
            self.phase1_fm.update_x(x0)
        t = self.t0
        self.outer_iters = 0
        self.inner_iters = []
        obj_val = None
        for it in range(self.max_outer_iters):
            if not self.suppress_print:
                print(f"Current slack: {self.phase1_fm.s}")
            if self._budget is not None:
                if self._budget[0] <= 0:
                    break
                self.phase1_ns.max_iters = min(self.max_inner_iters, self._budget[0])
            self.x, _, k, _, ok = self.phase1_ns.solve(self.x, t)
            if self._budget is not None:
                self._budget[0] -= k
                self.phase1_ns.max_iters = self.max_inner_iters
            self.outer_iters += 1
            self.inner_iters.append(k)
            obj_val = self.phase1_fm.objective(self.x)
            if obj_val < -self.tol:
                break
            if k >= self.max_inner_iters and not self.suppress_print:
                print(f"Reached max Newton steps during {it}th centering step (t={t}) of phase 1")
            t = min(t * self.mu, (self.n + 1.0) / self.epsilon)
            self.phase1_fm.update_t(t)
        return self.x[:-1], obj_val
