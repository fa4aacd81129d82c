"""Newton inner solvers (the reference's L2 seam), executed by the native engine.

``solve(x, t, v0=None) -> (x, v, iters, stat, success)`` exactly as
NewtonSolver.solve (NewtonSolver.py:80-155) and NewtonSolverInfeasibleStart.solve
(NewtonSolverInfeasibleStart.py:72-168).  The whole loop -- gradient, KKT
assembly, Cholesky, triangular solves, backtracking -- runs in
libipm355.so (ipm_newton_solve) with one device->host copy per iteration.

x (and v) may be torch device tensors (updated in place, Q8) or NumPy arrays
(copied to the device, solved, copied back in place).
"""
from __future__ import annotations

import numpy as np

from . import _lib as L


def _to_dev(a, prob):
    import torch
    if isinstance(a, torch.Tensor):
        return a, False
    return torch.as_tensor(np.asarray(a, dtype=np.float64), device=prob.dev).clone(), True


class NewtonSolver:
    """Base: NewtonSolver.__init__ (NewtonSolver.py:16-78)."""

    method = "cholesky"
    infeasible = False

    def __init__(self, A=None, b=None, C=None, d=None, function_manager=None, lower_bound=None,
                 upper_bound=None, max_iters=50, epsilon=1e-5, suppress_print=True, max_cg_iters=50,
                 alpha=0.2, beta=0.6, mu=20, use_gpu=True, track_loss=False, phase1_flag=False,
                 phase1_tol=0.1, use_psd_condition=False, update_slacks_every=0):
        self.A, self.b, self.C, self.d = A, b, C, d
        self.fm = function_manager
        self.max_iters, self.eps = max_iters, epsilon
        self.suppress_print = suppress_print
        self.max_cg_iters = max_cg_iters
        self.alpha, self.beta, self.mu = alpha, beta, mu
        self.use_gpu = True
        self.track_loss = track_loss
        self.phase1_flag, self.phase1_tol = phase1_flag, phase1_tol
        self.use_psd_condition = use_psd_condition
        self.update_slacks_every = update_slacks_every
        if self.method in ("lu", "lstsq") and self.fm is not None:
            self.fm.prob.use_backup = True       # np.linalg.solve / lstsq / inv from the start
        self.last_result = None
        self.trace = []          # per-iteration (step, nd | residual) like the oracle's trace

    @property
    def use_backup(self):
        return self.fm.prob.use_backup

    def solve(self, x, t, v0=None):
        import torch
        prob = self.fm.prob
        xd, copied = _to_dev(x, prob)
        v = None
        if self.infeasible:
            if v0 is None:
                v = torch.zeros(prob.desc.p, dtype=torch.float64, device=prob.dev)
                vcopied = False
            else:
                v, vcopied = _to_dev(v0, prob)
        r = prob.newton_solve(xd, self.fm.t, v, max_iters=self.max_iters, eps=self.eps, alpha=self.alpha,
                              beta=self.beta, update_slacks_every=self.update_slacks_every,
                              phase1_flag=self.phase1_flag, phase1_tol=self.phase1_tol,
                              use_psd_condition=self.use_psd_condition)
        self.last_result = r
        self.trace.extend(prob.last_trace)
        self.fm._x.copy_(xd.reshape(-1)) if xd.numel() == prob.N else None
        if copied:
            np.copyto(x, xd.cpu().numpy())
            xd = x
        if self.infeasible and v0 is not None and vcopied:
            np.copyto(v0, v.cpu().numpy())
            v = v0
        stat = r.stat if r.stat_valid else None
        if not self.suppress_print and r.linalg_error:
            print("OVERFLOW ERROR: Problem likely unbounded")      # (NewtonSolver.py:148-155)
        elif not self.suppress_print and r.iters >= self.max_iters and not r.success:
            print("REACHED MAX ITERATIONS: Problem likely infeasible or unbounded")
        return xd, v, int(r.iters), stat, bool(r.success)


class NewtonSolverCholesky(NewtonSolver):
    """NewtonSolver.py:250-341: Cholesky; first failure -> permanent fallback (Q9): from then on
    lstsq(H, -g, rcond=None) (backup_solve, :334-341), the device minimum-norm solve."""


class NewtonSolverDiagonal(NewtonSolver):
    """NewtonSolver.py:403-420: H diagonal (LP, C is None, try_diag)."""
    method = "diag"


class NewtonSolverNPSolve(NewtonSolver):
    """NewtonSolver.py:230-247: np.linalg.solve -> device LU with partial pivoting."""
    method = "lu"


class NewtonSolverNPLstSq(NewtonSolver):
    """NewtonSolver.py:212-227: lstsq(H, -g, rcond=None) -> the device minimum-norm solve
    (eigenvectors of H, |lambda| <= eps n max|lambda| dropped: gelsd's rcond rule)."""
    method = "lstsq"


class NewtonSolverDirect(NewtonSolverNPSolve):
    """NewtonSolver.py:344-361: explicit inverse -> same system solved by LU."""


class NewtonSolverCG(NewtonSolver):
    def __init__(self, *a, **k):
        raise NotImplementedError("linear_solve_method='cg' is not provided by the HIP backend "
                                  "(see DESIGN.md, next steps)")


class NewtonSolverInfeasibleStart(NewtonSolver):
    """NewtonSolverInfeasibleStart.py:13-273 (A x = b via block elimination)."""
    infeasible = True

    def __init__(self, A, b, C, d, function_manager, **kw):
        kw.pop("phase1_flag", None)
        kw.pop("phase1_tol", None)
        super().__init__(A, b, C, d, function_manager, **kw)


class NewtonSolverCholeskyInfeasibleStart(NewtonSolverInfeasibleStart):
    """NewtonSolverInfeasibleStart.py:356-538."""


class NewtonSolverCholeskyDiagonalInfeasibleStart(NewtonSolverInfeasibleStart):
    """NewtonSolverInfeasibleStart.py:757-809."""
    method = "diag"


class NewtonSolverNPSolveInfeasibleStart(NewtonSolverInfeasibleStart):
    """NewtonSolverInfeasibleStart.py:312-354 -> device LU."""
    method = "lu"


class NewtonSolverNPLstSqInfeasibleStart(NewtonSolverInfeasibleStart):
    """NewtonSolverInfeasibleStart.py:279-316: block elimination with four lstsq calls."""
    method = "lstsq"


class NewtonSolverDirectInfeasibleStart(NewtonSolverNPSolveInfeasibleStart):
    pass


class NewtonSolverKKTNPSolveInfeasibleStart(NewtonSolverNPSolveInfeasibleStart):
    """NewtonSolverInfeasibleStart.py:663-689.  The reference assembles the full KKT matrix with
    np.bmat([[np.diag(H), A^T], [A, 0]]); with a dense (2-D) Hessian np.diag returns its diagonal
    VECTOR and np.bmat raises ValueError at the first Newton step -- kept: same error, same point."""

    def solve(self, x, t, v0=None):
        raise ValueError("all the input array dimensions except for the concatenation axis must match "
                         "exactly (reference NewtonSolverKKTNPSolveInfeasibleStart: np.diag of a dense "
                         "Hessian inside np.bmat, NewtonSolverInfeasibleStart.py:680-685)")


def _cg_unsupported(*a, **k):
    raise NotImplementedError("CONJUGATE GRADIENT GIVING UNSTABLE RESULTS, NEEDS TO BE DEBUGGED")


class NewtonSolverCGInfeasibleStart(NewtonSolverInfeasibleStart):
    __init__ = _cg_unsupported


class NewtonSolverCGDiagonalInfeasibleStart(NewtonSolverInfeasibleStart):
    __init__ = _cg_unsupported


class NewtonSolverNPSolveDiagonalInfeasibleStart(NewtonSolverCholeskyDiagonalInfeasibleStart):
    """Diagonal H: S = A diag(1/h) A^T solved by Cholesky on the device (same system)."""


class NewtonSolverNPLstSqDiagonalInfeasibleStart(NewtonSolverCholeskyDiagonalInfeasibleStart):
    """NewtonSolverInfeasibleStart.py:692-724: diagonal H, w = lstsq(A diag(1/h) A^T, r)."""
    method = "diag_lstsq"


NewtonSolverDirectDiagonalInfeasibleStart = NewtonSolverNPSolveDiagonalInfeasibleStart
NewtonSolverKKTNPSolveDiagonalInfeasibleStart = NewtonSolverNPSolveDiagonalInfeasibleStart
