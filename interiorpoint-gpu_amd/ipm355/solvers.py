"""Problem facades: LPSolver / QPSolver / SOCPSolver with the reference's API.

Constructor kwargs, defaults, validation errors, x0 defaults, the solver
dispatch, the outer barrier loop and the result attributes follow
LPSolver.py:18-705, QPSolver.py:18-689 and SOCPSolver.py:18-833.  Differences:
  * every numeric step runs on the MI355X through libipm355.so -- ``use_gpu`` is
    accepted for signature compatibility; there is no CPU path;
  * ``check_cvxpy`` degrades to a no-op when cvxpy is not installed;
  * ``linear_solve_method='cg'`` is not provided (the reference marks CG broken).
Results: ``value`` (float), ``xstar`` (NumPy), ``optimality_gap``, ``outer_iters``,
``inner_iters``, ``objective_vals``, ``lam_star``, ``v_star``, ``optimal``.
"""
from __future__ import annotations

import warnings

import numpy as np

from . import _lib as L
from . import newton as NS
from .device import ConeData, DeviceProblem, expand_bound
from .function_manager import FunctionManagerLP, FunctionManagerQP, FunctionManagerSOCP
from .phase_one import PhaseOneSolver


def _default_x0(n, lb, ub):
    """LPSolver.py:128-143 (identical in QP/SOCP)."""
    if lb is not None and ub is not None:
        return (np.maximum(lb, -1e2) + np.minimum(ub, 1e2)) / 2 * np.ones(n)
    if lb is not None:
        return (np.maximum(lb, -1e2) + 1e-1) * np.ones(n)
    if ub is not None:
        return (np.minimum(ub, 1e2) - 1e-1) * np.ones(n)
    return np.random.rand(n)


def _check_bounds(lb, ub, dims):
    """LPSolver.py:271-314 bound validation (dims: lengths the bounds must match)."""
    if lb is not None:
        try:
            lb = np.array(lb)
        except Exception:
            raise ValueError("Lower bound must be a scalar or list!")
        if lb.ndim > 0 and any(len(lb) != k for k in dims):
            raise ValueError("Lower bound must be a scalar or have the same number of dimensions as other parameters!")
    if ub is not None:
        try:
            ub = np.array(ub)
        except Exception:
            raise ValueError("Upper bound must be a scalar or list!")
        if ub.ndim > 0 and any(len(ub) != k for k in dims):
            raise ValueError("Upper bound must be a scalar or have the same number of dimensions as other parameters!")
    if lb is not None and ub is not None:
        diff = ub - lb
        if (np.asarray(diff) < 0).any():
            raise ValueError("Lower bound must be lower than upper bound")
    return lb, ub


_METHODS = ("np_lstsq", "np_solve", "direct", "cg", "kkt", "cholesky")


def _feasible_class(method, diag):
    if method not in _METHODS:
        raise ValueError("Please enter a valid linear solve method!")
    if diag:
        return NS.NewtonSolverDiagonal
    return {"np_lstsq": NS.NewtonSolverNPLstSq, "np_solve": NS.NewtonSolverNPSolve,
            "direct": NS.NewtonSolverDirect, "cg": NS.NewtonSolverCG, "cholesky": NS.NewtonSolverCholesky,
            "kkt": None}[method]


def _infeasible_class(method, diag):
    if method not in _METHODS:
        raise ValueError("Please enter a valid linear solve method!")
    if diag:
        return {"np_lstsq": NS.NewtonSolverNPLstSqDiagonalInfeasibleStart,
                "np_solve": NS.NewtonSolverNPSolveDiagonalInfeasibleStart,
                "direct": NS.NewtonSolverDirectDiagonalInfeasibleStart,
                "cg": NS.NewtonSolverCGDiagonalInfeasibleStart,
                "kkt": NS.NewtonSolverKKTNPSolveDiagonalInfeasibleStart,
                "cholesky": NS.NewtonSolverCholeskyDiagonalInfeasibleStart}[method]
    return {"np_lstsq": NS.NewtonSolverNPLstSqInfeasibleStart, "np_solve": NS.NewtonSolverNPSolveInfeasibleStart,
            "direct": NS.NewtonSolverDirectInfeasibleStart, "cg": NS.NewtonSolverCGInfeasibleStart,
            "kkt": NS.NewtonSolverKKTNPSolveInfeasibleStart,
            "cholesky": NS.NewtonSolverCholeskyInfeasibleStart}[method]


def _solve_method_for(cls):
    if cls.method == "diag":
        return L.SOLVE_DIAGONAL
    if cls.method == "diag_lstsq":
        return L.SOLVE_DIAGONAL_LSTSQ
    if cls.method == "lu":
        return L.SOLVE_LU
    if cls.method == "lstsq":
        return L.SOLVE_LSTSQ
    return L.SOLVE_CHOLESKY


class _BarrierSolver:
    """Shared outer loop (LPSolver.py:514-653 / QPSolver.py:500-638 / SOCPSolver.py:616-753)."""

    _eq_name = "A"
    _title = "Solver"

    # --- set by subclasses: self.fm, self.ns, self.phase1_solver (or None), self.eqA, self.eqb
    def _maybe_cvxpy(self, check_cvxpy, suppress_print):
        self.feasible, self.cvxpy_val, self.cvxpy_sol = None, None, None
        if not check_cvxpy:
            return
        try:
            import cvxpy  # noqa: F401
        except Exception:
            warnings.warn("check_cvxpy=True but cvxpy is not installed; skipping the CVXPY check")
            return
        warnings.warn("CVXPY feasibility check is not part of the HIP hot path; skipped")

    def _eq_residual_ok(self, x):
        if self.eqA is None:
            return True
        import torch
        r = self.eqA_t @ x - self.eqb_t
        return float(torch.linalg.norm(r).item()) < self._eq_tol()

    def __str__(self):
        opt_val = "Not yet solved" if self.optimal is False else self.value
        return f"{self._title}(Optimal Value: {opt_val})"

    __repr__ = __str__

    def solve(self, resolve=True, **kwargs):
        import torch
        if not resolve and self.optimal:
            return self.value
        t = kwargs.get("t0", self.t0)
        max_outer_iters = kwargs.get("max_outer_iters", self.max_outer_iters)
        self.track_loss = kwargs.get("track_loss", self.track_loss)
        # extension (benchmarks): stop after exactly this many Newton iterations in total
        budget = kwargs.get("iteration_budget")
        self._budget = [budget] if budget is not None else None
        host_x = None
        if "x0" in kwargs:
            x = kwargs["x0"]
            self._check_x0(x)
            update_x = True
        else:
            x = self.x
            update_x = False
        if self.phase1_solver is not None and self.phase1_solver.phase1_fm.s >= 1:   # Q11
            if not self.suppress_print:
                print("running phase 1 solver")
            self.phase1_solver._budget = self._budget
            x, s = self.phase1_solver.solve(x0=x) if update_x else self.phase1_solver.solve()
            self.phase1_solver._budget = None
            if self._budget is not None and self._budget[0] <= 0:
                self.xstar = None
                return None
            if s > -self.phase1_tol:
                raise ValueError("Phase 1 Solver did not successfully find a feasible point!")
            if not self.suppress_print:
                print(f"found a feasible point with slack {s}")
        else:
            host_x = x if isinstance(x, np.ndarray) else None   # mutated in place like the reference (Q8)
            x = torch.as_tensor(np.asarray(x, dtype=np.float64), device=self.dev).clone()
        if not self.suppress_print:
            print("proceeding to solve method")
        self.outer_iters = 0
        objective_vals = []
        self.inner_iters = []
        self.fm.update_x(x)
        self.fm.update_t(t)
        v = torch.zeros(self.eqA.shape[0], dtype=torch.float64, device=self.dev) if self.eqA is not None else None
        dual_gap = self.num_constraints
        best_x = x.clone()
        best_obj = np.inf
        for it in range(max_outer_iters):
            if self._budget is not None:
                if self._budget[0] <= 0:
                    break
                self.ns.max_iters = min(self.max_inner_iters, self._budget[0])
            x, v, numiters_t, _, success_flag = self.ns.solve(x, t, v0=v)
            self.x_last = x              # extension: the current iterate (truncated parity runs)
            if self._budget is not None:
                self._budget[0] -= numiters_t
                self.ns.max_iters = self.max_inner_iters
            self.outer_iters += 1
            self.inner_iters.append(numiters_t)
            if self._eq_residual_ok(x):
                obj_val = self.fm.objective()
                if not self.suppress_print:
                    print(f"Objective value is now {obj_val}")
                if self.track_loss:
                    objective_vals.append(obj_val)
                if obj_val < best_obj:
                    best_obj = obj_val
                    best_x = x.clone()
                elif success_flag:
                    break
            else:
                if not self.suppress_print:
                    print(f"Newton step at iteration {it + 1} did not converge")
                if len(objective_vals) > 0:
                    objective_vals.append(objective_vals[-1])
            if not self.suppress_print and numiters_t >= self.max_inner_iters:
                print(f"Reached max Newton steps during {it + 1}th centering step (t={t})")
            dual_gap = self.num_constraints / t
            if dual_gap < self.epsilon:
                break
            t = t * self.mu
            self.fm.update_t(t)
        if host_x is not None:
            np.copyto(host_x, x.cpu().numpy())
        self.xstar = best_x.cpu().numpy()
        if self.get_dual_variables:
            if self._has_ineq or self.bounded:
                self.fm.update_x(best_x)
                self.lam_star = 1 / (t * self.fm.slacks)
            if self.eqA is not None:
                self.v_star = (v / t).cpu().numpy()
        self.optimal = True
        self.value = best_obj
        self.optimality_gap = dual_gap
        self.objective_vals = objective_vals
        return self.value

    def plot(self, subtract_cvxpy=True):
        if not (self.optimal and self.track_loss):
            raise ValueError("Need to solve problem with track_loss set to True to be able to plot convergence!")
        import matplotlib.pyplot as plt
        ax = plt.subplot()
        base = self.cvxpy_val if (subtract_cvxpy and self.cvxpy_val is not None) else 0.0
        ax.step(np.cumsum(self.inner_iters[-len(self.objective_vals):]), np.array(self.objective_vals) - base,
                where="post")
        ax.set_xlabel("Cumulative Newton iterations")
        ax.set_ylabel("Optimality gap")
        ax.set_title(f"Convergence of {self._title}")
        ax.set_yscale("log")
        return ax

    def _common(self, t0, max_outer_iters, max_inner_iters, epsilon, inner_epsilon, max_cg_iters, alpha, beta,
                mu, suppress_print, track_loss, linear_solve_method, get_dual_variables, phase1_tol,
                phase1_max_inner_iters, update_slacks_every, use_gpu, device):
        import torch
        self.dev = torch.device("cuda", device)
        self.device = device
        self.use_gpu = True
        self.alpha, self.beta = alpha, beta
        self.t0, self.mu = t0, mu
        self.outer_iters = 0
        self.inner_iters = []
        self.max_outer_iters, self.max_inner_iters = max_outer_iters, max_inner_iters
        self.epsilon, self.inner_epsilon = epsilon, inner_epsilon
        self.max_cg_iters = max_cg_iters
        self.optimal = False
        self.value = None
        self.optimality_gap = None
        self.xstar = None
        self.lam_star = None
        self.vstar = None
        self.suppress_print = suppress_print
        self.track_loss = track_loss
        self.linear_solve_method = linear_solve_method
        self.get_dual_variables = get_dual_variables
        self.phase1_tol = phase1_tol
        self.phase1_max_inner_iters = phase1_max_inner_iters
        self.update_slacks_every = update_slacks_every
        self.objective_vals = []


class LPSolver(_BarrierSolver):
    """min c'x s.t. Ax = b, Cx <= d, lower_bound <= x <= upper_bound  (LPSolver.py:18-705)."""

    _title = "LinearSolver"

    def __init__(self, c=None, A=None, b=None, C=None, d=None, lower_bound=0, upper_bound=None, t0=0.1,
                 max_outer_iters=20, max_inner_iters=50, phase1_max_inner_iters=500, epsilon=1e-10,
                 inner_epsilon=1e-5, check_cvxpy=True, linear_solve_method="cholesky", max_cg_iters=50,
                 alpha=0.2, beta=0.6, mu=15, suppress_print=False, use_gpu=False, try_diag=True,
                 track_loss=False, get_dual_variables=False, phase1_tol=0, phase1_t0=0.01, x0=None,
                 update_slacks_every=0, device=0):
        self.A, self.c, self.C, self.b, self.d = A, c, C, b, d
        self.lb, self.ub = lower_bound, upper_bound
        self._check_inputs()
        self.equality_constrained = A is not None
        self.n = len(c) if c is not None else (A.shape[1] if A is not None else C.shape[1])
        self.x = x0 if x0 is not None else _default_x0(self.n, self.lb, self.ub)
        self.bounded = self.lb is not None or self.ub is not None
        self._maybe_cvxpy(check_cvxpy, suppress_print)
        self.num_constraints = (len(d) if d is not None else 0) + self.n * (self.lb is not None) + \
            self.n * (self.ub is not None)
        self._common(t0, max_outer_iters, max_inner_iters, epsilon, inner_epsilon, max_cg_iters, alpha, beta, mu,
                     suppress_print, track_loss, linear_solve_method, get_dual_variables, phase1_tol,
                     phase1_max_inner_iters, update_slacks_every, use_gpu, device)
        self.try_diag = try_diag
        self.phase1_t0 = phase1_t0
        self._has_ineq = C is not None
        self.eqA, self.eqb = A, b
        self.phase1_solver = None
        if C is not None:
            self.phase1_solver = PhaseOneSolver(C=C, d=d, lower_bound=self.lb, upper_bound=self.ub, x0=self.x,
                                                max_outer_iters=max_outer_iters,
                                                max_inner_iters=phase1_max_inner_iters, epsilon=epsilon,
                                                inner_epsilon=inner_epsilon, alpha=alpha, beta=beta, mu=mu,
                                                suppress_print=suppress_print, n=self.n, tol=phase1_tol,
                                                t0=phase1_t0, update_slacks_every=update_slacks_every,
                                                device=device)
        diag = not (C is not None or not try_diag)
        if self.equality_constrained:
            cls = _infeasible_class(linear_solve_method, diag)
        else:
            cls = _feasible_class(linear_solve_method, diag)
            if cls is None:
                raise ValueError("No KKT System non-equality-constrained problems! Please choose another solver")
        if cls.method in ("diag", "diag_lstsq") and C is None and not self.bounded:
            cls = NS.NewtonSolverCholesky if not self.equality_constrained else NS.NewtonSolverCholeskyInfeasibleStart
        self.fm = FunctionManagerLP(c=c, A=A, b=b, C=C, d=d, x0=self.x, lower_bound=self.lb, upper_bound=self.ub,
                                    t=1, n=self.n, try_diag=try_diag, solve_method=_solve_method_for(cls),
                                    device=device)
        if A is not None:
            self.eqA_t, self.eqb_t = self.fm.prob.A, self.fm.prob.b
        self.ns = cls(A, b, C, d, self.fm, max_iters=max_inner_iters, epsilon=inner_epsilon,
                      suppress_print=suppress_print, max_cg_iters=max_cg_iters, lower_bound=self.lb,
                      upper_bound=self.ub, alpha=alpha, beta=beta, mu=mu, update_slacks_every=update_slacks_every)

    def _eq_tol(self):
        return 1e-4 * self.n

    def _check_inputs(self):
        """LPSolver.py:226-318."""
        c, A, b, C, d = self.c, self.A, self.b, self.C, self.d
        if c is not None and c.ndim != 1:
            raise ValueError("c must be 1-dimensional!")
        dims = []
        if (A is not None) ^ (b is not None):
            raise ValueError("Both A and b must be defined, or neither!")
        if A is not None:
            if A.ndim != 2:
                raise ValueError("A must be 2-dimensional!")
            m, nA = A.shape
            if b.ndim != 1:
                raise ValueError("b must be 1-dimensional!")
            if len(b) != m:
                raise ValueError("A and b must have agreeing dimensions!")
            if c is not None and len(c) != nA:
                raise ValueError("c must have the same number of entries as A has columns!")
            dims.append(nA)
        if (C is not None) ^ (d is not None):
            raise ValueError("Both C and d must be defined, or neither!")
        if C is not None:
            if C.ndim != 2:
                raise ValueError("C must be 2-dimensional!")
            m, nC = C.shape
            if d.ndim != 1:
                raise ValueError("d must be 1-dimensional!")
            if len(d) != m:
                raise ValueError("C and d must have agreeing dimensions!")
            if c is not None and len(c) != nC:
                raise ValueError("c must have the same number of entries as A has columns!")
            dims.append(nC)
        if c is not None:
            dims.append(len(c))
        self.lb, self.ub = _check_bounds(self.lb, self.ub, dims)
        if C is not None and A is not None and C.shape[1] != A.shape[1]:
            raise ValueError("A and C must have the same number of columns!")

    def _check_x0(self, x):
        """LPSolver.py:655-682."""
        if self.lb is not None and (x <= self.lb).any():
            raise ValueError("Initial x must be in domain of problem (all entries greater than lower bound)")
        elif self.ub is not None and (x >= self.ub).any():
            raise ValueError("Initial x must be in domain of problem (all entries less than upper bound)")
        if self.c is not None and len(self.c) != len(x):
            raise ValueError("Initial x must be the same dimension as c!")
        if self.C is not None and self.C.shape[1] != len(x):
            raise ValueError("Initial x must have the same number of columns as C!")
        if self.A is not None and self.A.shape[1] != len(x):
            raise ValueError("Initial x must have the same number of columns as A!")


class QPSolver(_BarrierSolver):
    """min 1/2 x'Px + q'x s.t. Ax = b, Cx <= d, bounds  (QPSolver.py:18-689)."""

    _title = "QPSolver"

    def __init__(self, P=None, q=None, A=None, b=None, C=None, d=None, lower_bound=0, upper_bound=None, t0=0.1,
                 max_outer_iters=20, max_inner_iters=50, phase1_max_inner_iters=500, epsilon=1e-10,
                 inner_epsilon=1e-5, check_cvxpy=True, linear_solve_method="cholesky", max_cg_iters=50,
                 alpha=0.2, beta=0.6, mu=15, suppress_print=False, use_gpu=False, track_loss=False,
                 get_dual_variables=False, phase1_tol=0, phase1_t0=0.01, x0=None, update_slacks_every=0,
                 device=0):
        if P is None:
            raise ValueError("Setting P to None is just an LP! Please use LP solver or set a value to P.")
        self.q, self.P, self.A, self.C, self.b, self.d = q, P, A, C, b, d
        self.lb, self.ub = lower_bound, upper_bound
        self._check_inputs()
        self.equality_constrained = A is not None
        if q is not None:
            self.n = len(q)
        elif A is not None:
            self.n = A.shape[1]
        elif C is not None:
            self.n = C.shape[1]
        else:
            self.n = P.shape[1]
        self.x = x0 if x0 is not None else _default_x0(self.n, self.lb, self.ub)
        self.bounded = self.lb is not None or self.ub is not None
        self._maybe_cvxpy(check_cvxpy, suppress_print)
        self.num_constraints = (len(d) if d is not None else 0) + self.n * (self.lb is not None) + \
            self.n * (self.ub is not None)
        self._common(t0, max_outer_iters, max_inner_iters, epsilon, inner_epsilon, max_cg_iters, alpha, beta, mu,
                     suppress_print, track_loss, linear_solve_method, get_dual_variables, phase1_tol,
                     phase1_max_inner_iters, update_slacks_every, use_gpu, device)
        self.phase1_t0 = phase1_t0
        self._has_ineq = C is not None
        self.eqA, self.eqb = A, b
        self.phase1_solver = None
        if C is not None:
            self.phase1_solver = PhaseOneSolver(C=C, d=d, lower_bound=self.lb, upper_bound=self.ub, x0=self.x,
                                                max_outer_iters=max_outer_iters,
                                                max_inner_iters=phase1_max_inner_iters, epsilon=epsilon,
                                                inner_epsilon=inner_epsilon, alpha=alpha, beta=beta, mu=mu,
                                                suppress_print=suppress_print, n=self.n, tol=phase1_tol,
                                                t0=phase1_t0, update_slacks_every=update_slacks_every,
                                                device=device)
        if self.equality_constrained:
            cls = _infeasible_class(linear_solve_method, False)
        else:
            cls = _feasible_class(linear_solve_method, False)
            if cls is None:
                raise ValueError("No KKT System non-equality-constrained problems! Please choose another solver")
        self.fm = FunctionManagerQP(P=P, q=q, A=A, b=b, C=C, d=d, x0=self.x, lower_bound=self.lb,
                                    upper_bound=self.ub, t=1, n=self.n, solve_method=_solve_method_for(cls),
                                    device=device)
        if A is not None:
            self.eqA_t, self.eqb_t = self.fm.prob.A, self.fm.prob.b
        self.ns = cls(A, b, C, d, self.fm, max_iters=max_inner_iters, epsilon=inner_epsilon,
                      suppress_print=suppress_print, max_cg_iters=max_cg_iters, lower_bound=self.lb,
                      upper_bound=self.ub, alpha=alpha, beta=beta, mu=mu, update_slacks_every=update_slacks_every)

    def _eq_tol(self):
        return 1e-3

    def _check_inputs(self):
        """QPSolver.py:234-330 (vector bounds are checked against q, not the reference's self.c)."""
        q, A, b, C, d, P = self.q, self.A, self.b, self.C, self.d, self.P
        if q is not None and q.ndim != 1:
            raise ValueError("c must be 1-dimensional!")
        dims = []
        if (A is not None) ^ (b is not None):
            raise ValueError("Both A and b must be defined, or neither!")
        if A is not None:
            if A.ndim != 2:
                raise ValueError("A must be 2-dimensional!")
            m, nA = A.shape
            if b.ndim != 1:
                raise ValueError("b must be 1-dimensional!")
            if len(b) != m:
                raise ValueError("A and b must have agreeing dimensions!")
            if q is not None and len(q) != nA:
                raise ValueError("c must have the same number of entries as A has columns!")
            if P.shape[1] != nA:
                raise ValueError("P must have the same number of columns as A!")
            dims.append(nA)
        if (C is not None) ^ (d is not None):
            raise ValueError("Both C and d must be defined, or neither!")
        if C is not None:
            if C.ndim != 2:
                raise ValueError("C must be 2-dimensional!")
            m, nC = C.shape
            if d.ndim != 1:
                raise ValueError("d must be 1-dimensional!")
            if len(d) != m:
                raise ValueError("C and d must have agreeing dimensions!")
            if q is not None and len(q) != nC:
                raise ValueError("q must have the same number of entries as C has columns!")
            if P.shape[1] != nC:
                raise ValueError("P must have the same number of columns as C!")
            dims.append(nC)
        if C is not None and A is not None and C.shape[1] != A.shape[1]:
            raise ValueError("A and C must have the same number of columns!")
        if q is not None:
            dims.append(len(q))
        self.lb, self.ub = _check_bounds(self.lb, self.ub, dims)

    def _check_x0(self, x):
        """QPSolver.py:640-666."""
        if self.lb is not None and (x <= self.lb).any():
            raise ValueError("Initial x must be in domain of problem (all entries greater than lower bound)")
        elif self.ub is not None and (x >= self.ub).any():
            raise ValueError("Initial x must be in domain of problem (all entries less than upper bound)")
        if self.q is not None and len(self.q) != len(x):
            raise ValueError("Initial x must be the same dimension as c!")
        if self.C is not None:
            if (self.C @ x >= self.d).any():
                raise ValueError("Initial x must be in domain of problem (Cx <= d)")
            if self.C.shape[1] != len(x):
                raise ValueError("Initial x must have the same number of columns as C!")
        if self.A is not None and self.A.shape[1] != len(x):
            raise ValueError("Initial x must have the same number of columns as A!")


def normalize_socp_inputs(A, b, c, d, q=None, F=None):
    """SOCPSolver.py:274-382 (Q16): lists, diagonal compression of 2-D A_i, broadcast b/d."""
    if A is None:
        return A, b, c, d
    A = list(A) if isinstance(A, list) else [A]
    m = None
    for i, Ai in enumerate(A):
        Ai = np.asarray(Ai)
        if Ai.ndim > 2:
            raise ValueError("A must be 1- or 2-dimensional!")
        if Ai.ndim == 2:
            m, nA = Ai.shape
            dg = np.diag(Ai).copy()
            off = Ai.copy()
            np.fill_diagonal(off, 0)
            if (off == 0).all():
                A[i] = dg
        else:
            nA = Ai.shape[0]
            m = nA
        if q is not None and len(q) != nA:
            raise ValueError("q must have the same number of entries as A has columns!")
    if b is not None:
        b = list(b) if isinstance(b, list) else [b]
        for bi in b:
            if np.asarray(bi).ndim != 1:
                raise ValueError("b must be 1-dimensional!")
        if len(b) == 1:
            b = b * len(A)
        if len(A) != len(b):
            raise ValueError("Must provide an equal number of A and b")
    if c is not None:
        c = list(c) if isinstance(c, list) else [c]
        for ci in c:
            if np.asarray(ci).ndim != 1:
                raise ValueError("c must be 1-dimensional!")
            if q is not None and len(ci) != len(q):
                raise ValueError("q and c must have the same number of entries!")
    if d is not None:
        d = list(d) if isinstance(d, list) else [d]
        for di in d:
            if not np.isscalar(di):
                raise ValueError("d must be a scalar!")
        if c is not None and len(d) != len(c):
            raise ValueError("Must provide equal number of c and d")
        if len(d) == 1:
            d = d * len(A)
        if len(d) != len(A):
            raise ValueError("Must provide equal number of A and d")
    if c is not None and len(A) != len(c):
        raise ValueError("Must provide equal number of c and A")
    return A, b, c, d


class SOCPSolver(_BarrierSolver):
    """min 1/2 x'Px + q'x s.t. ||A_i x + b_i|| <= c_i'x + d_i, Fx = g, bounds  (SOCPSolver.py:18-833)."""

    _title = "SOCPSolver"

    def __init__(self, P=None, q=None, A=None, b=None, c=None, d=None, F=None, g=None, lower_bound=0,
                 upper_bound=None, t0=0.1, phase1_t0=0.01, max_outer_iters=20, max_inner_iters=50,
                 phase1_max_inner_iters=500, epsilon=1e-10, inner_epsilon=1e-5, check_cvxpy=True,
                 linear_solve_method="cholesky", max_cg_iters=50, alpha=0.2, beta=0.6, mu=15,
                 suppress_print=False, use_gpu=False, try_diag=True, track_loss=False, get_dual_variables=False,
                 phase1_tol=0, use_psd_condition=False, x0=None, update_slacks_every=0, device=0):
        import torch
        if P is not None:
            if P.ndim != 2:
                raise ValueError("P must be 2-dimensional!")
            if P.shape[0] != P.shape[1]:
                raise ValueError("P must be a symmetric, square PSD matrix!")
        if q is not None:
            if q.ndim != 1:
                raise ValueError("q must be q-dimensional!")
            if P is not None and P.shape[1] != len(q):
                raise ValueError("P and q must have the same dimension")
        if F is not None and F.ndim != 2:
            raise ValueError("F must be 2-dimensional!")
        if g is not None:
            if g.ndim != 1:
                raise ValueError("g must be 1-dimensional!")
            if F is not None and len(g) != F.shape[0]:
                raise ValueError("F and g must have agreeing dimensions!")
        A, b, c, d = normalize_socp_inputs(A, b, c, d, q=q, F=F)
        self.P, self.q, self.A, self.b, self.c, self.d, self.F, self.g = P, q, A, b, c, d, F, g
        self.equality_constrained = F is not None
        self.inequality_constrained = A is not None
        if not self.inequality_constrained:
            raise ValueError("No cone contraints detected. Run with LPSolver or QPSolver for better performance.")
        if q is not None:
            self.n = len(q)
        elif P is not None:
            self.n = P.shape[1]
        elif F is not None:
            self.n = F.shape[1]
        else:
            self.n = np.asarray(A[0]).shape[-1]
        dims = [self.n]
        self.lb, self.ub = _check_bounds(lower_bound, upper_bound, dims)
        self.x = x0 if x0 is not None else _default_x0(self.n, self.lb, self.ub)
        self.bounded = self.lb is not None or self.ub is not None
        self._maybe_cvxpy(check_cvxpy, suppress_print)
        self.num_constraints = len(A) + self.n * (self.lb is not None) + self.n * (self.ub is not None)
        self._common(t0, max_outer_iters, max_inner_iters, epsilon, inner_epsilon, max_cg_iters, alpha, beta, mu,
                     suppress_print, track_loss, linear_solve_method, get_dual_variables, phase1_tol,
                     phase1_max_inner_iters, update_slacks_every, use_gpu, device)
        self.phase1_t0 = phase1_t0
        self.use_psd_condition = use_psd_condition
        self._has_ineq = True
        self.eqA, self.eqb = F, g
        cones = ConeData(A, b, c, d, self.n, torch.device("cuda", device))
        self.phase1_solver = PhaseOneSolver(socp=True, socp_params=(A, b, c, d), lower_bound=self.lb,
                                            upper_bound=self.ub, x0=self.x, max_outer_iters=max_outer_iters,
                                            max_inner_iters=phase1_max_inner_iters, epsilon=epsilon,
                                            inner_epsilon=inner_epsilon, alpha=alpha, beta=beta, mu=mu,
                                            suppress_print=suppress_print, n=self.n, tol=phase1_tol,
                                            use_psd_condition=use_psd_condition, t0=phase1_t0,
                                            update_slacks_every=update_slacks_every, device=device,
                                            _cones=cones)
        if self.equality_constrained:
            cls = _infeasible_class(linear_solve_method, False)
        else:
            cls = _feasible_class(linear_solve_method, False)
            if cls is None:
                raise ValueError("No KKT System non-equality-constrained problems! Please choose another solver")
        self.fm = FunctionManagerSOCP(P=P, q=q, A=A, b=b, c=c, d=d, F=F, g=g, lower_bound=self.lb,
                                      upper_bound=self.ub, x0=self.x, t=1, n=self.n,
                                      solve_method=_solve_method_for(cls), device=device, _cones=cones)
        if F is not None:
            self.eqA_t, self.eqb_t = self.fm.prob.A, self.fm.prob.b
        self.ns = cls(F, g, None, None, self.fm, max_iters=max_inner_iters, epsilon=inner_epsilon,
                      suppress_print=suppress_print, max_cg_iters=max_cg_iters, lower_bound=self.lb,
                      upper_bound=self.ub, alpha=alpha, beta=beta, mu=mu, use_psd_condition=use_psd_condition,
                      update_slacks_every=update_slacks_every)

    def _eq_tol(self):
        return 1e-3

    def _check_x0(self, x):
        """SOCPSolver.py:755-807."""
        if self.lb is not None and (x <= self.lb).any():
            raise ValueError("Initial x must be in domain of problem (all entries greater than lower bound)")
        elif self.ub is not None and (x >= self.ub).any():
            raise ValueError("Initial x must be in domain of problem (all entries less than upper bound)")
        if self.q is not None and len(self.q) != len(x):
            raise ValueError("Initial x must be the same dimension as q!")
        if self.P is not None and len(self.P) != len(x):
            raise ValueError("Initial x must be the same dimension as P!")
        if self.F is not None and self.F.shape[1] != len(x):
            raise ValueError("Initial x must have the same number of columns as F!")
