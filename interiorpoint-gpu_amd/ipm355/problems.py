"""Seeded synthetic problem generators for the BASELINE.json configurations.

Shapes and solver kwargs follow SURVEY.md §8(d), which derives them from the
reference's own generators (``testSolver.py:104-148`` for LP, ``:499-582`` for
QP, ``:860-945`` for SOCP) and the demo notebook (``demo.ipynb`` cells 4-8).
All arrays are fp64, row-major (C-contiguous).  Generation is pure NumPy and
is NOT part of the timed region of any benchmark.
"""
from __future__ import annotations

import numpy as np

# testSolver.py:130-148 (test_LP kwargs)
LP_KWARGS = dict(epsilon=1e-4, mu=15, t0=1, max_inner_iters=20, max_outer_iters=10, beta=0.5, alpha=0.05)
# testSolver.py:563-582 (test_QP kwargs)
QP_KWARGS = dict(epsilon=1e-8, mu=15, t0=0.01, max_inner_iters=100, max_outer_iters=10, beta=0.6, alpha=0.4)
# testSolver.py:924-945 (test_SOCP kwargs)
SOCP_KWARGS = dict(epsilon=1e-4, mu=15, t0=0.1, max_inner_iters=500, max_outer_iters=10, beta=0.5, alpha=0.05)


def lp_eq_box(n=200, p=50, seed=0):
    """M1a (demo.ipynb cells 4-8 pattern): min c'x s.t. Ax = b, 0 <= x <= 3.

    Solved with update_slacks_every=5 -> NewtonSolverCholeskyDiagonalInfeasibleStart."""
    rng = np.random.default_rng(seed)
    A = rng.normal(size=(p, n))
    b = A @ np.abs(rng.normal(size=n))
    c = rng.normal(size=n)
    return dict(c=c, A=A, b=b, lower_bound=0, upper_bound=3)


def lp_ineq_box(n=200, m=50, seed=0):
    """M1b / M3-LP: min c'x s.t. Cx <= d, -3 <= x <= 3 with d = C x_f + 1 (strictly feasible)."""
    rng = np.random.default_rng(seed)
    C = rng.uniform(-2, 2, size=(m, n))
    xf = rng.uniform(-2, 2, size=n)
    d = C @ xf + 1
    c = rng.uniform(-2, 2, size=n)
    return dict(c=c, C=C, d=d, lower_bound=-3, upper_bound=3)


def qp_ineq_box(n=2048, m=512, seed=0):
    """M2 / M3-QP / M4: P = Pp'Pp + I (Pp: floor(0.8 n) x n), q, Cx <= d = C x_f + 1, -3 <= x <= 3."""
    rng = np.random.default_rng(seed)
    Pp = rng.uniform(-2, 2, size=(int(0.8 * n), n))
    P = Pp.T @ Pp + np.eye(n)
    del Pp
    q = rng.uniform(-2, 2, size=n)
    C = rng.uniform(-2, 2, size=(m, n))
    xf = rng.uniform(-2, 2, size=n)
    d = C @ xf + 1
    return dict(P=P, q=q, C=C, d=d, lower_bound=-3, upper_bound=3)


def socp_cones(n=4096, K=256, mi=16, seed=0, eq=0):
    """M5: min 1/2 x'x + q'x s.t. ||A_i x + b_i|| <= c_i'x + d_i (K cones of mi rows),
    d_i = ||A_i x0 + b_i|| - c_i'x0 + 1 so that x0 is strictly feasible (phase 1 skipped).
    eq > 0 adds F x = g with g = F x0 (infeasible-start Newton)."""
    rng = np.random.default_rng(seed)
    x0 = rng.normal(size=n)
    A = [rng.normal(size=(mi, n)) for _ in range(K)]
    b = [rng.normal(size=mi) for _ in range(K)]
    c = [rng.normal(size=n) for _ in range(K)]
    d = [float(np.linalg.norm(A[i] @ x0 + b[i]) - c[i] @ x0 + 1) for i in range(K)]
    q = rng.normal(size=n)
    out = dict(P=np.eye(n), q=q, A=A, b=b, c=c, d=d, lower_bound=None, upper_bound=None, x0=x0)
    if eq:
        F = rng.normal(size=(eq, n))
        out.update(F=F, g=F @ x0)
    return out


def instance_seeds(total, rank, world):
    """M4 partitioning: rank r takes instances r::world."""
    return list(range(rank, total, world))
