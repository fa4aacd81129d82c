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


GRID = 2.0 ** -10


def _u(rng, size, grid):
    """U(-2, 2); with ``grid`` the values are rounded to multiples of 2^-10.  Every product of two
    such values is a multiple of 2^-20 and every dot product used by the generators stays below
    2^15, so it needs at most 35 significand bits: P = Pp'Pp and d = C x_f + 1 are then EXACT in
    fp64 whatever BLAS, thread count or summation order computes them.  The large parity fixtures
    (tests/golden/make_golden_large.py) use this so that the GPU box regenerates bit-identical
    inputs without shipping them."""
    a = rng.uniform(-2, 2, size=size)
    return np.round(a / GRID) * GRID if grid else a


def lp_ineq_box(n=200, m=50, seed=0, grid=False, with_xf=False):
    """M1b / M3-LP: min c'x s.t. Cx <= d, -3 <= x <= 3 with d = C x_f + 1 (strictly feasible)."""
    rng = np.random.default_rng(seed)
    C = _u(rng, (m, n), grid)
    xf = _u(rng, n, grid)
    d = C @ xf + 1
    c = _u(rng, n, grid)
    out = dict(c=c, C=C, d=d, lower_bound=-3, upper_bound=3)
    if with_xf:
        out["xf"] = xf
    return out


def qp_ineq_box(n=2048, m=512, seed=0, grid=False, with_xf=False, gram=None):
    """M2 / M3-QP / M4: P = Pp'Pp + I (Pp: floor(0.8 n) x n), q, Cx <= d = C x_f + 1, -3 <= x <= 3.

    ``gram(Pp) -> Pp'Pp`` may be supplied (e.g. a device GEMM for n=8192); with ``grid`` any exact
    product gives the same P bit for bit."""
    rng = np.random.default_rng(seed)
    Pp = _u(rng, (int(0.8 * n), n), grid)
    P = gram(Pp) if gram is not None else Pp.T @ Pp
    del Pp
    P[np.diag_indices(n)] += 1.0
    q = _u(rng, n, grid)
    C = _u(rng, (m, n), grid)
    xf = _u(rng, n, grid)
    d = C @ xf + 1
    out = dict(P=P, q=q, C=C, d=d, lower_bound=-3, upper_bound=3)
    if with_xf:
        out["xf"] = xf
    return out


def input_digest(inst):
    """sha256 over the array inputs of an instance (sorted keys): proves regenerated inputs are the
    ones a fixture was computed on."""
    import hashlib
    h = hashlib.sha256()
    for k in sorted(inst):
        v = inst[k]
        if isinstance(v, np.ndarray):
            h.update(k.encode())
            h.update(np.ascontiguousarray(v, dtype=np.float64).tobytes())
    return h.hexdigest()


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


def _g(a):
    """round to multiples of 2^-10 (products and the dot products below stay exact in fp64)"""
    return np.round(a / GRID) * GRID


LASSO_CASES = ("lasso_demo", "lasso_regpath", "lasso_positive", "lasso_chunks", "lasso_testsolver", "lasso_n1024")


def lasso_instance(name):
    """LassoSolver instances in the reference's own usage patterns -> (A, b, reg, kwargs).

    demo.ipynb cells 47-48 (m=500, n=150, 30 problems, bias, normalised A, loss tracked; positive and
    chunked variants), cells 53-54 (one b, 50 regularisation strengths), testSolver.py:1057-1160
    (test_Lasso: rows = 3 x 0.8 n, 30 problems, reg = 0.05 + 0.01 N).  Values sit on the 2^-10 grid so
    that b = A x_true + noise is exact whatever BLAS computes it (the GPU box regenerates the inputs
    bit for bit; the fixtures store only their digest)."""
    rng = np.random.default_rng(dict(zip(LASSO_CASES, range(7, 7 + len(LASSO_CASES))))[name])
    base = dict(rho=0.4, max_iters=1000, check_stop=10, add_bias=True, normalize_A=False, positive=False,
                compute_loss=False, adaptive_rho=False, eps_abs=1e-6, eps_rel=1e-6, use_gpu=False, num_chunks=0,
                check_cvxpy=False)

    def sparse_x(n, S, nnz):
        xt = np.zeros((n, S))
        xt[np.unravel_index(rng.integers(0, n * S, nnz), (n, S))] = _g(rng.uniform(0, 50, nnz))
        return xt
    if name in ("lasso_demo", "lasso_positive", "lasso_chunks"):
        m, n, S = 500, 150, 30
        A = _g(rng.random((m, n)))
        b = A @ sparse_x(n, S, 1000) + _g(rng.standard_normal((m, S)))
        reg = 0.05 + 0.01 * rng.standard_normal(S)
        kw = dict(base, normalize_A=True, compute_loss=True, eps_rel=1e-4)
        if name == "lasso_positive":
            kw.update(positive=True, compute_loss=False, eps_abs=1e-4, eps_rel=3e-2, check_stop=5)
        if name == "lasso_chunks":
            kw.update(num_chunks=3, normalize_A=False)
        return A, b, reg, kw
    if name == "lasso_regpath":
        m, n = 800, 400
        A = _g(rng.random((m, n)))
        b = A @ sparse_x(n, 1, 10000) + _g(rng.standard_normal((m, 1)))
        return A, b, np.logspace(-5, 2, 50), dict(base, rho=0.004, max_iters=3000, check_stop=100)
    n = 400 if name == "lasso_testsolver" else 1024
    rows, S = 3 * int(0.8 * n), 30
    A = _g(rng.random((rows, n)))
    b = A @ sparse_x(n, S, int(n * S / 4)) + _g(rng.standard_normal((rows, S)))
    reg = 0.05 + 0.01 * rng.standard_normal(S)
    return A, b, reg, dict(base, max_iters=1000 if name == "lasso_testsolver" else 400)


LP_NPY_ORDER = ("c", "A", "b", "C", "d", "upper_bound", "lower_bound")


def save_lp_npy(path, c, A, b, C, d, upper_bound, lower_bound):
    """The reference's sparse-LP file format (testSolver.py:278-300): seven arrays written one
    after another into ONE .npy file -- c, A, b, C, d, upper bound, lower bound (dense arrays; the
    MIPLIB instances aflow40b / 30n20b8 ship in it)."""
    with open(path, "wb") as f:
        for a in (c, A, b, C, d, upper_bound, lower_bound):
            np.save(f, np.asarray(a, dtype=np.float64), allow_pickle=False)


def load_lp_npy(path):
    """Read a file in that format -> LPSolver kwargs (c, A, b, C, d, upper_bound, lower_bound)."""
    with open(path, "rb") as f:
        vals = [np.load(f, allow_pickle=False) for _ in LP_NPY_ORDER]
    return dict(zip(LP_NPY_ORDER, vals))


def lp_miplib_like(n=600, p=120, m=240, density=0.03, seed=0):
    """A MIPLIB-style LP relaxation in the format above (the reference's blobs are absent here):
    sparse 0/1/integer-coefficient equality rows A x = b and inequality rows C x <= d, box bounds
    per variable, feasible by construction (x_f strictly inside the bounds, d = C x_f + slack)."""
    rng = np.random.default_rng(seed)

    def sparse(rows):
        M = (rng.random((rows, n)) < density) * rng.integers(1, 6, (rows, n)).astype(float)
        for i in range(rows):                       # at least two nonzeros per row
            M[i, rng.choice(n, 2, replace=False)] = rng.integers(1, 6, 2)
        return M
    lb = np.zeros(n)
    ub = rng.integers(1, 10, n).astype(float)
    xf = lb + (ub - lb) * rng.uniform(0.2, 0.8, n)
    A = sparse(p)
    C = sparse(m) * rng.choice([-1.0, 1.0], (m, 1))
    return dict(c=rng.integers(-20, 20, n).astype(float), A=A, b=A @ xf, C=C, d=C @ xf + rng.uniform(0.5, 2.0, m),
                upper_bound=ub, lower_bound=lb)


def instance_seeds(total, rank, world):
    """M4 partitioning: rank r takes instances r::world."""
    return list(range(rank, total, world))
