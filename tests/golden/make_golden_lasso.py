"""Golden vectors for the batched-ADMM LassoSolver, made by running the REFERENCE itself (build
container only; ~1-2 min).

    PYTHONDONTWRITEBYTECODE=1 OPENBLAS_NUM_THREADS=1 python tests/golden/make_golden_lasso.py

The reference (LassoSolver.py) is imported read-only with an empty ``cvxpy`` stub module (cvxpy is
only touched when ``check_cvxpy=True``).  Instances: ipm355.problems.lasso_instance (the
reference's own usage patterns, seeded, values on a 2^-10 grid so the GPU box regenerates them bit
for bit).  Stored: the digest of the inputs, the kwargs, X, solutions, gaps, iterations, the column
scale normalize_A applied to the caller's A (it divides the array in place), and the spread of X
under a 1e-15 relative perturbation of b (the reference's own envelope).
"""
from __future__ import annotations

import os
import sys
import types

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.modules.setdefault("cvxpy", types.ModuleType("cvxpy"))
sys.path.insert(0, REF)

import numpy as np  # noqa: E402

from LassoSolver import LassoSolver as RefLasso  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "interiorpoint-gpu_amd"))
from ipm355 import problems  # noqa: E402


def run(A, b, reg, kw):
    A = np.array(A, copy=True)
    s = RefLasso(A, np.array(b, copy=True), reg=np.array(reg, copy=True), **kw)
    X, sol, gaps, iters = s.solve()
    return A, np.array(X), np.array(sol), np.array(gaps), iters


def make(name):
    A, b, reg, kw = problems.lasso_instance(name)
    An, X, sol, gaps, iters = run(A, b, reg, kw)
    rng = np.random.default_rng(1234)
    bp = b * (1 + 1e-15 * rng.standard_normal(b.shape))
    _, Xp, solp, _, itp = run(A, bp, reg, kw)
    out = dict(digest=np.array(problems.input_digest(dict(A=A, b=b, reg=reg))), kwargs=np.array(repr(kw)),
               A_colscale=np.abs(A).max(axis=0) / np.abs(An).max(axis=0), X=X, solutions=sol, gaps=gaps,
               iters=np.array(iters), sens_X_rel=np.array(np.linalg.norm(Xp - X) / np.linalg.norm(X)),
               sens_sol_rel=np.array(np.max(np.abs(solp - sol) / np.abs(sol))),
               sens_iters_stable=np.array(np.array_equal(np.array(itp), np.array(iters))))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(f"{name}: iters={iters} sens X {float(out['sens_X_rel']):.1e} stable={bool(out['sens_iters_stable'])}",
          flush=True)


if __name__ == "__main__":
    for c in sys.argv[1:] or problems.LASSO_CASES:
        make(c)
