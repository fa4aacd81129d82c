"""LassoSolver (batched ADMM): the oracle against the reference's own outputs
(CPU), and the HIP path against the same fixtures (-m gpu).

Fixtures: tests/golden/lasso_*.npz, written by tests/golden/make_golden_lasso.py running the
reference LassoSolver (inputs regenerated here from ipm355.problems.lasso_instance, digest-checked).
Bars (north star: x* within 1e-6 relative of the reference): X within 1e-6 relative, iteration
counts identical (the reference's own count is stable under a 1e-15 perturbation of b in every
fixture), solutions and the per-iteration loss (gaps) within 1e-9 relative.
"""
import ast
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN

X_RTOL = 1e-6
VAL_RTOL = 1e-9

CASES = ["lasso_demo", "lasso_regpath", "lasso_positive", "lasso_chunks", "lasso_testsolver", "lasso_n1024"]


def _case(name):
    from ipm355 import problems
    z = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    A, b, reg, kw = problems.lasso_instance(name)
    assert problems.input_digest(dict(A=A, b=b, reg=reg)) == str(z["digest"])
    assert ast.literal_eval(str(z["kwargs"])) == kw
    return z, A, b, reg, kw


def _rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - b) / max(np.linalg.norm(b), 1e-300))


def _check(name, A, z, X, sol, gaps, iters):
    print(f"[{name}] iters {iters} (ref {z['iters'].tolist()}), X rel {_rel(X, z['X']):.2e}, "
          f"solutions rel {_rel(sol, z['solutions']):.2e}")
    assert np.array_equal(np.array(iters), z["iters"])
    assert _rel(X, z["X"]) <= X_RTOL
    assert _rel(sol, z["solutions"]) <= VAL_RTOL
    assert np.asarray(gaps).shape == z["gaps"].shape
    assert _rel(gaps, z["gaps"]) <= VAL_RTOL if np.any(z["gaps"]) else not np.any(gaps)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    from oracle import lasso_oracle as O
    z, A, b, reg, kw = _case(name)
    A0 = A.copy()
    X, sol, gaps, iters = O.LassoSolver(A, b, reg=reg, **kw).solve()
    _check(name, A, z, X, sol, gaps, iters)
    if kw["normalize_A"]:
        np.testing.assert_allclose(np.abs(A0).max(0) / np.abs(A).max(0), z["A_colscale"], rtol=1e-14)


def test_lasso_args_layout():
    from ipm355.lasso import LassoArgs
    # 4 int64 + (ptr, int64, ptr, int64, ptr) + 6 ptr + 4 double + 10 int32 + 9 pointer/int64 fields
    # + qs_blocked (int32, padded to the struct's 8-byte alignment)
    assert ctypes.sizeof(LassoArgs) == 32 + 40 + 48 + 32 + 40 + 72 + 8
    assert LassoArgs.qs_blocked.offset == 32 + 40 + 48 + 32 + 40 + 72


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_device_matches_reference(name):
    import ipm355
    z, A, b, reg, kw = _case(name)
    A0 = A.copy()
    s = ipm355.LassoSolver(A, b, reg=reg, **kw)
    X, sol, gaps, iters = s.solve()
    _check(name, A, z, X, sol, gaps, iters)
    if kw["normalize_A"]:   # the caller's A is divided in place by its column std
        np.testing.assert_allclose(np.abs(A0).max(0) / np.abs(A).max(0), z["A_colscale"], rtol=1e-14)


@pytest.mark.gpu
def test_device_reference_errors_and_helpers():
    import ipm355
    from oracle import lasso_oracle as O
    z, A, b, reg, kw = _case("lasso_positive")
    with pytest.raises(AttributeError, match="AtA_cache"):
        ipm355.LassoSolver(A.copy(), b, reg=reg, **dict(kw, add_bias=False))
    with pytest.raises(TypeError):
        ipm355.LassoSolver(A.copy(), b, reg=1.0, **kw)
    kw2 = dict(kw, normalize_A=False, positive=False)
    s = ipm355.LassoSolver(A.copy(), b, reg=reg, **kw2)
    o = O.LassoSolver(A.copy(), b, reg=reg, **kw2)
    s.solve()
    o.solve()
    v = np.random.default_rng(3).normal(size=(s.n, s.num_samples))
    np.testing.assert_array_equal(s.prox(v, s.eta), o.prox(v, o.eta))
    # objective(): the reference's CPU branch sums alpha without |.| unless positive (LassoSolver.py:505-510)
    f_ref = 1 / (2 * o.m) * ((o.A @ o.alpha - o.b) ** 2).sum(axis=0) + o.reg * o.alpha[1:].sum(axis=0)
    assert _rel(s.objective(), f_ref) <= 1e-9
