"""Diagnostic: device vs oracle per-Newton-step traces on one golden case (first divergence)."""
import sys

import numpy as np

sys.path[:0] = [".", "interiorpoint-gpu_amd", "tests"]
from golden_io import SOLVE_CASES, load, solver_kwargs  # noqa: E402

import ipm355  # noqa: E402
from oracle import ipm_oracle as O  # noqa: E402

name = sys.argv[1]
z = load(name)
kind = SOLVE_CASES[name]
kw = solver_kwargs(z)
kw["x0"] = z["x_init"].copy()
g = getattr(ipm355, kind + "Solver")(check_cvxpy=False, suppress_print=True, **dict(kw, x0=kw["x0"].copy()))
g.solve()
c = getattr(O, kind + "Solver")(**dict(kw, x0=kw["x0"].copy()))
c.solve()
gt = [t for t in g.ns.trace]
ct = [(t["step"], t.get("stat", t.get("nd", t.get("res")))) for t in c.ns.trace]
print("iters", list(g.inner_iters), list(c.inner_iters))
for i, (a, b) in enumerate(zip(gt, ct)):
    flag = "" if a[0] == b[0] else "  <-- step differs"
    if i < 60 or flag:
        print(i, a, b, flag)
    if flag:
        break
