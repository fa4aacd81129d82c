import sys
sys.path[:0] = ["/root/repo", "/root/repo/tests", "/root/repo/interiorpoint-gpu_amd"]
import numpy as np
from golden_io import load, solver_kwargs
import ipm355
from oracle import ipm_oracle as O
z = load("lp_eq_ineq")
for m in ["cholesky", "np_solve"]:
    kw = solver_kwargs(z); kw["x0"] = z["x_init"].copy(); kw["linear_solve_method"] = m
    s = ipm355.LPSolver(check_cvxpy=False, suppress_print=True, **kw); v = s.solve()
    c = O.LPSolver(**kw); vc = c.solve()
    print(m, "dev", v, list(s.inner_iters), "cpu", vc, list(c.inner_iters))
    print("  dev", [(round(t[0], 6), float("%.6g" % t[1])) for t in s.ns.trace])
    print("  cpu", [(round(t["step"], 6), float("%.6g" % t["res"])) for t in c.ns.trace])
