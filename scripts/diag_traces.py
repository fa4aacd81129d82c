"""Diagnostic: per-iteration trajectory of the HIP path vs the CPU oracle on golden cases."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "interiorpoint-gpu_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402

import ipm355  # noqa: E402
from golden_io import SOLVE_CASES, load, solver_kwargs  # noqa: E402
from oracle import ipm_oracle as O  # noqa: E402

names = sys.argv[1:] or ["lp_eq_box", "lp_eq_ineq", "qp_eq_phase1", "socp_group_lasso"]
for name in names:
    z = load(name)
    kw = solver_kwargs(z)
    kw["x0"] = z["x_init"].copy()
    kind = SOLVE_CASES[name]
    g = {"LP": ipm355.LPSolver, "QP": ipm355.QPSolver, "SOCP": ipm355.SOCPSolver}[kind](
        check_cvxpy=False, suppress_print=True, **{k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in kw.items()})
    g.solve()
    o = {"LP": O.LPSolver, "QP": O.QPSolver, "SOCP": O.SOCPSolver}[kind](**kw)
    o.solve()
    gt = (g.phase1_solver.phase1_ns.trace if g.phase1_solver is not None and o.phase1_iters else []) + g.ns.trace
    ot = [(t["step"], t.get("nd", t.get("res"))) for t in ((o.phase1.ns.trace if o.phase1_iters else []) + o.ns.trace)]
    print(f"== {name}: gpu inner {list(g.inner_iters)} oracle {list(o.inner_iters)}  "
          f"x* rel {np.linalg.norm(g.xstar - o.xstar) / np.linalg.norm(o.xstar):.2e}  "
          f"value {g.value!r} vs {o.value!r}")
    first = None
    for i, (a, b) in enumerate(zip(gt, ot)):
        if a[0] != b[0]:
            first = i
            break
    print(f"   traces: gpu {len(gt)} oracle {len(ot)} first step mismatch at {first}")
    if first is not None:
        for i in range(max(0, first - 3), min(len(gt), len(ot), first + 4)):
            print(f"   it {i:4d}  gpu step {gt[i][0]:.6e} stat {gt[i][1]!s:>24}   oracle step {ot[i][0]:.6e} stat {ot[i][1]!s:>24}")
