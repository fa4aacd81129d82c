"""Config 5: SOCPSolver, K=256 second-order cones of 16 rows, n=4096, on
one MI355X.  Reports Newton iterations/s of the real solve (budget of --steps iterations) and a
short parity check against the CPU oracle (same inputs, first outer iteration truncated to a
few Newton steps)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "interiorpoint-gpu_amd")]
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--K", type=int, default=256)
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--parity-steps", type=int, default=3)
args = ap.parse_args()

import torch  # noqa: E402
import ipm355  # noqa: E402
from ipm355 import problems  # noqa: E402

inst = problems.socp_cones(n=args.n, K=args.K, mi=16, seed=0)
kw = dict(problems.SOCP_KWARGS)
x0 = inst.pop("x0")
s = ipm355.SOCPSolver(check_cvxpy=False, suppress_print=True, x0=x0.copy(), **inst, **kw)
s.solve(iteration_budget=2)                       # warmup
s = ipm355.SOCPSolver(check_cvxpy=False, suppress_print=True, x0=x0.copy(), **inst, **kw)
torch.cuda.synchronize()
t0 = time.perf_counter()
s.solve(iteration_budget=args.steps)
torch.cuda.synchronize()
el = time.perf_counter() - t0
iters = int(sum(s.inner_iters))
rec = {"workload": f"SOCPSolver n={args.n}, K={args.K} cones x 16 rows, P=I, x0 strictly feasible",
       "newton_iters": iters, "seconds": el, "iters_per_s": iters / el,
       "hessian_flops_per_iter": (args.K * 16 + 2 * args.K) * args.n * (args.n + 1)}

# parity: a few Newton steps of the first centering step, GPU vs oracle
from oracle import ipm_oracle as O  # noqa: E402
kwp = dict(kw, max_outer_iters=1, max_inner_iters=args.parity_steps)
g = ipm355.SOCPSolver(check_cvxpy=False, suppress_print=True, x0=x0.copy(), **inst, **kwp)
g.solve()
c = O.SOCPSolver(x0=x0.copy(), **inst, **kwp)
c.solve()
xg = np.asarray(g.xstar if g.xstar is not None else g.x, dtype=float)
xc = np.asarray(c.xstar if getattr(c, "xstar", None) is not None else c.x, dtype=float)
rec["parity_steps"] = args.parity_steps
rec["parity_x_rel_err"] = float(np.linalg.norm(xg - xc) / np.linalg.norm(xc))
rec["parity_iters"] = [list(map(int, g.inner_iters)), list(map(int, c.inner_iters))]
print(json.dumps(rec), flush=True)
