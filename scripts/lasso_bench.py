"""LassoSolver (batched ADMM) throughput on the device vs the NumPy oracle.

    python scripts/lasso_bench.py [n] [problems] [iters]

Instance: the test_Lasso pattern (testSolver.py:1057-1160): rows = 3 x 0.8 n, `problems` right-hand
sides with their own regularisation, bias column.  eps_abs = eps_rel = 0 so every run takes exactly
`iters` ADMM iterations (the stopping test is still evaluated every check_stop iterations).
Reported: ADMM iterations/s (setup -- the AtA GEMM, Cholesky and inverse -- excluded), the fused
iteration kernel's achieved fp64 TFLOP/s (2 n^2 S per iteration) and HBM GB/s (8 n^2 bytes of Q per
iteration), and the oracle (NumPy/OpenBLAS) on the same instance for a bounded number of iterations.
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "interiorpoint-gpu_amd")]
import numpy as np  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
S = int(sys.argv[2]) if len(sys.argv) > 2 else 30
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 500
rng = np.random.default_rng(0)
rows = 3 * int(0.8 * n)
A = rng.random((rows, n))
xt = np.zeros((n, S))
nnz = int(n * S / 4)
xt[np.unravel_index(rng.integers(0, n * S, nnz), (n, S))] = rng.uniform(0, 50, nnz)
b = A @ xt + rng.standard_normal((rows, S))
reg = 0.05 + 0.01 * rng.standard_normal(S)
kw = dict(reg=reg, rho=0.4, max_iters=iters, check_stop=10, add_bias=True, eps_abs=0.0, eps_rel=0.0, check_cvxpy=False)

import torch  # noqa: E402
import ipm355  # noqa: E402

s = ipm355.LassoSolver(A.copy(), b, **kw)
s.solve()                                   # warm-up
torch.cuda.synchronize()
t0 = time.perf_counter()
X, sol, gaps, it = s.solve()
torch.cuda.synchronize()
el = time.perf_counter() - t0
N = n + 1
rec = {"metric": "LassoSolver ADMM iterations/s", "n": N, "problems": S, "rows": rows, "iters": it,
       "seconds": el, "iters_per_s": it / el, "us_per_iter": el / it * 1e6,
       "achieved_tflops_iteration": 2.0 * N * N * S * it / el / 1e12,
       "achieved_gbs_Q": 8.0 * N * N * it / el / 1e9}
# CPU oracle, bounded sample
from oracle import lasso_oracle as O  # noqa: E402
ci = max(5, min(50, iters))
o = O.LassoSolver(A.copy(), b, **dict(kw, max_iters=ci))
t0 = time.perf_counter()
o.solve()
ce = time.perf_counter() - t0
rec["cpu_baseline"] = {"iters_per_s": ci / ce, "iters": ci, "seconds": ce, "kind": "port",
                       "threads": os.environ.get("OMP_NUM_THREADS", str(os.cpu_count()))}
print(json.dumps(rec), flush=True)
