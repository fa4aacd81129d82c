"""Time the oracle (oracle/ipm_oracle.py) beside the REFERENCE itself on the same instance, same
kwargs, same BLAS thread count (the CPU baseline bench.py reports is the oracle, so
it must run at the reference's own speed, within +-10 %).  Build container only -- it imports
/root/reference read-only (with an empty cvxpy stub, as tests/golden/make_golden*.py do); the GPU box
never sees the reference.

    PYTHONDONTWRITEBYTECODE=1 OPENBLAS_NUM_THREADS=8 python scripts/oracle_vs_reference.py [n m]

Workload: M2 (QPSolver.solve() on the seeded dense QP n=2048, m=512, test_QP kwargs; phase 1 +
barrier phase, testSolver.py:563-582), solved to completion by each, twice, alternating; reports
seconds per Newton iteration and the ratio.  Writes profiles/oracle_vs_reference.json.
"""
from __future__ import annotations

import json
import os
import sys
import time
import types

os.environ.setdefault("OPENBLAS_NUM_THREADS", "8")
sys.dont_write_bytecode = True
REF = "/root/reference"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "interiorpoint-gpu_amd")]
sys.modules.setdefault("cvxpy", types.ModuleType("cvxpy"))

import numpy as np  # noqa: E402

from ipm355 import problems  # noqa: E402
from oracle import ipm_oracle as O  # noqa: E402

sys.path.insert(0, REF)
from QPSolver import QPSolver as RefQP  # noqa: E402


def newton_iters(s):
    ph = getattr(s, "phase1_solver", None) or getattr(s, "phase1", None)   # (reference / oracle names)
    return int(sum(s.inner_iters)) + (int(sum(ph.inner_iters)) if ph is not None else 0)


def run(kind, inst, kw):
    args = {k: (np.array(v, copy=True) if isinstance(v, np.ndarray) else v) for k, v in inst.items()}
    t0 = time.perf_counter()
    if kind == "reference":
        s = RefQP(check_cvxpy=False, suppress_print=True, **args, **kw)
    else:
        s = O.QPSolver(**args, **kw)
    val = s.solve()
    el = time.perf_counter() - t0
    return dict(seconds=el, iters=newton_iters(s), value=float(val), xstar=np.asarray(s.xstar))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    inst = problems.qp_ineq_box(n, m, seed=0, grid=True)
    kw = dict(problems.QP_KWARGS)
    res = {"reference": [], "oracle": []}
    for rep in range(2):
        for kind in ("reference", "oracle"):
            r = run(kind, inst, kw)
            res[kind].append(r)
            print(f"{kind:9s} rep {rep}: {r['iters']} Newton iters in {r['seconds']:.1f} s = "
                  f"{r['seconds'] / r['iters'] * 1e3:.1f} ms/iter, value {r['value']!r}", flush=True)
    per = {k: min(r["seconds"] / r["iters"] for r in v) for k, v in res.items()}
    xr, xo = res["reference"][0]["xstar"], res["oracle"][0]["xstar"]
    out = {
        "workload": f"QPSolver.solve() dense QP n={n}, m={m}, seed 0, test_QP kwargs (M2), full solve",
        "blas_threads": int(os.environ["OPENBLAS_NUM_THREADS"]),
        "ms_per_newton_iter": {k: v * 1e3 for k, v in per.items()},
        "oracle_over_reference_time": per["oracle"] / per["reference"],
        "iters": {k: [r["iters"] for r in v] for k, v in res.items()},
        "xstar_rel_diff": float(np.linalg.norm(xo - xr) / np.linalg.norm(xr)),
        "within_10pct": abs(per["oracle"] / per["reference"] - 1.0) <= 0.10,
    }
    print(json.dumps(out, indent=1))
    with open(os.path.join(REPO, "profiles", "oracle_vs_reference.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
