"""Config 5's cone shape pinned to the REFERENCE itself (build container only).

    PYTHONDONTWRITEBYTECODE=1 OPENBLAS_NUM_THREADS=4 python tests/golden/make_golden_m5ref.py [n]

M5 proper (n=4096, K=256) needs 2 K n^2 doubles of reference cone caches (64 GiB,
FunctionManager.py:869-894), more than this container holds.  At n=2048 with the SAME cone count and
shape (K=256 cones of 16 rows, P=I, no bounds, strictly feasible x0, test_SOCP kwargs
testSolver.py:924-945) the caches are 16 GiB: this script runs the reference SOCPSolver to
completion there and records what tests/test_gpu_large.py::test_m5ref_socp_full_solve checks:
x*, value, inner iteration counts, every accepted backtracking step size and Newton decrement
(NewtonSolver.py:93-133, recorded by wrapping backtrack_search as make_golden_large.py does).
Envelope: one re-run with every d_i perturbed by 1e-15 relative.  Inputs come from
ipm355.problems.socp_cones(seed=0) (numpy Generator normals: the GPU box regenerates them bit for
bit; the fixture keeps only their digest), except d, which is a BLAS norm and is stored.
"""
from __future__ import annotations

import os
import sys
import time
import types

os.environ.setdefault("OPENBLAS_NUM_THREADS", "4")
sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "interiorpoint-gpu_amd"))
sys.modules.setdefault("cvxpy", types.ModuleType("cvxpy"))
sys.path.insert(0, REF)

import numpy as np  # noqa: E402

import NewtonSolver as RNS  # noqa: E402
from SOCPSolver import SOCPSolver as RefSOCP  # noqa: E402

from ipm355 import problems  # noqa: E402

STEPS, NDS = [], []


def _wrap():
    orig = RNS.NewtonSolver.backtrack_search

    def rec(self, x, xstep, t, gradf):
        s = orig(self, x, xstep, t, gradf)
        STEPS.append(float(s))
        NDS.append(float(-gradf.dot(xstep) / 2))
        return s
    RNS.NewtonSolver.backtrack_search = rec


def digest(inst):
    return problems.input_digest({"A": np.stack(inst["A"]), "b": np.stack(inst["b"]), "c": np.stack(inst["c"]),
                                  "q": inst["q"]})


def run(inst, x0, kw):
    STEPS.clear()
    NDS.clear()
    s = RefSOCP(check_cvxpy=False, suppress_print=True, x0=x0.copy(),
                **{k: ([np.array(a, copy=True) if isinstance(a, np.ndarray) else a for a in v] if isinstance(v, list) else v)
                   for k, v in inst.items()},
                **kw)
    t0 = time.time()
    val = s.solve()
    return dict(value=float(val), xstar=np.array(s.xstar, copy=True), inner=list(s.inner_iters),
                steps=list(STEPS), nds=list(NDS), seconds=time.time() - t0)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    K, mi = 256, 16
    _wrap()
    inst = problems.socp_cones(n=n, K=K, mi=mi, seed=0)
    x0 = inst.pop("x0")
    kw = dict(problems.SOCP_KWARGS)
    base = run(inst, x0, kw)
    print(f"m5ref n={n} base: {base['seconds']:.0f}s value={base['value']!r} inner={base['inner']} "
          f"steps={len(base['steps'])}", flush=True)
    rng = np.random.default_rng(1234)
    pert = dict(inst)
    pert["d"] = [float(v * (1 + 1e-15 * rng.standard_normal())) for v in inst["d"]]
    p = run(pert, x0, kw)
    stable = p["steps"] == base["steps"]
    wx = float(np.linalg.norm(p["xstar"] - base["xstar"]) / np.linalg.norm(base["xstar"]))
    wv = abs(p["value"] - base["value"]) / abs(base["value"])
    wnd = np.zeros(len(base["nds"]))
    if len(p["nds"]) == len(base["nds"]):
        b = np.array(base["nds"])
        wnd = np.abs(np.array(p["nds"]) - b) / np.maximum(np.abs(b), 1e-300)
    print(f"m5ref perturbed: {p['seconds']:.0f}s inner={p['inner']} stable={stable} x* spread {wx:.1e} "
          f"value spread {wv:.1e}", flush=True)
    np.savez_compressed(os.path.join(HERE, f"m5ref_socp_n{n}.npz"),
                        spec=np.array(repr(dict(gen="socp_cones", n=n, K=K, mi=mi, seed=0))),
                        digest=np.array(digest(inst)), d=np.array(inst["d"]), kwargs=np.array(repr(kw)),
                        value=np.array(base["value"]), xstar=base["xstar"], inner_iters=np.array(base["inner"]),
                        trace_step=np.array(base["steps"]), trace_nd=np.array(base["nds"]),
                        sens_steps_stable=np.array(stable), sens_xstar_rel=np.array(wx), sens_value_rel=np.array(wv),
                        sens_nd_rel=wnd, pert_inner_iters=np.array(p["inner"]),
                        pert_trace_step=np.array(p["steps"]), ref_seconds=np.array(base["seconds"]))


if __name__ == "__main__":
    main()
