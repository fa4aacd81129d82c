"""M5 (SOCPSolver, n=4096, 256 cones of 16 rows) solved to COMPLETION by the oracle's stacked-cone
restatement (build container only; a few minutes per run).

    PYTHONDONTWRITEBYTECODE=1 OPENBLAS_NUM_THREADS=2 python tests/golden/make_golden_m5.py

The reference's own FunctionManagerSOCP caches 2 K n^2 doubles (64 GiB at K=256, n=4096,
FunctionManager.py:834-1162), so it cannot run this size; the oracle (oracle/ipm_oracle.py
SOCPSolver) is pinned to the reference by the small SOCP fixtures (socp_small*, socp_phase1,
socp_group_lasso incl. the demo.ipynb FSTAR known answer: tests/test_oracle_golden.py), and this
fixture carries its full-solve result at the BASELINE size: x*, value, inner iteration counts,
every accepted step size and Newton decrement.  Envelope: one re-run with d perturbed by 1e-15
(relative).  ``d`` itself is stored (it comes from a BLAS norm, whose last bits may differ between
CPUs); the GPU test uses the stored d and checks the digest of the seeded A, b, c, q.
"""
from __future__ import annotations

import os
import sys
import time

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "interiorpoint-gpu_amd")]

import numpy as np  # noqa: E402

from ipm355 import problems  # noqa: E402
from oracle import ipm_oracle as O  # noqa: E402


def digest(inst):
    return problems.input_digest({"A": np.stack(inst["A"]), "b": np.stack(inst["b"]), "c": np.stack(inst["c"]),
                                  "q": inst["q"]})


def run(inst, x0, kw):
    c = O.SOCPSolver(x0=x0.copy(), **{k: (list(v) if isinstance(v, list) else v) for k, v in inst.items()}, **kw)
    t0 = time.time()
    val = c.solve()
    steps = [t["step"] for t in c.ns.trace]
    nds = [np.nan if t["nd"] is None else t["nd"] for t in c.ns.trace]
    return dict(value=float(val), xstar=np.asarray(c.xstar), inner=list(c.inner_iters), steps=steps, nds=nds,
                seconds=time.time() - t0)


def main():
    inst = problems.socp_cones(n=4096, K=256, mi=16, seed=0)
    x0 = inst.pop("x0")
    kw = dict(problems.SOCP_KWARGS)
    base = run(inst, x0, kw)
    print(f"m5 base: {base['seconds']:.0f}s value={base['value']!r} inner={base['inner']} steps={len(base['steps'])}",
          flush=True)
    rng = np.random.default_rng(1234)
    pert = dict(inst)
    pert["d"] = [float(v * (1 + 1e-15 * rng.standard_normal())) for v in inst["d"]]
    p = run(pert, x0, kw)
    stable = p["steps"] == base["steps"]
    wx = float(np.linalg.norm(p["xstar"] - base["xstar"]) / np.linalg.norm(base["xstar"]))
    wv = abs(p["value"] - base["value"]) / abs(base["value"])
    print(f"m5 perturbed: inner={p['inner']} stable={stable} x* spread {wx:.1e} value spread {wv:.1e}", flush=True)
    np.savez_compressed(os.path.join(HERE, "m5_socp_oracle.npz"),
                        spec=np.array(repr(dict(gen="socp_cones", n=4096, K=256, mi=16, seed=0))),
                        digest=np.array(digest(inst)), d=np.array(inst["d"]), kwargs=np.array(repr(kw)),
                        value=np.array(base["value"]), xstar=base["xstar"], inner_iters=np.array(base["inner"]),
                        trace_step=np.array(base["steps"]), trace_nd=np.array(base["nds"]),
                        sens_steps_stable=np.array(stable), sens_xstar_rel=np.array(wx), sens_value_rel=np.array(wv),
                        pert_inner_iters=np.array(p["inner"]), oracle_seconds=np.array(base["seconds"]))


if __name__ == "__main__":
    main()
