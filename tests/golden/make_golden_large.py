"""Golden vectors at the BASELINE.json sizes, made by running the REFERENCE itself (build container
only; ~15-30 min on 8 threads).

    PYTHONDONTWRITEBYTECODE=1 OPENBLAS_NUM_THREADS=8 python tests/golden/make_golden_large.py [case ...]

Cases (generator = ipm355.problems with ``grid=True``, i.e. U(-2,2)
rounded to multiples of 2^-10 so that P = Pp'Pp and d = C x_f + 1 are exact in fp64 and the GPU box
regenerates bit-identical inputs from the seed -- the fixture stores the sha256 of those inputs,
never the inputs themselves (P alone is 512 MiB at n=8192)):

* ``m2_qp``          M2: QP n=2048, m=512, seed 0, test_QP kwargs, FULL solve (phase 1 + barrier).
* ``m4_qp_<seed>``   M4 shard: QP n=2048, m=512, seeds 1000..1007 (rank 0's eight of the 64), full.
* ``m3_qp_ph1``      M3-QP headline instance n=8192, m=2048, seed 0: the first K Newton steps
                     (phase 1, bordered n+1 system).
* ``m3_qp_feas``     the same instance started at its strictly feasible x_f (phase 1 skipped): the
                     first K barrier-phase Newton steps (tP epilogue, P x GEMVs).
* ``m3_lp``          M3-LP n=8192, m=2048, seed 0, test_LP kwargs: the first K Newton steps.
* ``m3_qp_full``     the M3-QP headline instance solved to COMPLETION (phase 1 + barrier phase,
                     QPSolver.py:500-638): x*, value, inner / phase-1 iteration lists, the whole step
                     trace, x snapshots at steps 10 and 30 (bench.py's rank-0 evidence); envelope = one
                     1e-15 rhs-perturbed re-run (a 1-thread re-run would take ~6 h here).
* ``m3_lp_full``     the M3-LP instance solved to completion, same envelope.

Every case also stores ``x_snap_<k>``: the iterate handed to the (k+1)-th line search, k in SNAPS.

Recorded per accepted Newton step: the returned backtracking step size and the Newton decrement
nd = -g.dx/2 (both exactly what NewtonSolver.solve computes, NewtonSolver.py:93-133); for the
truncated cases the iterate x_K after K steps (the x handed to the (K+1)-th line search).
Sensitivity (the reference's own envelope, and whether its step sequence is stable): re-runs with
the right-hand side perturbed by 1e-15 relative (truncated and M4: one; M2: two), plus one re-run of
the unperturbed inputs at 1 OpenBLAS thread (a different summation order in dpotrf).
"""
from __future__ import annotations

import os
import sys
import time
import types

os.environ.setdefault("OPENBLAS_NUM_THREADS", "8")
sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "interiorpoint-gpu_amd"))
sys.modules.setdefault("cvxpy", types.ModuleType("cvxpy"))
sys.path.insert(0, REF)

import numpy as np  # noqa: E402

import NewtonSolver as RNS  # noqa: E402
from LPSolver import LPSolver as RefLP  # noqa: E402
from QPSolver import QPSolver as RefQP  # noqa: E402

from ipm355 import problems  # noqa: E402

K_TRUNC = int(os.environ.get("IPM_GOLDEN_K", "30"))
SNAPS = (10, 30)
ALT_THREADS = int(os.environ.get("IPM_GOLDEN_ALT_THREADS", "1"))


class _StopK(Exception):
    pass


class _Rec:
    def __init__(self):
        self.limit = None
        self.steps, self.nds, self.ph1 = [], [], []
        self.x_at_limit = None
        self.snaps = {}

    def reset(self, limit=None):
        self.__init__()
        self.limit = limit


REC = _Rec()


def _wrap():
    orig = RNS.NewtonSolver.backtrack_search

    def rec(self, x, xstep, t, gradf):
        if len(REC.steps) in SNAPS:
            REC.snaps[len(REC.steps)] = np.array(x, copy=True)
        if REC.limit is not None and len(REC.steps) >= REC.limit:
            REC.x_at_limit = np.array(x, copy=True)
            raise _StopK()
        s = orig(self, x, xstep, t, gradf)
        REC.steps.append(float(s))
        REC.nds.append(float(-gradf.dot(xstep) / 2))
        REC.ph1.append(bool(getattr(self, "phase1_flag", False)))
        return s
    RNS.NewtonSolver.backtrack_search = rec


def build(case):
    """-> (solver class, kwargs incl. inputs, generator spec)"""
    if case == "m2_qp" or case.startswith("m4_qp_"):
        seed = 0 if case == "m2_qp" else int(case.split("_")[-1])
        spec = dict(gen="qp_ineq_box", n=2048, m=512, seed=seed, grid=True)
        inst = problems.qp_ineq_box(2048, 512, seed=seed, grid=True)
        return RefQP, dict(inst, **problems.QP_KWARGS), spec, None
    if case in ("m3_qp_ph1", "m3_qp_feas", "m3_qp_full"):
        spec = dict(gen="qp_ineq_box", n=8192, m=2048, seed=0, grid=True)
        inst = problems.qp_ineq_box(8192, 2048, seed=0, grid=True, with_xf=True)
        xf = inst.pop("xf")
        kw = dict(inst, **problems.QP_KWARGS)
        if case == "m3_qp_feas":
            kw["x0"] = xf.copy()
            spec["x0"] = "xf"
        return RefQP, kw, spec, (None if case == "m3_qp_full" else K_TRUNC)
    if case in ("m3_lp", "m3_lp_full"):
        spec = dict(gen="lp_ineq_box", n=8192, m=2048, seed=0, grid=True)
        inst = problems.lp_ineq_box(8192, 2048, seed=0, grid=True)
        return RefLP, dict(inst, **problems.LP_KWARGS), spec, (None if case == "m3_lp_full" else K_TRUNC)
    raise KeyError(case)


def run_once(cls, kw, limit):
    REC.reset(limit)
    kw = {k: (np.array(v, copy=True) if isinstance(v, np.ndarray) else v) for k, v in kw.items()}
    s = cls(check_cvxpy=False, suppress_print=True, **kw)
    x_init = np.array(s.x, copy=True)
    val, xstar = None, None
    try:
        val = s.solve()
        xstar = np.asarray(s.xstar)
    except _StopK:
        pass
    except NameError as e:
        # NewtonSolver.solve's `except cp.linalg.LinAlgError` (NewtonSolver.py:152) names the absent
        # cupy module while our stop signal passes through it: the NameError carries _StopK
        if not isinstance(e.__context__, _StopK):
            raise
    ph = getattr(s, "phase1_solver", None)
    return dict(solver=s, x_init=x_init, value=val, xstar=xstar, steps=list(REC.steps), nds=list(REC.nds),
                ph1=list(REC.ph1), x_limit=REC.x_at_limit,
                snaps=dict(REC.snaps), inner_iters=list(getattr(s, "inner_iters", [])),
                phase1_inner_iters=list(getattr(ph, "inner_iters", []) if ph is not None else []))


def make(case):
    cls, kw, spec, limit = build(case)
    t0 = time.time()
    base = run_once(cls, kw, limit)
    el = time.time() - t0
    out = {"spec": np.array(repr(spec)), "digest": np.array(problems.input_digest(
        {k: v for k, v in kw.items() if isinstance(v, np.ndarray) and k != "x0"})),
        "x_init": base["x_init"], "trace_step": np.array(base["steps"]), "trace_nd": np.array(base["nds"]),
        "trace_phase1": np.array(base["ph1"]), "kwargs": np.array(repr({k: v for k, v in kw.items()
                                                                          if not isinstance(v, np.ndarray)})),
        "ref_seconds": np.array(el)}
    for k, xs in base["snaps"].items():
        out[f"x_snap_{k}"] = xs
    if limit is None:
        out.update(value=np.array(base["value"]), xstar=base["xstar"], inner_iters=np.array(base["inner_iters"]),
                   phase1_inner_iters=np.array(base["phase1_inner_iters"]))
    else:
        out.update(k_steps=np.array(limit), x_k=base["x_limit"])
    # the reference's own envelope: rhs perturbed by 1e-15 relative
    key = "d"
    rng = np.random.default_rng(1234)
    wx, wv, stable, wk = 0.0, 0.0, True, 0.0
    wnd = np.zeros(len(base["nds"]))
    big_full = case.endswith("_full")
    for _ in range(1 if (limit is not None or case.startswith("m4_") or big_full) else 2):
        kp = dict(kw)
        kp[key] = kw[key] * (1 + 1e-15 * rng.standard_normal(kw[key].shape))
        r = run_once(cls, kp, limit)
        stable &= r["steps"] == base["steps"]
        if len(r["nds"]) == len(base["nds"]):      # per-step spread of the Newton decrement
            b = np.array(base["nds"])
            wnd = np.maximum(wnd, np.abs(np.array(r["nds"]) - b) / np.maximum(np.abs(b), 1e-300))
        if limit is None:
            wx = max(wx, float(np.linalg.norm(r["xstar"] - base["xstar"]) / np.linalg.norm(base["xstar"])))
            wv = max(wv, abs(r["value"] - base["value"]) / max(abs(base["value"]), 1e-300))
        elif r["x_limit"] is not None and base["x_limit"] is not None and r["x_limit"].shape == base["x_limit"].shape:
            wk = max(wk, float(np.linalg.norm(r["x_limit"] - base["x_limit"]) / np.linalg.norm(base["x_limit"])))
    # ... and the reference's own spread under a different summation order: the unperturbed solve
    # at 1 OpenBLAS thread (dpotrf's blocking depends on the thread count; a GPU factorization is
    # just another summation order, so this is the envelope the Newton decrements are held to)
    from threadpoolctl import threadpool_limits
    if not big_full:
        with threadpool_limits(limits=ALT_THREADS, user_api="blas"):
            r = run_once(cls, kw, limit)
        stable &= r["steps"] == base["steps"]
        if len(r["nds"]) == len(base["nds"]):
            b = np.array(base["nds"])
            wnd = np.maximum(wnd, np.abs(np.array(r["nds"]) - b) / np.maximum(np.abs(b), 1e-300))
        if limit is None:
            wx = max(wx, float(np.linalg.norm(r["xstar"] - base["xstar"]) / np.linalg.norm(base["xstar"])))
            wv = max(wv, abs(r["value"] - base["value"]) / max(abs(base["value"]), 1e-300))
        elif r["x_limit"] is not None and base["x_limit"] is not None and r["x_limit"].shape == base["x_limit"].shape:
            wk = max(wk, float(np.linalg.norm(r["x_limit"] - base["x_limit"]) / np.linalg.norm(base["x_limit"])))
    else:   # the perturbed run's iteration lists, for the chaotic-envelope report
        out.update(pert_inner_iters=np.array(r["inner_iters"]), pert_phase1_inner_iters=np.array(r["phase1_inner_iters"]),
                   pert_trace_step=np.array(r["steps"]))
    out.update(sens_sources=np.array(f"{key} * (1 + 1e-15 N(0,1))" + ("" if big_full else
                                     f"; OpenBLAS {ALT_THREADS} thread(s) vs {os.environ['OPENBLAS_NUM_THREADS']}")))
    out.update(sens_key=np.array(key), sens_xstar_rel=np.array(wx), sens_value_rel=np.array(wv),
               sens_xk_rel=np.array(wk), sens_steps_stable=np.array(stable), sens_nd_rel=wnd)
    np.savez_compressed(os.path.join(HERE, case + ".npz"), **out)
    print(f"{case}: {el:.0f}s steps={len(base['steps'])} (phase1 {sum(base['ph1'])}) inner={base['inner_iters']} "
          f"ph1 inner={base['phase1_inner_iters']} value={base['value']} stable={stable} "
          f"sens x* {wx:.1e} x_K {wk:.1e}", flush=True)


def main():
    _wrap()
    cases = sys.argv[1:] or (["m2_qp"] + [f"m4_qp_{s}" for s in range(1000, 1008)]
                             + ["m3_qp_ph1", "m3_qp_feas", "m3_lp"])
    for c in cases:
        make(c)


if __name__ == "__main__":
    main()
