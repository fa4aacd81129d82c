"""-m gpu: parity at the BASELINE.json sizes.

The fixtures come from the REFERENCE itself (tests/golden/make_golden_large.py, run in the build
container): instances are regenerated here from their seed with ``grid=True`` (U(-2,2) on a 2^-10
grid, so P = Pp'Pp and d = C x_f + 1 are exact in fp64 whatever computes them) and checked against
the sha256 the fixture stores, so the GPU sees exactly the reference's inputs.

Bars (north star: x* within 1e-6 relative of the reference NumPy solve):
* full solves (M2, the M4 shard): x* <= max(1e-6, 4 x the reference's own 1e-15-perturbation
  spread); where the reference's step sequence is stable under that perturbation, the inner
  iteration counts and EVERY accepted step size must be identical;
* truncated n=8192 runs (M3-QP phase 1, M3-QP barrier phase from x_f, M3-LP): the first K Newton
  steps' step sizes identical, Newton decrements within 1e-6 relative, the iterate after K steps
  within 1e-6 relative;
* M5 (SOCP n=4096, 256 cones): the reference's own FunctionManagerSOCP caches 2 K n^2 doubles
  (64 GiB), so it is checked against the oracle's stacked-cone restatement (pinned to the
  reference by the small SOCP fixtures): the first Newton steps' sizes identical, x within 1e-6.
"""
import ast
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

XSTAR_RTOL = 1e-6
# Newton decrement nd = -g.dx/2: relative 1e-6, plus an absolute 1e-9 for the steps where nd has
# cancelled down to ~1e-8 (end of a centering step; g and dx are O(1e2..1e4) there)
ND_RTOL, ND_ATOL = 1e-6, 1e-9


def nd_excess(nds, ref, spread=None):
    """max over steps of |nd - nd_ref| / ((max(ND_RTOL, 4 spread_k)) |nd_ref| + ND_ATOL); <= 1 passes.
    spread_k = the reference's own relative change of nd at step k under the 1e-15 input
    perturbation: in the stuck centering steps at large t (Q1) H is so ill-conditioned that the
    reference itself moves nd by ~1e-5 there."""
    if not len(ref):
        return 0.0
    rt = ND_RTOL if spread is None else np.maximum(ND_RTOL, 4 * spread)
    e = np.abs(nds - ref) / (rt * np.abs(ref) + ND_ATOL)
    for i in np.argsort(e)[::-1][:4]:
        print(f"    nd step {i}: device {nds[i]!r} reference {ref[i]!r} excess {e[i]:.2f}")
    return float(e.max())


def centering_step_spread(spread, z):
    """The n=8192 full-solve fixtures sample the reference's envelope with ONE perturbed re-run (a
    second ordering would take hours), so the per-step Newton-decrement spread is a single noisy
    sample.  In the stuck steps of a centering step at large t (Q1: alpha -> 1e-13, H nearly
    singular) every step has the same conditioning: each step is held to the largest spread the
    re-run showed within its own centering step (phase-1 and barrier-phase centering steps alike,
    in the order NewtonSolver ran them)."""
    counts = list(z["phase1_inner_iters"]) + list(z["inner_iters"])
    out = np.array(spread, dtype=float, copy=True)
    k = 0
    for c in counts:
        c = int(c)
        if c > 0:
            out[k:k + c] = np.max(out[k:k + c])
        k += c
    return out


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _fixture(name):
    path = os.path.join(GOLDEN, name + ".npz")
    if not os.path.exists(path):
        pytest.skip(f"fixture {name}.npz not generated")
    return dict(np.load(path, allow_pickle=False))


def _gram_on_device(Pp):
    import torch
    t = torch.as_tensor(Pp, device="cuda")
    return (t.T @ t).cpu().numpy()


def _instance(z):
    """Regenerate the fixture's inputs from its generator spec and check the digest."""
    from ipm355 import problems
    spec = ast.literal_eval(str(z["spec"]))
    if spec["gen"] == "qp_ineq_box":
        inst = problems.qp_ineq_box(spec["n"], spec["m"], seed=spec["seed"], grid=spec["grid"], with_xf=True,
                                    gram=_gram_on_device)
    else:
        inst = problems.lp_ineq_box(spec["n"], spec["m"], seed=spec["seed"], grid=spec["grid"], with_xf=True)
    xf = inst.pop("xf")
    assert problems.input_digest(inst) == str(z["digest"]), "regenerated inputs differ from the reference's"
    kw = ast.literal_eval(str(z["kwargs"]))
    kw.pop("x0", None)
    if spec.get("x0") == "xf":
        kw["x0"] = xf
    return spec, dict(inst, **kw)


def _cls(spec):
    import ipm355
    return ipm355.QPSolver if spec["gen"] == "qp_ineq_box" else ipm355.LPSolver


def _device_trace(s):
    p1 = getattr(s, "phase1_solver", None)
    tr = (list(p1.phase1_ns.trace) if p1 is not None else []) + list(s.ns.trace)
    return np.array([t[0] for t in tr]), np.array([t[1] for t in tr])


def _check_full(name):
    z = _fixture(name)
    spec, kw = _instance(z)
    s = _cls(spec)(check_cvxpy=False, suppress_print=True, **kw)
    np.testing.assert_array_equal(np.asarray(s.x), z["x_init"])
    v = s.solve()
    err = rel(s.xstar, z["xstar"])
    xtol = max(XSTAR_RTOL, 4 * float(z["sens_xstar_rel"]))
    steps, nds = _device_trace(s)
    print(f"[{name}] x* rel {err:.2e} (tol {xtol:.1e}), value {v!r} vs {float(z['value'])!r}, "
          f"{len(steps)} Newton steps (reference {len(z['trace_step'])}), iters {list(s.inner_iters)}")
    assert err <= xtol, err
    assert abs(v - float(z["value"])) <= max(1e-8, 4 * float(z["sens_value_rel"])) * max(1.0, abs(float(z["value"])))
    if bool(z["sens_steps_stable"]):
        assert list(s.inner_iters) == list(z["inner_iters"])
        assert list(s.phase1_solver.inner_iters if s.phase1_solver is not None else []) == \
            list(z["phase1_inner_iters"])
        np.testing.assert_array_equal(steps, z["trace_step"])
        spread = z.get("sens_nd_rel")
        if spread is not None and "pert_trace_step" in z:
            spread = centering_step_spread(spread, z)
        ndx = nd_excess(nds, z["trace_nd"], spread)
        assert ndx <= 1.0, ndx
    return s


def test_m2_qp_full_solve():
    """M2: QP n=2048, m=512, test_QP kwargs, phase 1 + 10 barrier centering steps (881 Newton steps)."""
    _check_full("m2_qp")


@pytest.mark.parametrize("name", ["m3_qp_ph1", "m3_qp_feas", "m3_lp"])
def test_m3_truncated_trajectory(name):
    """M3 at n=8192, m=2048: the first K Newton steps of the headline QP (phase 1, then from x_f the
    barrier phase) and of the LP, against the reference's steps, decrements and iterate."""
    z = _fixture(name)
    spec, kw = _instance(z)
    K = int(z["k_steps"])
    s = _cls(spec)(check_cvxpy=False, suppress_print=True, **kw)
    np.testing.assert_array_equal(np.asarray(s.x), z["x_init"])
    s.solve(iteration_budget=K)
    steps, nds = _device_trace(s)
    xk_ref = z["x_k"]
    if len(xk_ref) == spec["n"] + 1:
        xk = s.phase1_solver.x.cpu().numpy()
    else:
        xk = s.x_last.cpu().numpy()
    err = rel(xk, xk_ref)
    nd_x = nd_excess(nds, z["trace_nd"], z.get("sens_nd_rel")) if len(nds) == len(z["trace_nd"]) else float("inf")
    print(f"[{name}] K={K}: x_K rel {err:.2e}, nd excess {nd_x:.2e}, steps equal "
          f"{np.array_equal(steps, z['trace_step'])}, reference stable {bool(z['sens_steps_stable'])}")
    assert len(steps) == K
    assert err <= max(XSTAR_RTOL, 4 * float(z["sens_xk_rel"])), err
    if bool(z["sens_steps_stable"]):
        np.testing.assert_array_equal(steps, z["trace_step"])
        assert nd_x <= 1.0, nd_x


@pytest.mark.parametrize("timing", [0, 1])
def test_m3_phase1_snapshots(timing):
    """bench.py's rank-0 evidence: the phase-1 iterate after K = 10 and K = 30 Newton
    steps against the reference's snapshots x_snap_K (m3_qp_full), with the engine's HIP-event
    timing mode (ipm_set_timing, what the bench runs under) off and on.  Both must give the same
    iterate bit for bit, within 1e-6 of the reference."""
    z = _fixture("m3_qp_full")
    spec, kw = _instance(z)
    out = {}
    for K in (10, 30):
        s = _cls(spec)(check_cvxpy=False, suppress_print=True, **kw)
        if timing:
            h = s.phase1_solver.phase1_fm.prob.handle
            h.lib.ipm_set_timing(h.ptr, 1)
        s.solve(iteration_budget=K)
        if timing:
            h.lib.ipm_set_timing(h.ptr, 0)
        steps, _ = _device_trace(s)
        x = s.phase1_solver.x.cpu().numpy()
        err = rel(x, z[f"x_snap_{K}"])
        out[K] = x
        print(f"[timing={timing}] K={K}: x rel {err:.2e}, steps identical "
              f"{np.array_equal(steps, z['trace_step'][:len(steps)])}")
        assert np.array_equal(steps, z["trace_step"][:len(steps)])
        assert err <= XSTAR_RTOL, err
    np.save(f"/tmp/ipm_ph1_snap_t{timing}.npy", np.stack([out[10], out[30]]))
    if timing and os.path.exists("/tmp/ipm_ph1_snap_t0.npy"):
        np.testing.assert_array_equal(np.load("/tmp/ipm_ph1_snap_t0.npy"), np.stack([out[10], out[30]]))


def test_m3_phase1_trajectory_is_deterministic():
    """Run to run, the bordered phase-1 trajectory (n = 8193) is bitwise the same.  r6 found the
    fused Cholesky's diagonal role racing with itself: wave 0 wrote the factored diagonal rows back
    over the LDS copy that wave 1 (a second leaf wave) had yet to read when a trailing tile on the
    same CU slowed wave 1 down -- 4 of 12 runs of this trajectory differed (up to 1.7e-4 at step
    30, some falling to the least-squares backup) once round 6 stopped keeping that CU free.  Wave 1
    now signals when its copy has landed (diag_role, ipm_blas.hip)."""
    z = _fixture("m3_qp_ph1")
    spec, kw = _instance(z)
    K = int(z["k_steps"])
    prev = None
    for r in range(4):
        s = _cls(spec)(check_cvxpy=False, suppress_print=True, **kw)
        s.solve(iteration_budget=K)
        xk = s.phase1_solver.x.cpu().numpy()
        err = rel(xk, z["x_k"])
        print(f"run {r}: x_K rel {err:.2e}")
        assert err <= max(XSTAR_RTOL, 4 * float(z["sens_xk_rel"])), err
        if prev is not None:
            np.testing.assert_array_equal(xk, prev)
        prev = xk


@pytest.mark.parametrize("name", ["m2_qp", "m3_qp_ph1", "m3_qp_feas", "m3_lp"])
def test_linesearch_flip_rate(name, monkeypatch):
    """The 64-candidate table line search against the reference-exact one (IPM_LINESEARCH=compare:
    every Newton step runs both, takes the exact step and counts the steps whose sizes differ) on
    the M2 and M3 trajectories; the trajectory must still meet the fixture's bars."""
    import json
    monkeypatch.setenv("IPM_LINESEARCH", "compare")
    z = _fixture(name)
    spec, kw = _instance(z)
    s = _cls(spec)(check_cvxpy=False, suppress_print=True, **kw)
    if "k_steps" in z:
        s.solve(iteration_budget=int(z["k_steps"]))
    else:
        s.solve()
    probs = [s.fm.prob] + ([s.phase1_solver.phase1_fm.prob] if s.phase1_solver is not None else [])
    cmp_, flips = sum(getattr(p, "ls_compared", 0) for p in probs), sum(getattr(p, "ls_flips", 0) for p in probs)
    steps, nds = _device_trace(s)
    same = np.array_equal(steps, z["trace_step"]) if len(steps) == len(z["trace_step"]) else False
    print(f"[{name}] line-search flips {flips} of {cmp_} Newton steps; step sequence equal to the reference: {same}")
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", f"ls_flips_{name}.json"), "w") as f:
        json.dump({"case": name, "compared": cmp_, "flips": flips, "steps_equal_reference": bool(same)}, f)
    assert cmp_ == len(steps)
    if bool(z["sens_steps_stable"]):
        assert same


@pytest.mark.parametrize("concurrent", [False, True])
def test_m4_shard_on_one_gpu(concurrent):
    """Config 4 shard: eight of the 64 M4 instances (seeds 1000..1007, n=2048, m=512) solved by the
    sharded driver (ipm355.dist.solve_sharded, world 1 -> every instance on this GPU), x* gathered
    through the same table the multi-GPU run all_gathers, each against its reference fixture.
    concurrent=True: the product path of config 4's per-GPU concurrency -- one HIP
    stream + host thread per instance (ipm355.dist.Shard) -- with the same bars, identical iteration
    counts included."""
    from ipm355 import dist
    from ipm355 import QPSolver
    names = [f"m4_qp_{sd}" for sd in range(1000, 1008)]
    zs = [_fixture(nm) for nm in names]
    insts = [_instance(z)[1] for z in zs]
    tab, X = dist.solve_sharded(lambda i: {k: v for k, v in insts[i].items()}, len(insts), QPSolver,
                                device=0, gather_x=True, concurrent=concurrent)
    for i, z in enumerate(zs):
        err = rel(X[i], z["xstar"])
        ref_iters = int(sum(z["inner_iters"]) + sum(z["phase1_inner_iters"]))
        print(f"[{names[i]}] x* rel {err:.2e}, value {tab[i, 0]!r} vs {float(z['value'])!r}, "
              f"iters {int(tab[i, 1])} vs {ref_iters}")
        assert err <= max(XSTAR_RTOL, 4 * float(z["sens_xstar_rel"])), (names[i], err)
        assert abs(tab[i, 0] - float(z["value"])) <= max(1e-8, 4 * float(z["sens_value_rel"])) * abs(float(z["value"]))
        if bool(z["sens_steps_stable"]):
            assert int(tab[i, 1]) == ref_iters


def test_sharded_two_ranks_real_solvers(tmp_path):
    """The sharded driver in TWO processes with the real device solver: launch_local
    starts 2 ranks (gloo: both share this box's GPU), each runs solve_sharded with QPSolver on its
    round-robin half of the eight M4 reference fixtures, and the all_gathered table and x* of every
    instance must match the fixtures on BOTH ranks (the same bars as the one-process shard test)."""
    import sys
    from ipm355 import dist
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_gpu_worker.py")
    rc = dist.launch_local(2, [sys.executable, "-u", worker, str(tmp_path)])
    assert rc == 0
    zs = [_fixture(f"m4_qp_{sd}") for sd in range(1000, 1008)]
    for r in range(2):
        tab = np.load(tmp_path / f"tab{r}.npy")
        X = np.load(tmp_path / f"x{r}.npy")
        for i, z in enumerate(zs):
            err = rel(X[i], z["xstar"])
            ref_iters = int(sum(z["inner_iters"]) + sum(z["phase1_inner_iters"]))
            if r == 0:
                print(f"[rank-gathered m4_qp_{1000 + i}, solved by rank {i % 2}] x* rel {err:.2e}, "
                      f"iters {int(tab[i, 1])} vs {ref_iters}")
            assert err <= max(XSTAR_RTOL, 4 * float(z["sens_xstar_rel"])), (r, i, err)
            assert abs(tab[i, 0] - float(z["value"])) <= \
                max(1e-8, 4 * float(z["sens_value_rel"])) * abs(float(z["value"]))
            if bool(z["sens_steps_stable"]):
                assert int(tab[i, 1]) == ref_iters
    np.testing.assert_array_equal(np.load(tmp_path / "x0.npy"), np.load(tmp_path / "x1.npy"))


def test_sharded_rccl_one_rank(tmp_path):
    """The RCCL branch of the sharded path (backend "nccl": the gather table lives on the rank's
    GPU and goes through a device all_gather), as far as a one-GPU box allows: ONE rank in an RCCL
    process group (RCCL refuses two ranks on one device), solve_sharded with the device QPSolver on
    two M4 reference fixtures, the table + x* through the RCCL all_gather, checked against them."""
    import sys
    from ipm355 import dist
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_gpu_worker.py")
    rc = dist.launch_local(1, [sys.executable, "-u", worker, str(tmp_path), "nccl", "2"])
    assert rc == 0
    assert (tmp_path / "backend0.txt").read_text() == "nccl"
    tab = np.load(tmp_path / "tab0.npy")
    X = np.load(tmp_path / "x0.npy")
    for i in range(2):
        z = _fixture(f"m4_qp_{1000 + i}")
        err = rel(X[i], z["xstar"])
        ref_iters = int(sum(z["inner_iters"]) + sum(z["phase1_inner_iters"]))
        print(f"[rccl m4_qp_{1000 + i}] x* rel {err:.2e}, iters {int(tab[i, 1])} vs {ref_iters}")
        assert err <= max(XSTAR_RTOL, 4 * float(z["sens_xstar_rel"])), (i, err)
        if bool(z["sens_steps_stable"]):
            assert int(tab[i, 1]) == ref_iters


@pytest.mark.parametrize("name", ["m3_qp_full", "m3_lp_full"])
def test_m3_full_solve(name):
    """The headline instance solved to COMPLETION: M3-QP n=8192, m=2048, test_QP
    kwargs, phase 1 + barrier phase (QPSolver.py:500-638; testSolver.py:563-582), and M3-LP with
    test_LP kwargs, against the reference's own full solve: x* within max(1e-6, 4x the reference's
    1e-15-perturbation spread), the value likewise, and -- where the reference's step sequence is
    stable under that perturbation -- identical iteration counts and step sizes."""
    s = _check_full(name)
    z = _fixture(name)
    steps, _ = _device_trace(s)
    ref = z["trace_step"]
    k = min(len(steps), len(ref))
    first = int(np.argmax(steps[:k] != ref[:k])) if np.any(steps[:k] != ref[:k]) else k
    p1 = s.phase1_solver
    print(f"[{name}] device iters {list(s.inner_iters)} phase 1 {list(p1.inner_iters) if p1 is not None else []}; "
          f"reference {list(z['inner_iters'])} phase 1 {list(z['phase1_inner_iters'])}; reference perturbed "
          f"{list(z['pert_inner_iters']) if 'pert_inner_iters' in z else '-'}; first differing step {first} of {k}")


def test_m5_socp_full_solve():
    """M5 solved to completion (3 steps before): SOCPSolver n=4096, 256 cones
    of 16 rows, SOCP_KWARGS (testSolver.py:924-945), against the oracle's stacked-cone full solve
    (tests/golden/m5_socp_oracle.npz; the reference itself would need 64 GiB of cone caches here).
    The oracle's own 1e-15 perturbation envelope sets the x* bar; where it is stable, the inner
    iteration counts and every step size must be identical."""
    import ast as _ast
    import ipm355
    from ipm355 import problems
    z = _fixture("m5_socp_oracle")
    spec = _ast.literal_eval(str(z["spec"]))
    inst = problems.socp_cones(n=spec["n"], K=spec["K"], mi=spec["mi"], seed=spec["seed"])
    x0 = inst.pop("x0")
    dg = problems.input_digest({"A": np.stack(inst["A"]), "b": np.stack(inst["b"]), "c": np.stack(inst["c"]),
                                "q": inst["q"]})
    assert dg == str(z["digest"])
    inst["d"] = [float(v) for v in z["d"]]
    kw = _ast.literal_eval(str(z["kwargs"]))
    g = ipm355.SOCPSolver(check_cvxpy=False, suppress_print=True, x0=x0.copy(), **inst, **kw)
    v = g.solve()
    err = rel(g.xstar, z["xstar"])
    gs = np.array([t[0] for t in g.ns.trace])
    xtol = max(XSTAR_RTOL, 4 * float(z["sens_xstar_rel"]))
    print(f"[m5 full] x* rel {err:.2e} (tol {xtol:.1e}), value {v!r} vs {float(z['value'])!r}, iters "
          f"{list(g.inner_iters)} vs {list(z['inner_iters'])}, oracle stable {bool(z['sens_steps_stable'])}")
    assert err <= xtol
    assert abs(v - float(z["value"])) <= max(1e-8, 4 * float(z["sens_value_rel"])) * abs(float(z["value"]))
    if bool(z["sens_steps_stable"]):
        assert list(g.inner_iters) == list(z["inner_iters"])
        np.testing.assert_array_equal(gs, z["trace_step"])


@pytest.mark.parametrize("name", ["m5ref_socp_n256", "m5ref_socp_n2048"])
def test_m5ref_socp_full_solve(name):
    """Config 5's cone shape pinned to the REFERENCE itself: SOCPSolver with
    K=256 cones of 16 rows, P=I, strictly feasible x0, SOCP_KWARGS (testSolver.py:924-945), at
    n=2048 (and n=256) where the reference's 2 K n^2 cone caches fit the build container
    (FunctionManager.py:869-894, 1104-1158; tests/golden/make_golden_m5ref.py).  Bars as for the M3
    full solves: x* within max(1e-6, 4x the reference's 1e-15-perturbation spread), the value
    likewise; where the reference's step sequence is stable under that perturbation, identical
    inner iteration counts and every accepted step size identical."""
    import ast as _ast
    import ipm355
    from ipm355 import problems
    z = _fixture(name)
    spec = _ast.literal_eval(str(z["spec"]))
    inst = problems.socp_cones(n=spec["n"], K=spec["K"], mi=spec["mi"], seed=spec["seed"])
    x0 = inst.pop("x0")
    dg = problems.input_digest({"A": np.stack(inst["A"]), "b": np.stack(inst["b"]), "c": np.stack(inst["c"]),
                                "q": inst["q"]})
    assert dg == str(z["digest"])
    inst["d"] = [float(v) for v in z["d"]]
    kw = _ast.literal_eval(str(z["kwargs"]))
    g = ipm355.SOCPSolver(check_cvxpy=False, suppress_print=True, x0=x0.copy(), **inst, **kw)
    v = g.solve()
    err = rel(g.xstar, z["xstar"])
    gs = np.array([t[0] for t in g.ns.trace])
    xtol = max(XSTAR_RTOL, 4 * float(z["sens_xstar_rel"]))
    ref = z["trace_step"]
    k = min(len(gs), len(ref))
    first = int(np.argmax(gs[:k] != ref[:k])) if np.any(gs[:k] != ref[:k]) else k
    print(f"[{name}] x* rel {err:.2e} (tol {xtol:.1e}), value {v!r} vs {float(z['value'])!r}, iters "
          f"{list(g.inner_iters)} vs reference {list(z['inner_iters'])}, reference stable "
          f"{bool(z['sens_steps_stable'])}, first differing step {first} of {k}")
    assert err <= xtol
    assert abs(v - float(z["value"])) <= max(1e-8, 4 * float(z["sens_value_rel"])) * abs(float(z["value"]))
    if bool(z["sens_steps_stable"]):
        assert list(g.inner_iters) == list(z["inner_iters"])
        np.testing.assert_array_equal(gs, ref)


def test_m5_socp_against_oracle():
    """M5: SOCPSolver n=4096, K=256 cones of 16 rows, P=I, strictly feasible x0 (phase 1 skipped):
    the first centering step truncated to 3 Newton steps on the device and in the oracle."""
    import ipm355
    from ipm355 import problems
    from oracle import ipm_oracle as O
    inst = problems.socp_cones(n=4096, K=256, mi=16, seed=0)
    x0 = inst.pop("x0")
    kw = dict(problems.SOCP_KWARGS, max_outer_iters=1, max_inner_iters=3)
    g = ipm355.SOCPSolver(check_cvxpy=False, suppress_print=True, x0=x0.copy(), **inst, **kw)
    g.solve()
    c = O.SOCPSolver(x0=x0.copy(), **inst, **kw)
    c.solve()
    err = rel(g.xstar, c.xstar)
    gs = [t[0] for t in g.ns.trace]
    cs = [t["step"] for t in c.ns.trace]
    print(f"[m5] x rel {err:.2e}, steps {gs} vs oracle {cs}, iters {list(g.inner_iters)} vs {list(c.inner_iters)}")
    assert gs == cs
    assert err <= XSTAR_RTOL
