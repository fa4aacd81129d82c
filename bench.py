"""Benchmark: Newton iterations/sec on the dense QP n=8192, m=2048 (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 8192] [--m 2048] [--instances I]

A "step" is one Newton iteration of the real QPSolver.solve() on the synthetic M3-QP instance of
SURVEY.md §8(d) (testSolver.py:499-582 generator and kwargs; U(-2,2) values on a 2^-10 grid, so
the rank-0 instance is exactly the one tests/golden/m3_qp_*.npz pins against the reference).
The K timed steps per instance are split over the two phases the reference runs:
* ceil(K/2) phase-1 iterations: QPSolver.solve() from the default x0 = 0, which is infeasible for
  d = C x_f + 1, so phase 1 runs first (bordered n+1 KKT system, PhaseOneSolver.py);
* floor(K/2) barrier-phase iterations: QPSolver.solve() from the strictly feasible x_f (phase 1
  skipped), i.e. the centering steps with the tP Hessian term and the P x GEMVs (QPSolver.py:500-638).
Each segment runs on fresh solvers built (inputs resident in HBM) before its timed region, which is
bracketed by barrier + synchronize; the reported time is the max over ranks of the two segments'
sum.  W untimed warmup iterations run first on throw-away solvers (split the same way).

N > 1: one process per GPU.  Without torchrun (WORLD_SIZE unset) `--gpus N` spawns the N ranks
itself BEFORE touching the GPU (RANK/LOCAL_RANK/WORLD_SIZE set per child).  Independent instances,
no data-path collective ("scaling": "weak"): rank r solves seed r (headline) or the instances
r::N of the batch (--instances I: I per GPU, seeds 1000 + index, config 4); rank 0 gathers
per-rank times with one all_gather at the end (RCCL when every rank has its own GPU, gloo when
ranks share one -- rehearsals on a 1-GPU box).

Also reported: the dominant kernel's roofline (the Cholesky k_potrf_block, fp64 MFMA), the KKT SYRK
beside it, the KKT+POTRF kernel-only fp64 fraction, the committed PMC traffic and
MFMA counters when they were collected on this exact library build, and the CPU oracle timed on a
bounded sample of the same workload at 1 and all available BLAS threads.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "interiorpoint-gpu_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense fp64 matrix peak (256 CU x 2.4 GHz x 128)
HBM_PEAK_GBS = 8000.0
LIB = os.path.join(REPO, "interiorpoint-gpu_amd", "ipm355", "libipm355.so")
# PMC profiles of this bench (scripts/pmc_summary.py): HBM bytes per launch (FETCH_SIZE and
# WRITE_SIZE in separate passes, FETCH doubled per MI355X_MICROARCH.md) and MFMA busy cycles
PMC_SYRK = os.path.join(REPO, "profiles", "pmc_kkt_syrk.json")
PMC_POTRF = os.path.join(REPO, "profiles", "pmc_potrf_block.json")


def lib_digest(path=LIB):
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()
    except OSError:
        return None


def pmc_record(path, n, m):
    """A committed PMC summary, only if it was collected on this (n, m) AND this exact library
    build (sha256 of libipm355.so recorded by scripts/pmc_summary.py); stale files are refused."""
    try:
        d = json.load(open(path))
    except Exception:
        return None
    if (d.get("n"), d.get("m")) != (n, m) or d.get("lib_sha256") != lib_digest():
        return None
    return d


def trailing_bytes(N, nb=256):
    """HBM bytes of a right-looking blocked Cholesky: the lower trailing matrix read + written once
    per block (16 B per element)."""
    tot = 0.0
    for b0 in range(0, N, nb):
        r = N - b0
        tot += 16.0 * r * (r + 1) / 2
    return tot


def potrf_launches(N, nb=256):
    """k_potrf_block launches of one factorization of the N-column Newton matrix (N + 1 rows with
    the bordered right-hand side): one per 256-column block, except that a last block of <= 8
    columns with <= 16 rows below its origin is finished by the launch before it (potrf_plan's
    tail workgroup; the phase-1 system N = n + 1)."""
    blocks = math.ceil(N / nb)
    cbl = (blocks - 1) * nb
    return blocks - 1 if blocks >= 2 and N - cbl <= 8 and N + 1 - cbl <= 16 else blocks


def potrf_flops(N):
    """Cholesky of the N x N Newton matrix (the bordered right-hand side row adds O(N^2))."""
    return N ** 3 / 3 + N ** 2 / 2 + N / 6


GOLDEN = os.path.join(REPO, "tests", "golden")


def fixture_parity(s, seg, seed, args, k):
    """The bench's rank-0 instance IS the reference fixture instance (seed 0, n=8192, m=2048, grid
    values): compare the K timed Newton steps' sizes and the iterate after them with the reference
    run (tests/golden/m3_qp_full.npz phase-1 steps / m3_qp_feas.npz barrier steps; x_snap_K is the
    reference iterate handed to its (K+1)-th line search).  None when no fixture covers the run."""
    if seed != 0 or args.instances != 1 or args.problem != "qp" or (args.n, args.m) != (8192, 2048):
        return None
    name = {"phase1": "m3_qp_full", "barrier": "m3_qp_feas"}[seg]
    path = os.path.join(GOLDEN, name + ".npz")
    if not os.path.exists(path):
        name = {"phase1": "m3_qp_ph1", "barrier": "m3_qp_feas"}[seg]
        path = os.path.join(GOLDEN, name + ".npz")
        if not os.path.exists(path):
            return None
    z = np.load(path, allow_pickle=False)
    p1 = s.phase1_solver
    tr = list(p1.phase1_ns.trace) if (seg == "phase1" and p1 is not None) else list(s.ns.trace)
    steps = np.array([t[0] for t in tr])
    ref = z["trace_step"][:len(steps)]
    out = {"fixture": name, "newton_steps": int(len(steps)), "steps_identical": bool(np.array_equal(steps, ref))}
    key = f"x_snap_{k}"
    if key in z.files:
        x = (p1.x if seg == "phase1" else s.x_last).cpu().numpy()
        xr = z[key]
        if x.shape == xr.shape:
            out["x_rel_err"] = float(np.linalg.norm(x - xr) / np.linalg.norm(xr))
    return out


def hbm_kernels(prob):
    """HIP-event GB/s of the HBM-bound kernels of one Newton step (engine ipm_time_hbm_kernels)."""
    try:
        t = prob.time_hbm_kernels(20)
    except Exception as e:  # noqa: BLE001 -- reported, never fatal to the bench line
        return {"error": str(e)}
    return {k: {"ms": ms, "bytes": by, "GB/s": by / (ms * 1e-3) / 1e9, "frac_of_hbm_peak": by / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
            for k, (ms, by) in t.items()}


def launch_ranks(n):
    """Parent of a self-launched N-rank run: no GPU call happens here (device_count does not
    initialise the runtime on this image); each child is a fresh process owning LOCAL_RANK."""
    import torch

    from ipm355 import dist as D
    ndev = torch.cuda.device_count()
    backend = "nccl" if 0 < n <= ndev else "gloo"
    return D.launch_local(n, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                          extra_env={"IPM_BENCH_BACKEND": backend})


def make_instance(n, m, seed, dev, problem="qp"):
    """M3-QP instance (grid values); P = Pp^T Pp + I with the Gram product on the device (setup only,
    exact on the grid, not timed).  problem="lp": the M3-LP generator (testSolver.py:104-148);
    "socp": M5 (n variables, m cones of 16 rows, strictly feasible x0 -> barrier phase only)."""
    import torch
    from ipm355 import problems

    def gram(Pp):
        t = torch.as_tensor(Pp, device=dev)
        return (t.T @ t).cpu().numpy()
    if problem == "socp":
        inst = problems.socp_cones(n=n, K=m, mi=16, seed=seed)
        return inst, inst.pop("x0")
    if problem == "lp":
        inst = problems.lp_ineq_box(n, m, seed=seed, grid=True, with_xf=True)
    else:
        inst = problems.qp_ineq_box(n, m, seed=seed, grid=True, with_xf=True, gram=gram)
    xf = inst.pop("xf")
    return inst, xf


def blas_info():
    try:
        from threadpoolctl import threadpool_info
        for i in threadpool_info():
            if i.get("user_api") == "blas":
                return {"internal_api": i.get("internal_api"), "version": i.get("version"),
                        "architecture": i.get("architecture"), "max_threads": i.get("num_threads")}
    except Exception:
        pass
    return {}


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        d = dict(line.split(":", 1) for line in out.splitlines() if ":" in line)
        return {k: d.get(k, "").strip() for k in ("Model name", "Socket(s)", "Core(s) per socket",
                                                    "Thread(s) per core", "CPU(s)")}
    except Exception:
        return {}


def _cpu_worker(argv):
    """Child process of cpu_baseline: phase-1 Newton iterations of the saved instance with the BLAS
    thread count fixed by the environment before NumPy loads (OpenBLAS sizes its thread buffers at
    load time; raising the count in-process past the box's OMP_NUM_THREADS crashed it)."""
    d, seconds, kw = argv[0], float(argv[1]), json.loads(argv[2])
    from oracle import ipm_oracle as O
    C = np.load(os.path.join(d, "C.npy"), mmap_mode="r")
    C = np.ascontiguousarray(C)
    dv = np.load(os.path.join(d, "d.npy"))
    lb = np.load(os.path.join(d, "lb.npy"))
    ub = np.load(os.path.join(d, "ub.npy"))
    n = C.shape[1]
    ph = O.PhaseOne(C=C, d=dv, lb=lb, ub=ub, x0=O.default_x0(n, lb, ub), max_outer_iters=1,
                    max_inner_iters=1, epsilon=kw["epsilon"], inner_epsilon=1e-5,
                    alpha=kw["alpha"], beta=kw["beta"], mu=kw["mu"], t0=0.01, n=n, tol=0)
    iters, t0 = 0, time.perf_counter()
    while (time.perf_counter() - t0 < seconds or iters == 0) and iters < 200:
        ph.x, _, k, _, _ = ph.ns.solve(ph.x, 0.01)
        iters += k
    el = time.perf_counter() - t0
    print(json.dumps({"iters": iters, "seconds": el, "blas": blas_info()}), flush=True)


def cpu_baseline(inst, kwargs, seconds):
    """Oracle (NumPy/SciPy restatement, oracle/ipm_oracle.py) on a bounded sample of the same
    workload: phase-1 Newton iterations of this instance (bordered n+1 SYRK + Cholesky + solves),
    at 1 BLAS thread, at the box's CPU share (OMP_NUM_THREADS) and at the physical core count, ~`seconds` each
    (>= 1 iteration); the fastest is the baseline.  Each thread count runs in its own child process
    (_cpu_worker) with the count set in its environment; a failing child is recorded, not fatal."""
    import tempfile
    n = len(inst["q"])
    avail = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", avail) or avail)
    # 1 thread, the box's CPU share (OMP_NUM_THREADS), and every physical core of the host
    # (the baseline at the physical core count as well)
    lc = cpu_model()
    try:
        phys = int(lc.get("Socket(s)", "0")) * int(lc.get("Core(s) per socket", "0"))
    except ValueError:
        phys = 0
    nthreads = sorted({1, max(1, min(avail, cap))} | ({min(avail, phys)} if phys > 0 else set()))
    runs, fails, blas = [], [], {}
    kw = json.dumps({k: kwargs[k] for k in ("epsilon", "alpha", "beta", "mu")})
    with tempfile.TemporaryDirectory(prefix="ipm_cpu_") as td:
        np.save(os.path.join(td, "C.npy"), np.asarray(inst["C"], dtype=np.float64))
        np.save(os.path.join(td, "d.npy"), np.asarray(inst["d"], dtype=np.float64))
        np.save(os.path.join(td, "lb.npy"), np.asarray(inst["lower_bound"], dtype=np.float64))
        np.save(os.path.join(td, "ub.npy"), np.asarray(inst["upper_bound"], dtype=np.float64))
        for nt in nthreads:
            env = dict(os.environ)
            for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
                env[k] = str(nt)
            try:
                r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-worker", td, str(seconds), kw],
                                   env=env, capture_output=True, text=True, timeout=max(120.0, 10 * seconds))
                if r.returncode != 0:
                    fails.append({"threads": nt, "rc": r.returncode, "stderr": r.stderr[-300:]})
                    continue
                o = json.loads(r.stdout.strip().splitlines()[-1])
            except Exception as e:   # noqa: BLE001  (a baseline failure must not sink the bench line)
                fails.append({"threads": nt, "error": repr(e)[:300]})
                continue
            blas = o.get("blas") or blas
            runs.append({"threads": nt, "iters": o["iters"], "seconds": o["seconds"],
                         "value": o["iters"] / o["seconds"]})
    if not runs:
        return {"value": None, "unit": "Newton iters/s", "cores": 0, "kind": "port", "failed": fails}
    best = max(runs, key=lambda r: r["value"])   # the fastest thread count is the baseline
    out = {"value": best["value"], "unit": "Newton iters/s", "cores": best["threads"], "kind": "port",
           "sample": f"{best['iters']} phase-1 Newton iterations (bordered n+1={n + 1} KKT, m={len(inst['d'])}) of "
                     f"the same instance, oracle/ipm_oracle.py on NumPy/OpenBLAS, {best['seconds']:.1f} s",
           "by_threads": runs, "host": {"os_cpu_count": os.cpu_count(), "affinity_cpus": avail,
                                        "physical_cores": phys, "lscpu": lc, "blas": blas}}
    if fails:
        out["failed"] = fails
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--n", type=int, default=int(os.environ.get("IPM_BENCH_N", 8192)))
    ap.add_argument("--m", type=int, default=int(os.environ.get("IPM_BENCH_M", 2048)))
    ap.add_argument("--cpu-seconds", type=float, default=float(os.environ.get("IPM_BENCH_CPU_S", 12)))
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--phase", choices=["both", "phase1", "barrier"], default="both",
                    help="which phase(s) the timed steps run in (default: half each)")
    ap.add_argument("--concurrent", action="store_true",
                    help="solve the instances concurrently: one HIP stream + host thread each")
    ap.add_argument("--problem", choices=["qp", "lp", "socp"], default="qp",
                    help="qp: the headline M3-QP (default); lp: M3-LP (config 3); socp: M5, --m = cones (config 5)")
    ap.add_argument("--instances", type=int, default=1,
                    help="independent instances per GPU (config 4: --n 2048 --m 512 --instances 8); each runs "
                         "`steps` Newton iterations")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if args.concurrent:
        # each instance = its own stream; HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues
        # (4 by default) -- streams sharing a queue serialise.  Must be set before the HIP runtime
        # starts (the box presets 4: override it, <= 32 allowed).  8 x n=2048 (config 4): 4 queues
        # 1610, 8 queues 2231-2279, 16 queues 1645-2142, 32 queues 869 it/s (profiles/r4f, r4g) --
        # more concurrent kernels than that fill the CUs with waiting Cholesky roles.
        from ipm355 import dist as _D
        _D.configure_queues(int(os.environ.get("IPM_HW_QUEUES", "8")))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    backend = os.environ.get("IPM_BENCH_BACKEND") or ("nccl" if world <= ndev else "gloo")
    if backend == "nccl" and local >= ndev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} has no GPU of its own ({ndev} visible) under RCCL")
    dev_index = local % max(ndev, 1)       # gloo rehearsals: ranks share the visible GPU(s)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    sdev = dev if backend == "nccl" else torch.device("cpu")

    import ipm355
    from ipm355 import _lib as L
    from ipm355 import dist as D
    from ipm355 import problems

    kwargs = dict({"qp": problems.QP_KWARGS, "lp": problems.LP_KWARGS, "socp": problems.SOCP_KWARGS}[args.problem])
    Cls = {"qp": ipm355.QPSolver, "lp": ipm355.LPSolver, "socp": ipm355.SOCPSolver}[args.problem]
    # instances of this rank: ipm355.dist's round-robin shard (the API a user calls for config 4);
    # headline: instance index = rank (one n=8192 instance per GPU, seed = rank); config 4
    # (--instances I): indices r::world of world*I, seeds 1000 + index
    n_inst = world * args.instances
    indices = D.shard(n_inst, rank, world)
    seeds = {i: (i if args.instances == 1 else 1000 + i) for i in indices}
    insts = {i: make_instance(args.n, args.m, seed=seeds[i], dev=dev, problem=args.problem) for i in indices}

    def builder(feasible):
        def make(i):
            inst, xf = insts[i]
            kw = dict(inst, **kwargs)
            if feasible:
                kw["x0"] = xf.copy()           # strictly feasible -> phase 1 skipped (Q11)
            return kw
        return make

    def new_shard(feasible):
        # ipm355.dist.Shard: solvers built (inputs resident in HBM) on this rank's GPU; with
        # --concurrent each instance has its own HIP stream and is solved from its own host thread
        return D.Shard(builder(feasible or args.problem == "socp"), indices, Cls, None, device=dev_index,
                       concurrent=args.concurrent)

    if args.problem == "socp":
        args.phase = "barrier"               # M5 starts strictly feasible (phase 1 skipped, Q11)
    k1 = {"both": (args.steps + 1) // 2, "phase1": args.steps, "barrier": 0}[args.phase]
    segs = [("phase1", k1), ("barrier", args.steps - k1)]
    w1 = (args.warmup + 1) // 2
    for feasible, budget in ((False, w1), (True, args.warmup - w1)):   # warmup, untimed
        if budget > 0:
            new_shard(feasible).solve(iteration_budget=budget)
    import ctypes
    res, evidence, hbm_rates = {}, {}, {}
    for name, budget in segs:
        if budget <= 0:
            res[name] = dict(iters=0, seconds=0.0, kkt_ms=0.0, potrf_ms=0.0, kkt_flops=0.0, N=0)
            continue
        sh = new_shard(name == "barrier")   # inputs resident in HBM before timing
        s0 = sh.solvers[0]
        fm0 = s0.phase1_solver.phase1_fm if name == "phase1" else s0.fm
        kkt_flops = fm0.prob.kkt_flops()[0]
        h = fm0.prob.handle                # (instance 0's handle: the timings below are its own)
        h.lib.ipm_set_timing(h.ptr, 1)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        local = sh.solve(iteration_budget=budget)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        h.lib.ipm_last_timings(h.ptr, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        h.lib.ipm_set_timing(h.ptr, 0)
        # Newton iterations of this segment (phase-1 ones only in the phase-1 segment: the barrier
        # segment starts strictly feasible)
        iters = float(sum(v[1] for v in local.values()))
        res[name] = dict(iters=iters, seconds=el, kkt_ms=a.value, potrf_ms=b.value, kkt_flops=kkt_flops,
                         N=args.n + (1 if name == "phase1" else 0))
        if rank == 0:
            # after the timed region: rank 0's own evidence (trace/iterate vs the reference fixture,
            # HBM-kernel GB/s on this solver's buffers)
            evidence[name] = fixture_parity(s0, name, seeds[indices[0]], args, budget)
            if args.problem in ("qp", "lp"):
                hbm_rates[name] = hbm_kernels(fm0.prob)
        del sh, s0, fm0

    keys = ("iters", "seconds", "kkt_ms", "potrf_ms")
    row = [res[nm][k] for nm, _ in segs for k in keys]
    stats = torch.tensor(row, dtype=torch.float64, device=sdev)
    if world > 1:
        allst = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allst, stats)          # the only collective: end-of-run gather
        allst = torch.stack(allst).cpu().numpy()
    else:
        allst = stats.cpu().numpy()[None]
    if rank == 0:
        n, m = args.n, args.m
        per = {}
        for j, (nm, _) in enumerate(segs):
            blk = allst[:, 4 * j:4 * j + 4]
            per[nm] = dict(iters=float(blk[:, 0].sum()), tmax=float(blk[:, 1].max()), rank_seconds=blk[:, 1],
                           kkt_ms=float(blk[0, 2]), potrf_ms=float(blk[0, 3]))
        rank_total = sum(per[nm]["rank_seconds"] for nm, _ in segs)
        tmax = float(np.max(rank_total))
        total_iters = sum(per[nm]["iters"] for nm, _ in segs)
        # rank 0's kernel timings, weighted by its per-segment iteration counts
        it0 = {nm: float(allst[0, 4 * j]) for j, (nm, _) in enumerate(segs)}
        tot0 = max(sum(it0.values()), 1.0)
        pf_tot = sum(it0[nm] * potrf_flops(res[nm]["N"]) for nm, _ in segs if it0[nm])
        pt_tot = sum(it0[nm] * per[nm]["potrf_ms"] for nm, _ in segs)
        launches = sum(it0[nm] * potrf_launches(res[nm]["N"]) for nm, _ in segs)
        kf_tot = sum(it0[nm] * res[nm]["kkt_flops"] for nm, _ in segs)
        kt_tot = sum(it0[nm] * per[nm]["kkt_ms"] for nm, _ in segs)
        potrf_tf = pf_tot / (pt_tot * 1e-3) / 1e12 if pt_tot > 0 else 0.0
        kkt_tf = kf_tot / (kt_tot * 1e-3) / 1e12 if kt_tot > 0 else 0.0
        f_iter = sum(it0[nm] * (res[nm]["kkt_flops"] + potrf_flops(res[nm]["N"]) + 2 * res[nm]["N"] ** 2)
                     for nm, _ in segs) / tot0
        pmc_p, pmc_s = pmc_record(PMC_POTRF, n, m), pmc_record(PMC_SYRK, n, m)
        Nmain = n + 1 if it0.get("phase1", 0) >= it0.get("barrier", 0) else n
        value = total_iters / tmax
        rec = {
            "metric": "Newton iters/sec, dense QP n=8192, 1/2/4/8 GPUs; achieved % fp64 roofline",
            "value": value, "unit": "Newton iters/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": tmax / max(total_iters / world, 1) * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded M3-QP generator, testSolver.py:499-582 shapes; U(-2,2) on a 2^-10 grid)",
            "config": {"workload": f"QPSolver.solve() dense QP n={n}, m={m} ineq, box +-3, test_QP kwargs; per "
                                   f"instance {k1} phase-1 iterations (from x0=0) + {args.steps - k1} barrier-phase "
                                   f"iterations (from the feasible x_f); {args.instances} independent instance(s) "
                                   f"per GPU" + (" solved concurrently (one stream + host thread each)"
                                                 if args.concurrent else ""),
                       "n": n, "m": m, "instances_per_gpu": args.instances,
                       "parallelism": f"instances{world * args.instances}", "backend": backend if world > 1 else None},
            "phases": {nm: {"iters": per[nm]["iters"], "seconds_max_rank": per[nm]["tmax"],
                            "iters_per_s": per[nm]["iters"] / per[nm]["tmax"] if per[nm]["tmax"] > 0 else None,
                            "kkt_ms": per[nm]["kkt_ms"], "potrf_ms": per[nm]["potrf_ms"],
                            "system_size": res[nm]["N"]} for nm, _ in segs},
            # dominant kernel: the Cholesky, one k_potrf_block launch per 256 columns; achieved =
            # factorization flops / HIP-event time of all its launches (= per-launch flops / avg launch)
            "roofline": {"bound": "mfma", "achieved": potrf_tf, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": potrf_tf / FP64_MFMA_PEAK_TFLOPS,
                         "traffic": pmc_p["hbm_bytes_per_launch"] if pmc_p else None,
                         "kernel": "k_potrf_block (blocked Cholesky of the Newton matrix, bordered RHS row)",
                         "flops_per_launch": pf_tot / max(launches, 1),
                         "avg_launch_ms": pt_tot / max(launches, 1),
                         "launches_per_factorization": launches / tot0,
                         # right-looking blocked Cholesky: each launch reads and writes the lower
                         # trailing matrix once (16 B per element), averaged over the launches
                         "algorithmic_bytes_per_launch": trailing_bytes(Nmain) / potrf_launches(Nmain),
                         "mfma_counters": (pmc_p or {}).get("mfma")},
            "kkt_syrk": {"kernel": "k_mfma_gemm<128,weighted> (KKT assembly H = [tP +] C^T diag(w) C + diag)",
                         "achieved_tflops": kkt_tf, "frac": kkt_tf / FP64_MFMA_PEAK_TFLOPS,
                         "flops_per_launch": kf_tot / tot0, "avg_launch_ms": kt_tot / tot0,
                         "traffic": pmc_s["hbm_bytes_per_launch"] if pmc_s else None,
                         "algorithmic_bytes_per_launch": 8 * (m * n + m + n * (n + 1) / 2 * 2),
                         "mfma_counters": (pmc_s or {}).get("mfma")},
            "potrf": {"achieved_tflops": potrf_tf, "avg_ms": pt_tot / tot0, "flops": pf_tot / tot0},
            # SURVEY.md §8(d) / BASELINE.md: KKT assembly + Cholesky, kernel time only (HIP events)
            "kkt_potrf_kernel_frac": ((kf_tot + pf_tot) / ((kt_tot + pt_tot) * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS)
                                     if kt_tot + pt_tot > 0 else 0.0,
            "whole_iteration_fp64_frac": (f_iter * total_iters / world / tmax) / 1e12 / FP64_MFMA_PEAK_TFLOPS,
            "newton_iters": total_iters,
            "lib_sha256": lib_digest(),
            "parity": evidence,
            "hbm_kernels": hbm_rates,
        }
        if args.problem == "lp":
            rec["metric"] = "Newton iters/sec, dense LP (config 3)"
            rec["data"] = "synthetic (seeded M3-LP generator, testSolver.py:104-148 shapes; U(-2,2) on a 2^-10 grid)"
            rec["config"]["workload"] = (f"LPSolver.solve() dense LP n={n}, m={m} ineq, box +-3, test_LP kwargs; per "
                                         f"instance {k1} phase-1 iterations (from x0=0) + {args.steps - k1} "
                                         f"barrier-phase iterations (from the feasible x_f)")
        elif args.problem == "socp":
            rec["metric"] = "Newton iters/sec, SOCP (config 5)"
            rec["data"] = ("synthetic (seeded M5 generator: P=I, K cones of 16 Gaussian rows, d_i making x0 "
                           "strictly feasible; no bounds)")
            rec["config"]["workload"] = (f"SOCPSolver.solve() n={n}, {m} second-order cones of 16 rows, P=I, no "
                                         f"bounds, test_SOCP kwargs; {args.steps} barrier-phase iterations from the "
                                         f"strictly feasible x0 (phase 1 skipped)")
        if not args.no_cpu and world == 1 and args.problem == "qp":
            rec["cpu_baseline"] = cpu_baseline(insts[indices[0]][0], kwargs, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--cpu-worker":
        _cpu_worker(sys.argv[2:])
    else:
        main()
