"""Benchmark: Newton iterations/sec on the dense QP n=8192, m=2048 (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 8192] [--m 2048]

A "step" is one Newton iteration of the real QPSolver.solve() (phase 1 first,
exactly as the reference runs it: x0 = 0 is infeasible for d = C x_f + 1), on the
synthetic M3-QP instance of SURVEY.md §8(d) (testSolver.py:499-582 generator and
kwargs).  W untimed iterations on one solver, then EXACTLY K timed iterations on
a fresh solver of the same instance (iteration budget), bracketed by barrier +
synchronize.  Inputs are resident in HBM before the timed region.

N > 1: one process per GPU (torchrun), each rank solves its own instance
(seed = rank) -- independent instances, no data-path collective ("scaling":
"weak"); rank 0 gathers per-rank times/objectives with one all_gather at the end.

Also reported: the dominant kernel's roofline (the Cholesky k_potrf_block, fp64 MFMA),
the KKT SYRK beside it, the KKT+POTRF kernel-only fp64 fraction, and
the CPU oracle timed on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "interiorpoint-gpu_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense fp64 matrix peak (256 CU x 2.4 GHz x 128)
HBM_PEAK_GBS = 8000.0
# HBM bytes per launch from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate passes,
# FETCH doubled per MI355X_MICROARCH.md) of this same bench: scripts/pmc_summary.py
PMC_SYRK = os.path.join(REPO, "profiles", "pmc_kkt_syrk.json")
PMC_POTRF = os.path.join(REPO, "profiles", "pmc_potrf_block.json")


def pmc_traffic(path, n, m):
    """PMC-measured HBM bytes per launch, only if the committed profile is of this (n, m)."""
    try:
        d = json.load(open(path))
        return float(d["hbm_bytes_per_launch"]) if (d.get("n"), d.get("m")) == (n, m) else None
    except Exception:
        return None


def trailing_bytes(N, nb=256):
    """HBM bytes of a right-looking blocked Cholesky: the lower trailing matrix read + written once
    per block (16 B per element)."""
    tot = 0.0
    for b0 in range(0, N, nb):
        r = N - b0
        tot += 16.0 * r * (r + 1) / 2
    return tot


def potrf_flops(N):
    """Cholesky of the N x N Newton matrix (the bordered right-hand side row adds O(N^2))."""
    return N ** 3 / 3 + N ** 2 / 2 + N / 6


def make_instance(n, m, seed, dev):
    """M3-QP instance; P = Pp^T Pp + I formed on the device (setup only, not timed)."""
    import torch
    rng = np.random.default_rng(seed)
    Pp = torch.as_tensor(rng.uniform(-2, 2, size=(int(0.8 * n), n)), device=dev)
    P = (Pp.T @ Pp).cpu().numpy()
    del Pp
    P[np.diag_indices(n)] += 1.0
    q = rng.uniform(-2, 2, size=n)
    C = rng.uniform(-2, 2, size=(m, n))
    xf = rng.uniform(-2, 2, size=n)
    d = C @ xf + 1
    return dict(P=P, q=q, C=C, d=d, lower_bound=-3, upper_bound=3)


def cpu_baseline(inst, kwargs, seconds=15.0):
    """Oracle (NumPy/SciPy restatement, oracle/ipm_oracle.py) on a bounded sample of the same
    workload: phase-1 Newton iterations of this instance, until ~`seconds` of CPU work."""
    from oracle import ipm_oracle as O
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("internal_api") == "openblas"]
                      or [1])
    except Exception:
        threads = int(os.environ.get("OPENBLAS_NUM_THREADS", "1"))
    n = len(inst["q"])
    lb = np.array(inst["lower_bound"], dtype=float)
    ub = np.array(inst["upper_bound"], dtype=float)
    x0 = O.default_x0(n, lb, ub)
    ph = O.PhaseOne(C=inst["C"], d=inst["d"], lb=lb, ub=ub, x0=x0, max_outer_iters=1,
                    max_inner_iters=1, epsilon=kwargs["epsilon"], inner_epsilon=1e-5,
                    alpha=kwargs["alpha"], beta=kwargs["beta"], mu=kwargs["mu"], t0=0.01, n=n, tol=0)
    iters, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds and iters < 200:
        ph.x, _, k, _, _ = ph.ns.solve(ph.x, 0.01)
        iters += k
    el = time.perf_counter() - t0
    return {"value": iters / el, "unit": "Newton iters/s", "cores": int(threads), "kind": "port",
            "sample": f"{iters} phase-1 Newton iterations (bordered n+1={n + 1} KKT, m={len(inst['d'])}) of the "
                      f"same instance, oracle/ipm_oracle.py on NumPy/OpenBLAS, {el:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=int(os.environ.get("IPM_BENCH_N", 8192)))
    ap.add_argument("--m", type=int, default=int(os.environ.get("IPM_BENCH_M", 2048)))
    ap.add_argument("--cpu-seconds", type=float, default=float(os.environ.get("IPM_BENCH_CPU_S", 15)))
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--concurrent", action="store_true",
                    help="solve the instances concurrently: one HIP stream + host thread each")
    ap.add_argument("--instances", type=int, default=1,
                    help="independent instances per GPU (config 4: --n 2048 --m 512 --instances 8); each runs "
                         "`steps` Newton iterations")
    args = ap.parse_args()
    if args.concurrent:
        # each instance = its stream + its Cholesky panel stream; HIP maps streams onto
        # GPU_MAX_HW_QUEUES hardware queues (4 by default) -- streams sharing a queue serialise.
        # Must be set before the HIP runtime starts.
        os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one rank per GPU; on a node with fewer GPUs than ranks (rehearsals) ranks share them
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import ipm355
    from ipm355 import _lib as L
    from ipm355 import problems

    kwargs = dict(problems.QP_KWARGS)
    # one instance: seed = rank (headline); several: seeds 1000 + rank * instances + i
    seeds = [rank] if args.instances == 1 else [1000 + rank * args.instances + i for i in range(args.instances)]
    insts = [make_instance(args.n, args.m, seed=sd, dev=dev) for sd in seeds]

    def new_solver(inst):
        return ipm355.QPSolver(check_cvxpy=False, suppress_print=True, device=local, **inst, **kwargs)

    # one stream per instance when concurrent (solvers bind their handle to the current stream)
    streams = [torch.cuda.Stream(device=dev) for _ in insts] if args.concurrent else [None] * len(insts)

    def on(stream):
        return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()

    # warmup: W iterations on a throw-away solver per stream (kernels, allocator, caches)
    if args.warmup > 0:
        for inst, stm in zip(insts, streams if args.concurrent else streams[:1]):
            with on(stm):
                new_solver(inst).solve(iteration_budget=args.warmup)
    solvers = []
    for inst, stm in zip(insts, streams):                 # inputs resident in HBM before timing
        with on(stm):
            solvers.append(new_solver(inst))
    with on(streams[0]):
        h = L.Handle.get(local)
    h.lib.ipm_set_timing(h.ptr, 1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    if args.concurrent:
        from concurrent.futures import ThreadPoolExecutor

        def run(k):
            with on(streams[k]):
                solvers[k].solve(iteration_budget=args.steps)
        with ThreadPoolExecutor(max_workers=len(solvers)) as ex:
            list(ex.map(run, range(len(solvers))))
    else:
        for solver in solvers:
            solver.solve(iteration_budget=args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    import ctypes
    a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    h.lib.ipm_last_timings(h.ptr, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    kkt_ms, potrf_ms, cnt = a.value, b.value, c.value
    p1 = sum(sum(s.phase1_solver.inner_iters) for s in solvers)
    done = p1 + sum(sum(s.inner_iters) for s in solvers)
    inst = insts[0]

    stats = torch.tensor([el, float(done), kkt_ms, potrf_ms, float(p1)], dtype=torch.float64, device=dev)
    if world > 1:
        allst = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allst, stats)          # the only collective: end-of-run gather over xGMI
        allst = torch.stack(allst).cpu().numpy()
    else:
        allst = stats.cpu().numpy()[None]
    if rank == 0:
        tmax = float(allst[:, 0].max())
        total_iters = float(allst[:, 1].sum())
        n, m = args.n, args.m
        syrk_flops = m * n * (n + 1) + n * n      # Cholesky-KKT assembly: SYRK + tP epilogue
        # phase-1 iterations factor the (n+1)-variable system, the others n (rank 0's mix)
        f1 = float(allst[0, 4]) / max(float(allst[0, 1]), 1.0)
        pf = f1 * potrf_flops(n + 1) + (1 - f1) * potrf_flops(n)
        launches = f1 * ((n + 1 + 255) // 256) + (1 - f1) * ((n + 255) // 256)   # one per 256 columns
        kkt_tf = syrk_flops / (float(allst[0, 2]) * 1e-3) / 1e12 if allst[0, 2] > 0 else 0.0
        potrf_tf = pf / (float(allst[0, 3]) * 1e-3) / 1e12 if allst[0, 3] > 0 else 0.0
        f_iter = m * n * (n + 1) + pf + 2 * n * n
        value = total_iters / tmax
        rec = {
            "metric": "Newton iters/sec, dense QP n=8192, 1/2/4/8 GPUs; achieved % fp64 roofline",
            "value": value, "unit": "Newton iters/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": tmax / max(total_iters / world, 1) * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded M3-QP generator, testSolver.py:499-582 shapes)",
            "config": {"workload": f"QPSolver.solve() dense QP n={n}, m={m} ineq, box +-3, phase 1 incl., "
                                   f"test_QP kwargs; {args.instances} independent instance(s) per GPU"
                                   + (" solved concurrently (one stream + host thread each)" if args.concurrent else ""),
                       "n": n, "m": m, "instances_per_gpu": args.instances,
                       "parallelism": f"instances{world * args.instances}"},
            # dominant kernel: the Cholesky, one k_potrf_block launch per 256 columns; achieved =
            # factorization flops / HIP-event time of all its launches (= per-launch flops / avg launch)
            "roofline": {"bound": "mfma", "achieved": potrf_tf, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": potrf_tf / FP64_MFMA_PEAK_TFLOPS, "traffic": pmc_traffic(PMC_POTRF, n, m),
                         "kernel": "k_potrf_block (blocked Cholesky of the Newton matrix, bordered RHS row)",
                         "flops_per_launch": pf / launches, "avg_launch_ms": float(allst[0, 3]) / launches,
                         "launches_per_factorization": launches,
                         # right-looking blocked Cholesky: each launch reads and writes the lower
                         # trailing matrix once (16 B per element), averaged over the launches
                         "algorithmic_bytes_per_launch": trailing_bytes(n + 1 if f1 >= 0.5 else n) / launches},
            "kkt_syrk": {"kernel": "k_mfma_gemm<128,weighted> (KKT assembly H = tP + C^T diag(w) C + diag)",
                         "achieved_tflops": kkt_tf, "frac": kkt_tf / FP64_MFMA_PEAK_TFLOPS,
                         "flops_per_launch": syrk_flops, "avg_launch_ms": float(allst[0, 2]),
                         "traffic": pmc_traffic(PMC_SYRK, n, m),
                         "algorithmic_bytes_per_launch": 8 * (m * n + m + n * (n + 1) / 2 * 2)},
            "potrf": {"achieved_tflops": potrf_tf, "avg_ms": float(allst[0, 3]), "flops": pf},
            # SURVEY.md §8(d) / BASELINE.md: KKT assembly + Cholesky, kernel time only (HIP events)
            "kkt_potrf_kernel_frac": ((syrk_flops + pf) / ((float(allst[0, 2]) + float(allst[0, 3])) * 1e-3)
                                      / 1e12 / FP64_MFMA_PEAK_TFLOPS) if allst[0, 2] + allst[0, 3] > 0 else 0.0,
            "whole_iteration_fp64_frac": (f_iter * total_iters / world / tmax) / 1e12 / FP64_MFMA_PEAK_TFLOPS,
            "newton_iters": total_iters,
        }
        if not args.no_cpu and world == 1:
            rec["cpu_baseline"] = cpu_baseline(inst, kwargs, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
