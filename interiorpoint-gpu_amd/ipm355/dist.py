"""Multi-GPU driver: independent problem instances sharded one process per GPU.

The reference has no distributed code. Its benchmark harness solves independent random instances
one after another (testSolver.py:437-808). Here rank r of a `torchrun` job solves instances
``r::world`` on its own GPU. No data moves between GPUs while solving. After the last solve, ONE
``all_gather`` (RCCL over xGMI on MI355X, ``gloo`` in the CPU tests) gives every rank every
instance's (objective, Newton iterations, seconds).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 my_batch.py
      -> ipm355.dist.solve_sharded(make_instance, 64, ipm355.QPSolver, kwargs)
"""
from __future__ import annotations

import os
import socket
import subprocess
import time

import numpy as np

FIELDS = 4  # (instance index, objective value, Newton iterations incl. phase 1, seconds)


def shard(n_instances: int, rank: int, world: int) -> list:
    """Instances owned by `rank`: round-robin, so every rank gets floor or ceil of n/world."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    return list(range(rank, n_instances, world))


def _world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


def _backend():
    import torch.distributed as dist
    return dist.get_backend() if dist.is_available() and dist.is_initialized() else None


def local_device(device=None) -> int:
    """The GPU this rank owns: the explicit ``device`` or LOCAL_RANK (one process per GPU)."""
    return int(device) if device is not None else int(os.environ.get("LOCAL_RANK", "0"))


def _table_device(device):
    """RCCL (backend "nccl") gathers device tensors; gloo and the single-process case host ones."""
    import torch
    return torch.device("cuda", local_device(device)) if _backend() == "nccl" else torch.device("cpu")


def gather_results(local: dict, n_instances: int, device=None, xs: dict | None = None, n: int = 0):
    """all_gather every rank's {index: (value, iters, seconds)} -> (n_instances, 3) array.

    Every rank contributes a fixed-size (ceil(n/world), FIELDS) table padded with index -1.
    With ``xs`` ({index: x* (n,)}) the x* rows travel in the same collective (appended columns),
    and the return value is (table, X) with X (n_instances, n).  This is the only collective of
    the sharded path; under RCCL the table lives on this rank's GPU.
    """
    import torch
    import torch.distributed as dist
    rank, world = _world()
    slots = -(-n_instances // world)
    width = FIELDS + (n if xs is not None else 0)
    tab = torch.full((slots, width), -1.0, dtype=torch.float64)
    for k, (idx, vals) in enumerate(sorted(local.items())):
        tab[k, 0] = float(idx)
        tab[k, 1:FIELDS] = torch.tensor([float(v) if v is not None else float("nan") for v in vals],
                                        dtype=torch.float64)
        if xs is not None:
            tab[k, FIELDS:] = torch.as_tensor(np.asarray(xs[idx], dtype=np.float64))
    tab = tab.to(_table_device(device))
    if dist.is_initialized():   # (world 1 too: a one-rank RCCL group runs the same device gather)
        parts = [torch.empty_like(tab) for _ in range(world)]
        dist.all_gather(parts, tab)
        allt = torch.cat(parts).cpu().numpy()
    else:
        allt = tab.cpu().numpy()
    out = np.full((n_instances, FIELDS - 1), np.nan)
    X = np.full((n_instances, n), np.nan) if xs is not None else None
    for row in allt:
        if row[0] >= 0:
            out[int(row[0])] = row[1:FIELDS]
            if X is not None:
                X[int(row[0])] = row[FIELDS:]
    return (out, X) if xs is not None else out


class Shard:
    """This rank's instances, built on this rank's GPU and ready to solve (inputs resident in HBM).

    concurrent=True (config 4): every instance gets its own HIP stream -- its solver and native
    handle are created under ``torch.cuda.stream(stream)`` -- and ``solve()`` runs the instances
    from one host thread per distinct stream (the native calls release the GIL), so their kernels
    overlap on the GPU.  The HIP runtime maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default;
    streams sharing a queue serialise): call ``configure_queues()`` before anything initialises
    the GPU.  concurrent=False: one after another on the current stream."""

    def __init__(self, make_instance, indices, solver_cls, kwargs=None, device=None, concurrent=False):
        import torch
        self.indices = list(indices)
        self.dev = local_device(device)
        self.concurrent = bool(concurrent)
        self.streams = ([torch.cuda.Stream(device=torch.device("cuda", self.dev)) for _ in self.indices]
                        if self.concurrent else [None] * len(self.indices))
        self.solvers = []
        for i, st in zip(self.indices, self.streams):
            with _on(st):
                s = solver_cls(check_cvxpy=False, suppress_print=True, device=self.dev, **make_instance(i),
                               **(kwargs or {}))
            if s.dev.index != self.dev:
                raise RuntimeError(f"solver placed on {s.dev}, rank owns cuda:{self.dev}")
            self.solvers.append(s)

    def solve(self, **solve_kwargs):
        """Solve every instance (solve_kwargs go to each solver's solve(), e.g. iteration_budget);
        returns {index: (value, Newton iterations incl. phase 1, seconds)}."""
        import torch

        def one(k):
            s = self.solvers[k]
            t0 = time.perf_counter()
            with _on(self.streams[k]):
                value = s.solve(**solve_kwargs)
                if self.streams[k] is not None:
                    self.streams[k].synchronize()
            p1 = getattr(s, "phase1_solver", None)
            iters = int(sum(s.inner_iters)) + (int(sum(p1.inner_iters)) if p1 is not None else 0)
            return self.indices[k], (value, iters, time.perf_counter() - t0)
        if self.concurrent and len(self.solvers) > 1:
            # one host thread per DISTINCT stream: torch hands out streams from a pool of 32 per
            # device, so past 32 instances (or beside another Shard) two instances can share a
            # stream -- and with it the native handle (Handle.get caches one per (device, stream)),
            # whose staging buffers and scratch are not safe to drive from two threads.  Instances
            # sharing a stream run one after another in that stream's thread.
            from concurrent.futures import ThreadPoolExecutor
            groups = {}
            for k, st in enumerate(self.streams):
                groups.setdefault(st.cuda_stream, []).append(k)

            def run_group(ks):
                return [one(k) for k in ks]
            with ThreadPoolExecutor(max_workers=len(groups)) as ex:
                out = dict(r for rs in ex.map(run_group, list(groups.values())) for r in rs)
        else:
            out = dict(one(k) for k in range(len(self.solvers)))
        if torch.cuda.is_available():
            torch.cuda.synchronize(self.dev)
        return out

    def xstar(self):
        return {i: s.xstar for i, s in zip(self.indices, self.solvers)}


def _on(stream):
    import contextlib

    import torch
    return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()


def configure_queues(queues: int = 8) -> bool:
    """Give the HIP runtime `queues` hardware queues per process (GPU_MAX_HW_QUEUES, read once when
    the runtime starts) so that concurrent instances do not serialise on shared queues.  Returns
    False when it is too late (the runtime already started); the box presets 4, gpurun allows 32.
    8 is the measured best for 8 x n=2048 per GPU (config 4): 4 / 8 / 16 / 32 queues gave 1610 /
    2231-2279 / 1645-2142 / 869 Newton it/s -- more concurrent kernels leave the CUs full of
    Cholesky roles waiting on their chains."""
    import torch
    if torch.cuda.is_initialized():
        return False
    os.environ["GPU_MAX_HW_QUEUES"] = str(int(queues))
    return True


def build_shard(make_instance, n_instances: int, solver_cls, kwargs=None, device=None, concurrent=False) -> Shard:
    """This rank's instances r::world of n_instances, built (not solved) on this rank's GPU."""
    rank, world = _world()
    return Shard(make_instance, shard(n_instances, rank, world), solver_cls, kwargs, device, concurrent)


def solve_sharded(make_instance, n_instances: int, solver_cls=None, kwargs=None, device=None,
                  solve_fn=None, gather_x: bool = False, concurrent: bool = False, solve_kwargs=None):
    """Solve this rank's shard on this rank's GPU, then gather every instance's (value, iters, seconds).

    make_instance(i) -> dict of constructor arguments for instance i (seeded by i);
    solver_cls: ipm355.LPSolver / QPSolver / SOCPSolver; kwargs: shared solver kwargs.
    device: this rank's GPU (default LOCAL_RANK); every solver is built on it.
    concurrent: solve this rank's instances concurrently, one HIP stream + host thread each (Shard).
    solve_kwargs: passed to every solve() (e.g. iteration_budget).
    solve_fn(i) -> (value, iters[, x*]) overrides the solver (host-logic tests run it without a GPU).
    gather_x: also gather every instance's x* -> returns (table, X).
    """
    rank, world = _world()
    local, xs = {}, {}
    if solve_fn is not None:
        for i in shard(n_instances, rank, world):
            t0 = time.perf_counter()
            r = solve_fn(i)
            local[i] = (r[0], r[1], time.perf_counter() - t0)
            if gather_x:
                xs[i] = r[2] if len(r) > 2 else None
    else:
        sh = build_shard(make_instance, n_instances, solver_cls, kwargs, device, concurrent)
        local = sh.solve(**(solve_kwargs or {}))
        if gather_x:
            xs = sh.xstar()
    if gather_x:
        nx = len(next(iter(xs.values()))) if xs else 0
        if world > 1 and dist_initialized():
            import torch
            import torch.distributed as dist
            t = torch.tensor([nx], dtype=torch.int64, device=_table_device(device))
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            nx = int(t.item())
        return gather_results(local, n_instances, device=device, xs=xs, n=nx)
    return gather_results(local, n_instances, device=device)


def dist_initialized() -> bool:
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_local(nprocs: int, argv: list, extra_env: dict | None = None, poll_s: float = 0.2) -> int:
    """Start `argv` as `nprocs` fresh rank processes on this node (torchrun's env contract: RANK,
    LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) and wait for them.

    Call it before anything initialises the GPU in this process: children are started, never
    exec'd.  If one rank fails the others are terminated (they would wait in a barrier forever).
    Returns 0 or the first failing rank's exit status (128 + signal for a killed rank)."""
    port = _free_port()
    procs = []
    for r in range(nprocs):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs),
                   LOCAL_WORLD_SIZE=str(nprocs), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.update(extra_env or {})
        procs.append(subprocess.Popen(argv, env=env))
    rc = 0
    while procs:
        for p in list(procs):
            c = p.poll()
            if c is None:
                continue
            procs.remove(p)
            if c != 0:
                rc = rc or (c if c > 0 else 128 - c)
                for q in procs:
                    q.terminate()
        if procs:
            time.sleep(poll_s)
    return rc
