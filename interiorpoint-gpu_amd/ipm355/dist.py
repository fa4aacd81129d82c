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


def gather_results(local: dict, n_instances: int, device=None) -> np.ndarray:
    """all_gather every rank's {index: (value, iters, seconds)} -> (n_instances, 3) array.

    Every rank contributes a fixed-size (ceil(n/world), FIELDS) table padded with index -1.
    This is the only collective of the sharded path.
    """
    import torch
    import torch.distributed as dist
    rank, world = _world()
    slots = -(-n_instances // world)
    tab = torch.full((slots, FIELDS), -1.0, dtype=torch.float64, device=device)
    for k, (idx, vals) in enumerate(sorted(local.items())):
        tab[k, 0] = float(idx)
        tab[k, 1:] = torch.tensor([float(v) for v in vals], dtype=torch.float64)
    if world > 1 and dist.is_initialized():
        parts = [torch.empty_like(tab) for _ in range(world)]
        dist.all_gather(parts, tab)
        allt = torch.cat(parts).cpu().numpy()
    else:
        allt = tab.cpu().numpy()
    out = np.full((n_instances, FIELDS - 1), np.nan)
    for row in allt:
        if row[0] >= 0:
            out[int(row[0])] = row[1:]
    return out


def solve_sharded(make_instance, n_instances: int, solver_cls=None, kwargs=None, device=None,
                  solve_fn=None) -> np.ndarray:
    """Solve this rank's shard, then gather every instance's (value, iters, seconds).

    make_instance(i) -> dict of constructor arguments for instance i (seeded by i);
    solver_cls: ipm355.LPSolver / QPSolver / SOCPSolver; kwargs: shared solver kwargs.
    solve_fn(i) -> (value, iters) overrides the solver (host-logic tests run it without a GPU).
    """
    rank, world = _world()
    local = {}
    for i in shard(n_instances, rank, world):
        t0 = time.perf_counter()
        if solve_fn is not None:
            value, iters = solve_fn(i)
        else:
            s = solver_cls(check_cvxpy=False, suppress_print=True, **make_instance(i), **(kwargs or {}))
            value = s.solve()
            p1 = getattr(s, "phase1_solver", None)
            iters = int(sum(s.inner_iters)) + (int(sum(p1.inner_iters)) if p1 is not None else 0)
        local[i] = (value, iters, time.perf_counter() - t0)
    return gather_results(local, n_instances, device=device)
