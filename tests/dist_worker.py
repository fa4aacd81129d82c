"""Rank process for tests/test_dist_gloo.py::test_launch_local_end_to_end (started by
ipm355.dist.launch_local, gloo backend, no GPU): solve_sharded with a stubbed device solve that
returns (value, iters, x*), x* gathered through the same all_gather table the GPU run uses."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "interiorpoint-gpu_amd")]

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ipm355 import dist as D  # noqa: E402


def stub(i):
    return 100.0 + i, 7 + i % 3, np.arange(5, dtype=float) * i


if __name__ == "__main__":
    n_inst, out_dir = int(sys.argv[1]), sys.argv[2]
    dist.init_process_group("gloo")
    try:
        tab, X = D.solve_sharded(None, n_inst, solve_fn=stub, gather_x=True)
        rank = dist.get_rank()
        np.save(os.path.join(out_dir, f"tab{rank}.npy"), tab)
        np.save(os.path.join(out_dir, f"x{rank}.npy"), X)
        with open(os.path.join(out_dir, f"env{rank}.txt"), "w") as f:
            f.write(f"{os.environ['RANK']} {os.environ['LOCAL_RANK']} {os.environ['WORLD_SIZE']}")
    finally:
        dist.destroy_process_group()
