"""Rank process for tests/test_gpu_large.py::test_sharded_two_ranks_real_solvers (started by
ipm355.dist.launch_local): the REAL sharded path on the GPU box -- gloo between the ranks (both
share the box's one GPU; RCCL refuses two ranks on one device), every rank runs
ipm355.dist.solve_sharded with the device QPSolver on its round-robin half of the M4 reference
fixtures (seeds 1000..1007), and the table + x* of all eight come back through the single
all_gather.  Writes tab<rank>.npy / x<rank>.npy into the output directory."""
import ast
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "interiorpoint-gpu_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ipm355 import QPSolver  # noqa: E402
from ipm355 import dist as D  # noqa: E402
from ipm355 import problems  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")


def instance(seed):
    z = np.load(os.path.join(GOLDEN, f"m4_qp_{seed}.npz"), allow_pickle=False)
    spec = ast.literal_eval(str(z["spec"]))

    def gram(Pp):
        t = torch.as_tensor(Pp, device="cuda")
        return (t.T @ t).cpu().numpy()
    inst = problems.qp_ineq_box(spec["n"], spec["m"], seed=spec["seed"], grid=spec["grid"], gram=gram)
    if problems.input_digest(inst) != str(z["digest"]):
        raise SystemExit(f"seed {seed}: regenerated inputs differ from the reference's")
    kw = ast.literal_eval(str(z["kwargs"]))
    kw.pop("x0", None)
    return dict(inst, **kw)


if __name__ == "__main__":
    out_dir = sys.argv[1]
    backend = sys.argv[2] if len(sys.argv) > 2 else "gloo"   # "nccl": RCCL (one rank per GPU)
    seeds = list(range(1000, 1008)) if len(sys.argv) <= 3 else list(range(1000, 1000 + int(sys.argv[3])))
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo")
    try:
        tab, X = D.solve_sharded(lambda i: instance(seeds[i]), len(seeds), QPSolver, device=0, gather_x=True)
        rank = dist.get_rank()
        np.save(os.path.join(out_dir, f"tab{rank}.npy"), tab)
        np.save(os.path.join(out_dir, f"x{rank}.npy"), X)
        with open(os.path.join(out_dir, f"backend{rank}.txt"), "w") as f:
            f.write(dist.get_backend())
    finally:
        dist.destroy_process_group()
