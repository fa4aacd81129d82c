"""Load golden fixtures (tests/golden/*.npz, written by make_golden.py) back into
solver kwargs.  Pure data handling -- no reference code is involved."""
import os

import numpy as np

from conftest import GOLDEN

SOLVE_CASES = {
    "lp_eq_box": "LP", "lp_ineq_box": "LP", "lp_ineq_box_testkw": "LP", "lp_eq_ineq": "LP",
    "qp_ineq_box": "QP", "qp_ineq_box_256": "QP", "qp_feasible": "QP", "qp_eq_phase1": "QP",
    "socp_small": "SOCP", "socp_small_eq": "SOCP", "socp_phase1": "SOCP", "socp_group_lasso": "SOCP",
    # round 2: feasible NewtonSolverDiagonal (bounds only) and stable diagonal infeasible-start runs
    "lp_box_diag": "LP", "lp_box_diag_vec": "LP",
    "lp_eq_box_tk1": "LP", "lp_eq_box_tk2": "LP", "lp_eq_box_tk1_us5": "LP",
    # LPs in the reference's sequential .npy format, get_dual_variables=True
    "lp_npy_miplib": "LP", "lp_ineq_box_duals": "LP", "lp_eq_box_tk1_duals": "LP",
    "qp_eq_many": "QP",
}

# linear_solve_method np_solve / np_lstsq / direct, pinned by the reference (make_golden.py extra)
METHOD_CASES = {f"meth_{case}_{meth}": kind
                for case, kind in (("qp_ineq_box", "QP"), ("qp_eq_phase1", "QP"), ("lp_ineq_box", "LP"))
                for meth in ("np_solve", "np_lstsq", "direct")}
# rank-deficient H (LP, n > m, no bounds): np_lstsq, and the Cholesky class on its lstsq backup
# (make_golden.py lstsq_singular) -- minimum-norm steps, where an LU solve has no answer
METHOD_CASES.update({f"lsq_sing_lp{n}_{meth}": "LP" for n in (100, 64) for meth in ("np_lstsq", "cholesky")})
# dense infeasible start + phase 1 with np_lstsq / np_solve / direct (make_golden.py eq_ineq_methods;
# the LU fixtures' envelope includes the reference's sensitivity to its LU's rounding, round 4)
METHOD_CASES.update({f"meth_lp_eq_ineq_{meth}": "LP" for meth in ("np_lstsq", "np_solve", "direct")})

# kwargs that are stored as scalars in the fixture but are not array inputs
_SCALAR_KW = {"t0", "mu", "epsilon", "alpha", "beta", "max_inner_iters", "max_outer_iters",
              "update_slacks_every", "lower_bound", "upper_bound", "linear_solve_method", "get_dual_variables"}


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def solver_kwargs(z):
    kw = {}
    lists = {k[3:-6] for k in z if k.startswith("in_") and k.endswith("_count")}
    for key in lists:
        if key == "A_dense":
            continue
        cnt = int(z[f"in_{key}_count"])
        kw[key] = [z[f"in_{key}_{i}"] for i in range(cnt)]
        kw[key] = [float(v) if np.ndim(v) == 0 else v for v in kw[key]]
    for k, v in z.items():
        if not k.startswith("in_") or k.endswith("_count"):
            continue
        name = k[3:]
        if any(name.startswith(l + "_") and name[len(l) + 1:].isdigit() for l in lists):
            continue
        if name in _SCALAR_KW and np.ndim(v) == 0:
            v = v.item()
        kw[name] = v
    for b in ("lower_bound", "upper_bound"):
        kw.setdefault(b, None)
    return kw
