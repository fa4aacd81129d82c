"""ctypes binding of libipm355.so (include/ipm355.h).

The product path has NO CPU fallback: if the HIP library is missing, or no
MI355X is visible, importing the solvers still works but constructing one
raises ``IPMBackendError`` (loudly, with the reason).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("IPM355_LIB", os.path.join(_HERE, "libipm355.so"))   # override: experiments only

IPM_OK = 0
IPM_NOT_POSITIVE_DEFINITE = 1
IPM_INVALID_ARG = 2
IPM_HIP_ERROR = 3
IPM_NOT_SUPPORTED = 4
IPM_LINALG_NOT_CONVERGED = 5

KIND_LP, KIND_QP, KIND_SOCP = 0, 1, 2
SOLVE_CHOLESKY, SOLVE_DIAGONAL, SOLVE_LU, SOLVE_LSTSQ, SOLVE_DIAGONAL_LSTSQ = 0, 1, 2, 3, 4
LS_TABLE, LS_EXACT, LS_COMPARE = 0, 1, 2

P = C.c_void_p
I32 = C.c_int32
I64 = C.c_int64
F64 = C.c_double


class IPMBackendError(RuntimeError):
    """The HIP backend is unavailable or failed (never silently replaced by a CPU path)."""


class ProblemDesc(C.Structure):
    """ipm_problem_desc (include/ipm355.h)."""
    _fields_ = [
        ("kind", I32), ("phase1", I32), ("solve_method", I32), ("reserved0", I32),
        ("n", I64),
        ("c", P), ("P", P), ("ldp", I64), ("q", P),
        ("m", I64), ("C", P), ("ldc", I64), ("d", P),
        ("lb", P), ("ub", P),
        ("p", I64), ("A", P), ("lda", I64), ("AT", P), ("b", P),
        ("K", I64), ("R", I64), ("X", P), ("ldx", I64),
        ("cone_row_off", P), ("cone_row_off_host", P), ("cone_b", P), ("cone_d", P),
        ("has_cone_c", I32), ("reserved1", I32),
        ("Kd", I64), ("Ad", P), ("bd", P), ("dcone_id", P), ("dcone_id_host", P),
    ]


class NewtonOpts(C.Structure):
    _fields_ = [("max_iters", I32), ("update_slacks_every", I32), ("phase1_flag", I32),
                ("use_psd_condition", I32), ("eps", F64), ("alpha", F64), ("beta", F64),
                ("phase1_tol", F64), ("trace", C.POINTER(F64)), ("trace_cap", I32), ("linesearch_mode", I32)]


class NewtonResult(C.Structure):
    _fields_ = [("iters", I32), ("success", I32), ("stat_valid", I32), ("use_backup", I32),
                ("stat", F64), ("last_step", F64), ("backtracks", I64), ("ls_compared", I64),
                ("ls_flips", I64), ("linalg_error", I64)]


EXPORTS = {
    "ipm_version": (C.c_int, []),
    "ipm_create": (C.c_int, [C.c_int, P, C.POINTER(P)]),
    "ipm_destroy": (C.c_int, [P]),
    "ipm_last_error": (C.c_char_p, [P]),
    "ipm_workspace_bytes": (I64, [C.POINTER(ProblemDesc)]),
    "ipm_problem_create": (C.c_int, [P, C.POINTER(ProblemDesc), P, I64, C.POINTER(P)]),
    "ipm_problem_destroy": (C.c_int, [P]),
    "ipm_newton_solve": (C.c_int, [P, P, F64, P, C.POINTER(NewtonOpts), C.POINTER(NewtonResult)]),
    "ipm_get_use_backup": (C.c_int, [P]),
    "ipm_set_use_backup": (C.c_int, [P, C.c_int]),
    "ipm_fm_update_x": (C.c_int, [P, P, C.c_int]),
    "ipm_fm_slacks": (C.c_int, [P, P]),
    "ipm_fm_num_slacks": (I64, [P]),
    "ipm_fm_objective": (C.c_int, [P, C.POINTER(F64)]),
    "ipm_fm_newton_objective": (C.c_int, [P, F64, C.POINTER(F64)]),
    "ipm_fm_gradient": (C.c_int, [P, F64, P]),
    "ipm_fm_hessian": (C.c_int, [P, F64, P, I64]),
    "ipm_gemv": (C.c_int, [P, C.c_int, I64, I64, F64, P, I64, P, F64, P]),
    "ipm_syrk": (C.c_int, [P, I64, I64, P, I64, P, F64, F64, P, I64]),
    "ipm_potrf": (C.c_int, [P, I64, P, I64, C.POINTER(C.c_int)]),
    "ipm_potrf_partial": (C.c_int, [P, I64, I64, P, I64, C.POINTER(C.c_int)]),
    "ipm_potrs": (C.c_int, [P, I64, I64, P, I64, P, I64]),
    "ipm_getrf": (C.c_int, [P, I64, P, I64, P, C.POINTER(C.c_int)]),
    "ipm_getrs": (C.c_int, [P, I64, I64, P, I64, P, P, I64]),
    "ipm_lstsq_sym": (C.c_int, [P, I64, I64, P, I64, P, I64, C.POINTER(C.c_int)]),
    "ipm_last_timings": (C.c_int, [P, C.POINTER(F64), C.POINTER(F64), C.POINTER(F64)]),
    "ipm_kkt_flops": (C.c_int, [P, C.POINTER(F64), C.POINTER(F64)]),
    "ipm_time_hbm_kernels": (C.c_int, [P, C.c_int, C.POINTER(F64)]),
    "ipm_problem_sizes": (C.c_int, [P, C.POINTER(I64)]),
    "ipm_set_timing": (C.c_int, [P, C.c_int]),
    "ipm_debug_set_trsv_spin_limit": (C.c_int, [C.c_uint]),
    "ipm_debug_set_trsv_publish_delay": (C.c_int, [C.c_int]),
    "ipm_debug_set_potrf_spin_limit": (C.c_int, [C.c_uint]),
    "ipm_debug_lstsq_fail_call": (C.c_int, [C.c_int]),
    # batched ADMM Lasso (ipm_lasso.hip; ipm355/lasso.py)
    "ipm_gemm_tn": (C.c_int, [P, I64, I64, I64, F64, P, I64, P, I64, F64, P, I64]),
    "ipm_transpose": (C.c_int, [P, I64, I64, P, I64, P, I64]),
    "ipm_copy": (C.c_int, [P, P, P, I64]),
    "ipm_lasso_colnorm": (C.c_int, [P, I64, I64, P, I64, P]),
    "ipm_lasso_bias": (C.c_int, [P, I64, I64, P, I64, P, I64]),
    "ipm_lasso_qinv": (C.c_int, [P, I64, I64, P, I64, F64, P, P, I64, C.POINTER(C.c_int)]),
    "ipm_lasso_scale": (C.c_int, [P, I64, I64, P, I64, F64, F64, C.c_int]),
    "ipm_lasso_prox": (C.c_int, [P, I64, I64, P, I64, P, C.c_int, C.c_int, C.c_int, P, I64]),
    "ipm_lasso_loss": (C.c_int, [P, P, C.c_int, P, P]),
    "ipm_lasso_partial_doubles": (I64, [I64, I64]),
    "ipm_lasso_admm": (C.c_int, [P, P, C.POINTER(C.c_int32)]),
    "ipm_lasso_qb_doubles": (I64, [I64]),
    "ipm_lasso_block_qs": (C.c_int, [P, I64, P, I64, P]),
}

_lib = None


def load_library(path: str = LIB_PATH):
    """Load libipm355.so and declare every exported symbol. Raises IPMBackendError."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise IPMBackendError(f"HIP library not built: {path} (run `make` or __graft_entry__.build())")
    try:
        lib = C.CDLL(path)
    except OSError as e:
        raise IPMBackendError(f"cannot load {path}: {e}") from e
    default = os.path.join(_HERE, "libipm355.so")
    for name, (res, args) in EXPORTS.items():
        if path != default and not hasattr(lib, name):
            continue          # an older build under IPM355_LIB (A/B experiments): only what it has
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class Handle:
    """One ipm_handle per (process, device, stream): bound to torch's CURRENT stream at creation.

    Solvers built under different `torch.cuda.stream(...)` contexts get different handles, so
    independent instances can run concurrently from host threads (the C calls release the GIL).
    """

    _cache = {}

    def __init__(self, device: int = 0, stream: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise IPMBackendError("no HIP device visible: the ipm355 solvers run on MI355X only")
        self.lib = load_library()
        self.device = device
        self.stream = stream
        self.torch_device = torch.device("cuda", device)
        h = P()
        self.check(self.lib.ipm_create(device, P(stream), C.byref(h)), None)
        self.ptr = h

    @classmethod
    def get(cls, device: int = 0) -> "Handle":
        import torch
        if not torch.cuda.is_available():
            raise IPMBackendError("no HIP device visible: the ipm355 solvers run on MI355X only")
        with torch.cuda.device(device):
            stream = torch.cuda.current_stream(device).cuda_stream
        key = (device, stream)
        h = cls._cache.get(key)
        if h is None:
            h = cls(device, stream)
            cls._cache[key] = h
        return h

    def check(self, rc, h=None):
        if rc == IPM_OK:
            return
        msg = self.lib.ipm_last_error(h if h is not None else getattr(self, "ptr", None))
        msg = msg.decode() if msg else ""
        if rc == IPM_NOT_POSITIVE_DEFINITE:
            raise np.linalg.LinAlgError(f"matrix not positive definite ({msg})")
        if rc == IPM_LINALG_NOT_CONVERGED:
            raise np.linalg.LinAlgError(f"SVD did not converge in Linear Least Squares ({msg})")
        raise IPMBackendError(f"ipm355 error {rc}: {msg}")


def dptr(t) -> P:
    """device pointer of a torch tensor (or None)."""
    return P(t.data_ptr()) if t is not None else P(0)
