"""Device-resident problem data + the ipm_problem handle (one per barrier oracle).

All static problem data is copied once to HBM as fp64 torch tensors (row-major,
exactly the NumPy layout the reference hands to CuPy, e.g. LPSolver.py:160-176);
everything the Newton loop touches afterwards stays on the device.
"""
from __future__ import annotations

import ctypes as ct

import numpy as np

from . import _lib as L


def _t(a, dev):
    import torch
    if a is None:
        return None
    if isinstance(a, torch.Tensor):
        return a.to(device=dev, dtype=torch.float64).contiguous()
    return torch.as_tensor(np.ascontiguousarray(np.asarray(a, dtype=np.float64)), device=dev)


def expand_bound(b, n):
    """Scalar or vector bound -> n-vector (the reference broadcasts, FunctionManager.py:131-141)."""
    if b is None:
        return None
    b = np.asarray(b, dtype=np.float64)
    return np.full(n, float(b)) if b.ndim == 0 else b.astype(np.float64, copy=False)



_LS_MODES = {"table": 0, "exact": 1, "compare": 2}
_ls_mode = None


def set_linesearch_mode(mode):
    """Feasible-start backtracking (NewtonSolver.py:157-206) for solves started after this call:
    "table" (default: 64 candidate steps per pass, decisions replayed on the host), "exact"
    (reference-exact: every trial point formed, fresh slacks by GEMV when the reference refreshes
    them, f evaluated directly; one device->host copy per trial), "compare" (both; the exact step is
    taken and disagreements are counted in DeviceProblem.ls_flips / ls_compared).  Default from
    the environment variable IPM_LINESEARCH."""
    global _ls_mode
    if mode not in _LS_MODES:
        raise ValueError(f"linesearch mode must be one of {sorted(_LS_MODES)}")
    _ls_mode = mode


def linesearch_mode():
    import os
    m = _ls_mode or os.environ.get("IPM_LINESEARCH", "table")
    if m not in _LS_MODES:
        raise ValueError(f"IPM_LINESEARCH must be one of {sorted(_LS_MODES)}, got {m!r}")
    return _LS_MODES[m]


class ConeData:
    """Stacked second-order-cone data (ipm_problem_desc SOCP fields).

    X = [dense A_i rows (R) ; c_i (K) ; scratch g_i (K)] row-major (R + 2K) x n.
    Diagonal cones (A_i given as a vector, SOCPSolver.py:285-292) are kept as a_i rows of Ad.
    """

    def __init__(self, A, b, c, d, n, dev):
        import torch
        K = len(A)
        dense_rows, off, dslot, Ad, bd, cb, dids = [], [0], [], [], [], [], []
        for i, Ai in enumerate(A):
            Ai = np.asarray(Ai, dtype=np.float64)
            if Ai.ndim == 2:
                dense_rows.append(Ai)
                off.append(off[-1] + Ai.shape[0])
                if b is not None:
                    cb.append(np.broadcast_to(np.asarray(b[i], dtype=np.float64), (Ai.shape[0],)))
            else:
                off.append(off[-1])
                dids.append(i)
                Ad.append(Ai)
                if b is not None:
                    bd.append(np.broadcast_to(np.asarray(b[i], dtype=np.float64), (n,)))
        R = off[-1]
        X = np.zeros((R + 2 * K, n))
        if R:
            X[:R] = np.vstack(dense_rows)
        if c is not None:
            X[R:R + K] = np.vstack([np.asarray(ci, dtype=np.float64) for ci in c])
        self.K, self.R, self.n = K, R, n
        self.X = _t(X, dev)
        self.off_host = np.asarray(off, dtype=np.int64)
        self.off = torch.as_tensor(self.off_host, device=dev)
        self.cb = _t(np.concatenate(cb), dev) if (b is not None and R) else None
        self.cd = _t(np.asarray([float(v) for v in d]), dev) if d is not None else None
        self.has_c = c is not None
        self.Kd = len(dids)
        self.Ad = _t(np.vstack(Ad), dev) if Ad else None
        self.bd = _t(np.vstack(bd), dev) if (b is not None and bd) else None
        self.dids_host = np.asarray(dids if dids else [0], dtype=np.int64)
        self.dids = torch.as_tensor(self.dids_host, device=dev)


class DeviceProblem:
    """An ipm_problem: static data pointers + workspace.  kind in {'LP','QP','SOCP'}."""

    def __init__(self, kind, n, *, phase1=False, solve_method=L.SOLVE_CHOLESKY, c=None, P=None,
                 q=None, C=None, d=None, lb=None, ub=None, A=None, b=None, AT=None, cones=None,
                 device=0):
        import torch
        self.handle = L.Handle.get(device)
        dev = self.handle.torch_device
        self.dev = dev
        self.hstream = torch.cuda.ExternalStream(self.handle.stream, device=dev)
        self.kind, self.n, self.phase1 = kind, n, phase1
        self.N = n + (1 if phase1 else 0)
        # keep references so the device memory outlives the problem
        self.c, self.P, self.q = _t(c, dev), _t(P, dev), _t(q, dev)
        self.C, self.d = _t(C, dev), _t(d, dev)
        self.lb, self.ub = _t(lb, dev), _t(ub, dev)
        self.A, self.b = _t(A, dev), _t(b, dev)
        self.AT = _t(AT, dev) if AT is not None else (self.A.t().contiguous() if self.A is not None else None)
        self.cones = cones
        desc = L.ProblemDesc()
        desc.kind = {"LP": L.KIND_LP, "QP": L.KIND_QP, "SOCP": L.KIND_SOCP}[kind]
        desc.phase1 = 1 if phase1 else 0
        desc.solve_method = solve_method
        desc.n = n
        dp = L.dptr
        desc.c, desc.P, desc.q = dp(self.c), dp(self.P), dp(self.q)
        desc.ldp = n
        if self.C is not None:
            desc.m, desc.C, desc.ldc, desc.d = self.C.shape[0], dp(self.C), n, dp(self.d)
        desc.lb, desc.ub = dp(self.lb), dp(self.ub)
        if self.A is not None:
            desc.p, desc.A, desc.lda, desc.AT, desc.b = self.A.shape[0], dp(self.A), n, dp(self.AT), dp(self.b)
        if cones is not None:
            desc.K, desc.R, desc.X, desc.ldx = cones.K, cones.R, dp(cones.X), n
            desc.cone_row_off = dp(cones.off)
            desc.cone_row_off_host = cones.off_host.ctypes.data_as(ct.c_void_p)
            desc.cone_b, desc.cone_d = dp(cones.cb), dp(cones.cd)
            desc.has_cone_c = 1 if cones.has_c else 0
            desc.Kd = cones.Kd
            desc.Ad, desc.bd = dp(cones.Ad), dp(cones.bd)
            desc.dcone_id = dp(cones.dids)
            desc.dcone_id_host = cones.dids_host.ctypes.data_as(ct.c_void_p)
        self.desc = desc
        lib = self.handle.lib
        nbytes = lib.ipm_workspace_bytes(ct.byref(desc))
        if nbytes <= 0:
            raise L.IPMBackendError("ipm_workspace_bytes failed")
        self.ws = torch.empty(int(nbytes), dtype=torch.uint8, device=dev)
        ptr = ct.c_void_p()
        self.handle.check(lib.ipm_problem_create(self.handle.ptr, ct.byref(desc), L.dptr(self.ws),
                                                 int(nbytes), ct.byref(ptr)), self.handle.ptr)
        self.ptr = ptr
        self.num_slacks = int(lib.ipm_fm_num_slacks(ptr))

    def __del__(self):
        try:
            if getattr(self, "ptr", None):
                self.handle.lib.ipm_problem_destroy(self.ptr)
                self.ptr = None
        except Exception:
            pass

    # ---- helpers
    def vec(self, a):
        return _t(a, self.dev)

    def check(self, rc):
        self.handle.check(rc, self.handle.ptr)

    def call(self, fn, *args):
        """Run one native entry point ordered against torch's CURRENT stream: the handle's stream
        waits for work queued on the caller's stream (e.g. the facade's clone of x), and the caller's
        stream waits for the native launches before it touches their outputs."""
        import torch
        cur = torch.cuda.current_stream(self.dev)
        other = cur.cuda_stream != self.handle.stream
        if other:
            self.hstream.wait_stream(cur)
        rc = fn(*args)
        if other:
            cur.wait_stream(self.hstream)
        self.check(rc)

    # ---- level 2
    def newton_solve(self, x, t, v, *, max_iters, eps, alpha, beta, update_slacks_every=0,
                     phase1_flag=False, phase1_tol=0.0, use_psd_condition=False):
        o = L.NewtonOpts(int(max_iters), int(update_slacks_every), 1 if phase1_flag else 0,
                         1 if use_psd_condition else 0, float(eps), float(alpha), float(beta),
                         float(phase1_tol))
        o.linesearch_mode = linesearch_mode()
        cap = int(max_iters)
        buf = (ct.c_double * (2 * max(cap, 1)))()
        o.trace = ct.cast(buf, ct.POINTER(ct.c_double))
        o.trace_cap = cap
        r = L.NewtonResult()
        self.call(self.handle.lib.ipm_newton_solve, self.ptr, L.dptr(x), float(t), L.dptr(v), ct.byref(o),
                                                    ct.byref(r))
        k = min(int(r.iters), cap)
        self.last_trace = [(buf[2 * i], buf[2 * i + 1]) for i in range(k)]
        self.ls_compared = getattr(self, "ls_compared", 0) + int(r.ls_compared)
        self.ls_flips = getattr(self, "ls_flips", 0) + int(r.ls_flips)
        return r

    def kkt_flops(self):
        """(KKT SYRK flops per Newton step, 0.0): the second value is the removed deferred-slice
        split, always 0"""
        a, b = ct.c_double(), ct.c_double()
        self.call(self.handle.lib.ipm_kkt_flops, self.ptr, ct.byref(a), ct.byref(b))
        return a.value, b.value

    def time_hbm_kernels(self, reps=20):
        """HIP-event times (ms) of the slack GEMV, the gradient GEMV and one line-search candidate
        pass on this problem's buffers, with their algorithmic HBM bytes -> {kernel: (ms, bytes)}"""
        ms = (ct.c_double * 3)()
        sz = (ct.c_int64 * 3)()
        self.call(self.handle.lib.ipm_problem_sizes, self.ptr, sz)
        self.call(self.handle.lib.ipm_time_hbm_kernels, self.ptr, int(reps), ms)
        m, n, S = int(sz[0]), int(sz[1]), int(sz[2])
        return {"k_gemv_n (slacks: C x)": (ms[0], 8.0 * (m * n + n + m)),
                "k_gemv_t_part (gradient: C^T w)": (ms[1], 8.0 * (m * n + m + n)),
                "k_ls_lin (64 line-search candidates)": (ms[2], 16.0 * S)}

    @property
    def use_backup(self):
        return bool(self.handle.lib.ipm_get_use_backup(self.ptr))

    @use_backup.setter
    def use_backup(self, f):
        self.handle.lib.ipm_set_use_backup(self.ptr, 1 if f else 0)

    # ---- level 1 (oracle protocol)
    def fm_update_x(self, x, update_slacks=True):
        self.call(self.handle.lib.ipm_fm_update_x, self.ptr, L.dptr(x), 1 if update_slacks else 0)

    def fm_slacks(self):
        import torch
        out = torch.empty(max(self.num_slacks, 0), dtype=torch.float64, device=self.dev)
        if self.num_slacks:
            self.call(self.handle.lib.ipm_fm_slacks, self.ptr, L.dptr(out))
        return out

    def fm_objective(self):
        v = ct.c_double()
        self.call(self.handle.lib.ipm_fm_objective, self.ptr, ct.byref(v))
        return v.value

    def fm_newton_objective(self, t):
        v = ct.c_double()
        self.call(self.handle.lib.ipm_fm_newton_objective, self.ptr, float(t), ct.byref(v))
        return v.value

    def fm_gradient(self, t):
        import torch
        g = torch.empty(self.N, dtype=torch.float64, device=self.dev)
        self.call(self.handle.lib.ipm_fm_gradient, self.ptr, float(t), L.dptr(g))
        return g

    def fm_hessian(self, t, diag=False):
        import torch
        if diag:
            H = torch.empty(self.n, dtype=torch.float64, device=self.dev)
            self.call(self.handle.lib.ipm_fm_hessian, self.ptr, float(t), L.dptr(H), self.n)
            return H
        H = torch.empty((self.N, self.N), dtype=torch.float64, device=self.dev)
        self.call(self.handle.lib.ipm_fm_hessian, self.ptr, float(t), L.dptr(H), self.N)
        return H
