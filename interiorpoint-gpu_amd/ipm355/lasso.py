"""LassoSolver: batched ADMM Lasso on the device.

Drop-in for the reference's ``LassoSolver`` (LassoSolver.py:17-236 constructor, :223-337 solve,
:339-485 chunked solve, :487-531 objective, :533-558 prox): same constructor arguments, same
``solve() -> (X, solutions, gaps, iterations)``, same attributes.  All arithmetic runs in
libipm355.so (ipm_lasso.hip): the setup GEMMs / Cholesky / inverse on the fp64-MFMA kernels, then
ONE fused launch per ADMM iteration (x-update GEMM + prox + dual update + stopping-test partial
sums).  Host code here only moves inputs to the device and replays the reference's control flow.

Reference behaviour kept on purpose:
* ``AtA_cache`` only exists with ``add_bias=True``: without it the reference raises AttributeError
  at the Cholesky (LassoSolver.py:124-131 vs 178-183) -- raised here at the same point;
* ``reg`` must have a length (``len(reg)``, LassoSolver.py:109): the default ``reg=1`` raises TypeError;
* ``normalize_A`` divides the CALLER's A in place (LassoSolver.py:122-123);
* ``adaptive_rho`` calls ``cp.linalg.eigvalsh`` and then discards the rho it computes
  (LassoSolver.py:145-156): without CuPy that is a NameError, as in the reference;
* several chunks: per-chunk stopping, ``num_iterations`` holds the last iteration INDEX of each chunk
  and ``gaps`` is returned whole (LassoSolver.py:474-485); the chunk form scales Q as
  ``Q * -m * rho`` (two roundings) and updates ``u = u + (x - alpha)``;
* ``objective()`` takes |alpha| only when ``positive`` (the inverted branch, LassoSolver.py:505-510).
Chunking: the reference sizes chunks for a 1.5 GB CuPy budget when ``use_gpu`` (LassoSolver.py:78-88);
an MI355X holds 288 GB, so there are only as many chunks as ``num_chunks`` asks for (the CPU rule,
LassoSolver.py:89-90), which is also what the parity fixtures pin.
"""
from __future__ import annotations

import ctypes as C
import warnings

import numpy as np

from . import _lib as L


class LassoArgs(C.Structure):
    """ipm_lasso_args (include/ipm355.h)."""
    _fields_ = [("n", L.I64), ("S", L.I64), ("m", L.I64), ("lds", L.I64),
                ("Qs", L.P), ("ldq", L.I64), ("bA", L.P), ("ldba", L.I64), ("eta", L.P),
                ("x", L.P), ("alpha", L.P), ("u", L.P), ("W0", L.P), ("W1", L.P), ("partial", L.P),
                ("rho", L.F64), ("eps_abs", L.F64), ("eps_rel", L.F64), ("stop_multiplier", L.F64),
                ("max_iters", L.I32), ("check_stop", L.I32), ("positive", L.I32), ("add_bias", L.I32),
                ("dual_form", L.I32), ("compute_loss", L.I32),
                ("ba_bcast", L.I32), ("eta_bcast", L.I32), ("b_bcast", L.I32), ("reg_bcast", L.I32),
                ("AT", L.P), ("ldat", L.I64), ("b", L.P), ("ldb", L.I64), ("reg", L.P), ("R", L.P),
                ("gaps", L.P), ("ldg", L.I64), ("gap_cols", L.P), ("qs_blocked", L.I32)]


def _dev(a, dev):
    import torch
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=dev).clone()


class LassoSolver:
    def __init__(self, A, b, reg=1, rho=0.4, max_iters=1000, check_stop=10, add_bias=False, normalize_A=False,
                 positive=False, compute_loss=False, adaptive_rho=False, eps_abs=1e-4, eps_rel=3e-2, use_gpu=False,
                 num_chunks=0, check_cvxpy=True, device=0):
        import torch
        self.h = L.Handle.get(device)
        self.lib = self.h.lib
        self.dev = torch.device("cuda", device)
        self.use_gpu = True
        self.num_chunks = max(1, num_chunks)
        self.A = A
        self.b = b
        if self.b.ndim < 2:
            self.b = self.b[:, None]
        self.reg, self.rho, self.max_iters, self.check_stop = reg, rho, max_iters, check_stop
        self.compute_loss, self.positive, self.add_bias = compute_loss, positive, add_bias
        self.EPS_ABS, self.EPS_REL = eps_abs, eps_rel
        assert len(reg) == self.b.shape[1] or len(reg) == 1 or self.b.shape[1] == 1
        self.num_samples = max(self.b.shape[1], len(self.reg))
        self.gaps = np.zeros((self.max_iters, self.num_samples))
        self.m, self.n = self.A.shape
        h, lib = self.h, self.lib
        Ad = _dev(A, self.dev)
        if normalize_A:
            if not np.issubdtype(np.asarray(A).dtype, np.floating):
                raise TypeError(f"Cannot cast ufunc 'divide' output from dtype('float64') to dtype('{A.dtype}') "
                                f"with casting rule 'same_kind'")
            h.check(lib.ipm_lasso_colnorm(h.ptr, self.m, self.n, L.dptr(Ad), self.n, L.P(0)), h.ptr)
            np.copyto(A, Ad.cpu().numpy())          # the caller's array, like the reference's A /= std
        if self.add_bias:
            Ab = torch.empty((self.m, self.n + 1), dtype=torch.float64, device=self.dev)
            h.check(lib.ipm_lasso_bias(h.ptr, self.m, self.n, L.dptr(Ad), self.n, L.dptr(Ab), self.n + 1), h.ptr)
            Ad = Ab
        self.n = int(Ad.shape[1])
        self.A_dev = Ad
        self.feasible, self.cvxpy_vals, self.cvxpy_sols = None, None, None
        if check_cvxpy:
            warnings.warn("check_cvxpy=True: the CVXPY comparison is not part of the HIP path (cvxpy is not "
                          "installed here); skipped")
        if not self.add_bias:
            # LassoSolver.py:178-183 reads self.AtA_cache, which only add_bias creates (:124-131)
            raise AttributeError("'LassoSolver' object has no attribute 'AtA_cache'")
        if adaptive_rho:
            raise NameError("name 'cp' is not defined")   # LassoSolver.py:147 (cp.linalg.eigvalsh)
        n = self.n
        # Qinv and its transpose: the transpose is the k-major operand of every product with Qinv
        # (Qinv itself is scratch of the solve: only the transpose is kept)
        Qinv = torch.empty((n, n), dtype=torch.float64, device=self.dev)
        self.QinvT = torch.empty((n, n), dtype=torch.float64, device=self.dev)
        info = C.c_int(0)
        rc = lib.ipm_lasso_qinv(h.ptr, self.m, n, L.dptr(Ad), n, float(rho), L.dptr(Qinv), L.dptr(self.QinvT),
                                n, C.byref(info))
        del Qinv
        if rc == L.IPM_NOT_POSITIVE_DEFINITE:
            raise np.linalg.LinAlgError(f"{info.value}-th leading minor of the array is not positive definite")
        h.check(rc, h.ptr)
        self.X = np.zeros((self.n, self.b.shape[1]))
        self._AT = None
        self._R = None
        if self.num_chunks == 1:
            self.solve_func = self._run_admm
            self.b = np.array(self.b)
            self.reg = np.array(reg)
            self.stop_multiplier = self.EPS_ABS * np.sqrt(self.n * self.num_samples)
            self.eta = self.reg / self.rho
            self._b_dev = _dev(self.b, self.dev)
            self.bA_cache = self._bA(self._b_dev)
            # Qinv_cache *= -m * rho (LassoSolver.py:220): in place on the transpose, which is all
            # the iteration reads
            h.check(lib.ipm_lasso_scale(h.ptr, n, n, L.dptr(self.QinvT), n, -self.m * self.rho, 1.0, 0), h.ptr)
            self.Qs = self._blocked(self.QinvT)
            self.QinvT = None           # the blocked copy is all the iteration reads from here on
        else:
            self._Qs_chunks = None      # the chunks' blocked Qs, built at the first solve
            self.solve_func = self._run_admm_chunks

    # ---------------------------------------------------------------------------------------
    def _bA(self, bdev):
        """Qinv (A^T b) (LassoSolver.py:214-219): A^T b, then Qinv (.) -- two MFMA GEMMs."""
        import torch
        h, n, Sb = self.h, self.n, int(bdev.shape[1])
        AtB = torch.empty((n, Sb), dtype=torch.float64, device=self.dev)
        h.check(self.lib.ipm_gemm_tn(h.ptr, n, Sb, self.m, 1.0, L.dptr(self.A_dev), n, L.dptr(bdev), Sb, 0.0,
                                     L.dptr(AtB), Sb), h.ptr)
        bA = torch.empty((n, Sb), dtype=torch.float64, device=self.dev)
        h.check(self.lib.ipm_gemm_tn(h.ptr, n, Sb, n, 1.0, L.dptr(self.QinvT), n, L.dptr(AtB), Sb, 0.0,
                                     L.dptr(bA), Sb), h.ptr)
        return bA

    def _blocked(self, Qs):
        """The ADMM step's tile-blocked copy of Qs (ipm_lasso_block_qs): each workgroup of the
        iteration GEMM then streams one contiguous span of it."""
        import torch
        n = self.n
        Qb = torch.empty(int(self.lib.ipm_lasso_qb_doubles(n)), dtype=torch.float64, device=self.dev)
        self.h.check(self.lib.ipm_lasso_block_qs(self.h.ptr, n, L.dptr(Qs), n, L.dptr(Qb)), self.h.ptr)
        return Qb

    def _loss_buffers(self, S):
        import torch
        if self._AT is None:
            self._AT = torch.empty((self.n, self.m), dtype=torch.float64, device=self.dev)
            h = self.h
            h.check(self.lib.ipm_transpose(h.ptr, self.m, self.n, L.dptr(self.A_dev), self.n, L.dptr(self._AT),
                                           self.m), h.ptr)
        if self._R is None or self._R.numel() < self.m * S:
            self._R = torch.empty(self.m * S, dtype=torch.float64, device=self.dev)
        return self._AT, self._R

    def _args(self, S, bA, Qs, eta, bdev, reg, dual_form, stop_mult, gaps_dev, gap_cols):
        import torch
        z = lambda: torch.zeros((self.n, S), dtype=torch.float64, device=self.dev)  # noqa: E731
        st = dict(x=z(), alpha=z(), u=z(), W0=z(), W1=z(),
                  partial=torch.zeros(int(self.lib.ipm_lasso_partial_doubles(self.n, S)), dtype=torch.float64,
                                      device=self.dev),
                  eta=_dev(np.atleast_1d(eta), self.dev), reg=_dev(np.atleast_1d(reg), self.dev))
        a = LassoArgs()
        a.n, a.S, a.m, a.lds = self.n, S, self.m, S
        a.Qs, a.ldq, a.qs_blocked = L.dptr(Qs), self.n, 1   # Qs: the tile-blocked copy (_blocked)
        a.bA, a.ldba, a.ba_bcast = L.dptr(bA), int(bA.shape[1]), int(bA.shape[1] == 1 and S > 1)
        a.eta, a.eta_bcast = L.dptr(st["eta"]), int(st["eta"].numel() == 1 and S > 1)
        for k in ("x", "alpha", "u", "W0", "W1", "partial"):
            setattr(a, k, L.dptr(st[k]))
        a.rho, a.eps_abs, a.eps_rel, a.stop_multiplier = float(self.rho), float(self.EPS_ABS), float(self.EPS_REL), \
            float(stop_mult)
        a.max_iters, a.check_stop = int(self.max_iters), int(self.check_stop)
        a.positive, a.add_bias, a.dual_form = int(bool(self.positive)), int(bool(self.add_bias)), dual_form
        a.compute_loss = int(bool(self.compute_loss))
        a.b, a.ldb, a.b_bcast = L.dptr(bdev), int(bdev.shape[1]), int(bdev.shape[1] == 1 and S > 1)
        a.reg, a.reg_bcast = L.dptr(st["reg"]), int(st["reg"].numel() == 1 and S > 1)
        AT, R = self._loss_buffers(S)            # the final loss needs them too
        a.AT, a.ldat, a.R = L.dptr(AT), self.m, L.dptr(R)
        a.gaps, a.ldg = (L.dptr(gaps_dev), self.num_samples) if gaps_dev is not None else (L.P(0), 0)
        a.gap_cols = L.dptr(gap_cols)
        return a, st

    def _run(self, a):
        if self.check_stop == 0:
            raise ZeroDivisionError("integer modulo by zero")
        if self.max_iters <= 0:
            raise UnboundLocalError("local variable 'iteration' referenced before assignment")
        it = C.c_int32(0)
        self.h.check(self.lib.ipm_lasso_admm(self.h.ptr, C.byref(a), C.byref(it)), self.h.ptr)
        return int(it.value)

    def _loss(self, a, absm, out, cols=None):
        self.h.check(self.lib.ipm_lasso_loss(self.h.ptr, C.byref(a), absm, L.dptr(out), L.dptr(cols)), self.h.ptr)

    def solve(self):
        return self.solve_func()

    def _run_admm(self):
        """LassoSolver.py:240-337."""
        import torch
        S = self.num_samples
        gaps_dev = torch.zeros((self.max_iters, S), dtype=torch.float64, device=self.dev) if self.compute_loss \
            else None
        a, st = self._args(S, self.bA_cache, self.Qs, self.eta, self._b_dev, self.reg, 0, self.stop_multiplier,
                           gaps_dev, None)
        it = self._run(a)
        sol = torch.empty(S, dtype=torch.float64, device=self.dev)
        self._loss(a, 0 if self.positive else 1, sol)
        self._state, self._a = st, a
        self.x, self.alpha, self.u = st["x"], st["alpha"], st["u"]
        self.solutions = sol.cpu().numpy()
        if gaps_dev is not None:
            self.gaps = gaps_dev.cpu().numpy()
        self.X = self.alpha.cpu().numpy()
        self.num_iterations = [it + 1]
        return self.X, self.solutions, self.gaps[: it + 1], it + 1

    def _run_admm_chunks(self):
        """LassoSolver.py:339-485: columns i::num_chunks solved one chunk after another."""
        import torch
        self.num_iterations = []
        self.solutions = np.empty(self.num_samples)
        reg_is_array = isinstance(self.reg, np.ndarray)
        n = self.n
        key = (self.m, float(self.rho))
        if self._Qs_chunks is None or self._Qs_chunks[0] != key:
            # Qinv_cache * -self.m * self.rho, left to right (LassoSolver.py:386): built once per
            # (m, rho) and reused by every solve
            Qs = torch.empty((n, n), dtype=torch.float64, device=self.dev)
            self.h.check(self.lib.ipm_copy(self.h.ptr, L.dptr(Qs), L.dptr(self.QinvT), n * n), self.h.ptr)
            self.h.check(self.lib.ipm_lasso_scale(self.h.ptr, n, n, L.dptr(Qs), n, float(-self.m), float(self.rho),
                                                  1), self.h.ptr)
            self._Qs_chunks = (key, self._blocked(Qs))
            del Qs
        Qs = self._Qs_chunks[1]
        gaps_dev = torch.zeros((self.max_iters, self.num_samples), dtype=torch.float64, device=self.dev) \
            if self.compute_loss else None
        indices = np.array(range(self.b.shape[1]))
        for i in range(self.num_chunks):
            cols = indices[i::self.num_chunks]
            b_iter = np.array(self.b[..., cols])
            S = b_iter.shape[1]
            iter_reg = np.array(self.reg[cols]) if reg_is_array else np.array(self.reg)
            stop_mult = self.EPS_ABS * np.sqrt(self.n * S)
            eta = iter_reg / self.rho
            bdev = _dev(b_iter, self.dev)
            bA = self._bA(bdev)
            cols_dev = torch.as_tensor(cols.astype(np.int64), device=self.dev)
            a, st = self._args(S, bA, Qs, eta, bdev, iter_reg, 1, stop_mult, gaps_dev, cols_dev)
            it = self._run(a)
            sol = torch.empty(S, dtype=torch.float64, device=self.dev)
            self._loss(a, 0 if self.positive else 1, sol)
            self.solutions[cols] = sol.cpu().numpy()
            self.X[:, cols] = st["alpha"].cpu().numpy()
            self.num_iterations.append(it)
        if gaps_dev is not None:
            self.gaps = gaps_dev.cpu().numpy()
        return self.X, self.solutions, self.gaps, self.num_iterations

    def objective(self):
        """LassoSolver.py:487-531 (CPU branch: |alpha| only when positive)."""
        import torch
        if not hasattr(self, "_a"):
            raise AttributeError("'LassoSolver' object has no attribute 'alpha'")
        out = torch.empty(self.num_samples, dtype=torch.float64, device=self.dev)
        self._loss(self._a, 1 if self.positive else 0, out)
        return out.cpu().numpy()

    def prox(self, v, eta):
        """LassoSolver.py:533-558 on the device (v: n x S, eta: S or scalar) -> NumPy array."""
        import torch
        v = np.asarray(v, dtype=np.float64)
        v2 = v if v.ndim == 2 else v[:, None]
        S = v2.shape[1]
        vd = _dev(v2, self.dev)
        ed = _dev(np.atleast_1d(eta), self.dev)
        out = torch.empty_like(vd)
        self.h.check(self.lib.ipm_lasso_prox(self.h.ptr, v2.shape[0], S, L.dptr(vd), S, L.dptr(ed),
                                             int(ed.numel() == 1 and S > 1), int(bool(self.positive)),
                                             int(bool(self.add_bias)), L.dptr(out), S), self.h.ptr)
        r = out.cpu().numpy()
        return r if v.ndim == 2 else r[:, 0]

    def plot(self, iteration_start=0, iteration_end=-1, subtract_opt=True):
        """LassoSolver.py:560-597 (matplotlib)."""
        if not self.compute_loss:
            raise ValueError("Need to solve problem with compute_loss set to True to be able to plot convergence!")
        import matplotlib.pyplot as plt
        if iteration_end == -1:
            iteration_end = self.num_iterations
        elif not isinstance(iteration_end, list):
            iteration_end = list(iteration_end)
        ax = plt.subplot()
        for i in range(self.gaps.shape[1]):
            g = self.gaps[iteration_start: iteration_end[i % self.num_chunks], i]
            if subtract_opt:
                mn = g.min()
                if self.cvxpy_vals is not None:
                    mn = min(self.cvxpy_vals[i], mn)
                ax.plot(g[:-1] - mn)
            else:
                ax.plot(g)
        ax.set_ylabel("Optimality gap")
        ax.set_xlabel("iteration number")
        ax.set_title("Convergence of LassoSolver")
        ax.set_yscale("log")
        return ax
