"""CPU oracle for the interior-point Newton hot path -- TEST INFRASTRUCTURE ONLY.

This module is a NumPy/SciPy restatement of the reference's barrier method
(fdeguire03/InteriorPoint-GPU @ /root/reference).  It exists so that tests,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg have a
checker; the product path (``interiorpoint-gpu_amd/ipm355``) never imports it.

Parity status: PINNED.  ``tests/golden/make_golden.py`` runs the reference
itself in the build container and stores inputs + outputs (per-function
values, per-iteration step sizes, final x*, objective values, phase-1 known
answers, the group-lasso SOCP known answer) under ``tests/golden/``;
``tests/test_oracle_golden.py`` checks this module against those vectors.

Every class/function below cites the reference lines whose semantics it
restates, including the numerically significant quirks listed in SURVEY.md
§8.1 (Q1-Q16): stale slacks in the line search, the one-step lag of the
Armijo loop, ``grad.x`` in the Armijo right-hand side, permanent fallback
after one Cholesky failure, the ``+c c^T`` SOCP Hessian term, the epsilon
constants.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg

EPS_LOG = 1e-15     # FunctionManager.py:223-227, 244-246 (log / reciprocal guard)
EPS_CONE = 1e-12    # FunctionManager.py:1084-1098, 1136, 1152-1154 (SOCP cone guard)
STEP_FLOOR = 1e-13  # NewtonSolver.py:176, 190; NewtonSolverInfeasibleStart.py:187, 243


class LinAlgFallback(Exception):
    pass


# --------------------------------------------------------------------------------------
# L1: barrier oracles (FunctionManager.py)
# --------------------------------------------------------------------------------------

class _BarrierBase:
    """Dirty-flag protocol of FunctionManager.py:94-116.

    update_x() marks every cached quantity stale; update_t() marks only the
    t-dependent ones (objective, barrier objective, gradient) stale -- the
    Hessian is NOT invalidated by t (FunctionManager.py:114-116), which is
    harmless because every Newton iteration calls gradient(x) first.
    """

    def _mark_all(self):
        self.dirty_obj = self.dirty_nobj = self.dirty_grad = True
        self.dirty_hess = self.dirty_ihess = True

    def update_t(self, t):
        if self.t != t:
            self.t = t
            self.dirty_obj = self.dirty_nobj = self.dirty_grad = True


class LPBarrier(_BarrierBase):
    """FunctionManagerLP (FunctionManager.py:11-356).

    slacks = [d - Cx | ub - x | x - lb]   (segments present only if given)
    psi    = t c.x - sum log(s + 1e-15)
    grad   = t c - 1/(s_lb+eps) + 1/(s_ub+eps) + C^T 1/(s_C+eps)
    hess   = C^T diag(1/(s_C+eps)^2) C + diag(1/s_lb^2 + 1/s_ub^2)  (bounds: NO eps)
    """

    def __init__(self, c=None, C=None, d=None, x0=None, lb=None, ub=None, t=1,
                 try_diag=True, n=None):
        self.C, self.d, self.lb, self.ub = C, d, lb, ub
        self.x = x0
        self.t = t
        self.try_diag = try_diag
        self.bounded = lb is not None or ub is not None
        self.constrained = C is not None or self.bounded
        if c is None:
            c = np.ones(len(x0) if x0 is not None else n)
        self.c = c
        nx = len(x0) if x0 is not None else n
        off = 0
        self.seg_C = self.seg_ub = self.seg_lb = None
        if C is not None:
            self.seg_C = slice(0, len(C)); off = len(C)
        if ub is not None:
            self.seg_ub = slice(off, off + nx); off += nx
        if lb is not None:
            self.seg_lb = slice(off, off + nx)
        self.slacks = None
        self.inv_slacks = None
        self.dirty_islacks = True
        self.obj = self.nobj = self.grad = self.hess = self.inv_hess = None
        self._mark_all()

    # FunctionManager.py:118-149
    def _refresh_slacks(self):
        parts = []
        if self.d is not None:
            parts.append(self.d - self.C @ self.x)
        if self.ub is not None:
            parts.append(self.ub - self.x)
        if self.lb is not None:
            parts.append(self.x - self.lb)
        s = parts[0]
        for p in parts[1:]:
            s = np.append(s, p)
        self.slacks = s.ravel() if s.ndim > 1 else s
        self.dirty_islacks = True

    # FunctionManager.py:94-103 + 199-206
    def update_x(self, x, update_slacks=True):
        self.x = x
        self._mark_all()
        self.dirty_islacks = True
        if self.constrained and update_slacks:
            self._refresh_slacks()

    def _inv(self):
        if self.constrained and self.dirty_islacks:
            self.inv_slacks = 1 / (self.slacks + EPS_LOG)
            self.dirty_islacks = False
        return self.inv_slacks

    def objective(self, x=None):  # FunctionManager.py:151-162
        if x is not None:
            self.update_x(x)
        elif not self.dirty_obj:
            return self.obj
        self.obj = self.c.dot(self.x)
        self.dirty_obj = False
        return self.obj

    def _barrier_value(self, s):
        return np.log(s + EPS_LOG).sum()

    def newton_objective(self, x=None, t=None):  # FunctionManager.py:208-230
        if x is not None:
            self.update_x(x)
        if t is not None:
            self.update_t(t)
        if not self.dirty_nobj:
            return self.nobj
        val = self.t * self.objective()
        if self.constrained:
            val = val - self._barrier_value(self.slacks)
        self.nobj = val
        self.dirty_nobj = False
        return val

    def _objective_gradient(self):
        return self.t * self.c

    def gradient(self, x=None, t=None):  # FunctionManager.py:232-265
        if x is not None:
            self.update_x(x)
        if t is not None:
            self.update_t(t)
        if not self.dirty_grad:
            return self.grad
        inv = self._inv()
        g = self._objective_gradient()
        if self.lb is not None:
            g -= inv[self.seg_lb]
        if self.ub is not None:
            g += inv[self.seg_ub]
        if self.C is not None:
            g += self.C.T @ inv[self.seg_C]
        self.grad = g
        self.dirty_grad = False
        return g

    def _bound_diag(self, H):
        dg = np.einsum("ii->i", H)
        if self.lb is not None:
            dg += 1 / (self.slacks[self.seg_lb]) ** 2
        if self.ub is not None:
            dg += 1 / (self.slacks[self.seg_ub]) ** 2

    def hessian(self, x=None):  # FunctionManager.py:267-326
        if x is not None:
            self.update_x(x)
        if not self.dirty_hess:
            return self.hess
        inv = self._inv()
        if self.C is None:
            if self.try_diag and self.bounded:
                # diagonal Hessian vector (WITH eps): FunctionManager.py:283-292
                if self.lb is not None:
                    h = inv[self.seg_lb] ** 2
                    if self.ub is not None:
                        h += inv[self.seg_ub] ** 2
                else:
                    h = inv[self.seg_ub] ** 2
                self.hess = h
                return h
            H = np.zeros((len(self.x), len(self.x)))
        else:
            H = self.C.T @ ((inv[self.seg_C] ** 2)[:, None] * self.C)
        if self.bounded:
            self._bound_diag(H)
        self.hess = H
        self.dirty_hess = False
        return H

    def inv_hessian(self, x=None):  # FunctionManager.py:328-356
        if x is not None:
            self.update_x(x)
        if not self.dirty_ihess:
            return self.inv_hess
        if self.C is None and self.try_diag:
            if self.bounded:
                self.inv_hess = 1 / self.hessian()
            else:
                self.hess = np.zeros((len(self.x), len(self.x)))
        else:
            raise ValueError("Hessian is not diagonal, cannot use inv hessian function!")
        self.dirty_ihess = False
        return self.inv_hess


class QPBarrier(LPBarrier):
    """FunctionManagerQP (FunctionManager.py:619-831): f = 1/2 x'Px + q'x.

    grad = t (Px + q) - 1/(s_lb+eps) + 1/(s_ub+eps) + C^T 1/(s_C+eps)
    hess = t P + C^T diag(1/(s_C+eps)^2) C + diag(1/s_lb^2 + 1/s_ub^2)
    """

    def __init__(self, P=None, q=None, C=None, d=None, x0=None, lb=None, ub=None, t=1, n=None):
        super().__init__(c=np.zeros(1), C=C, d=d, x0=x0, lb=lb, ub=ub, t=t, try_diag=False, n=n)
        self.P, self.q = P, q

    def objective(self, x=None):  # FunctionManager.py:682-704
        if x is not None:
            self.update_x(x)
        elif not self.dirty_obj:
            return self.obj
        val = 0
        if self.P is not None:
            val += 1 / 2 * self.x.dot(self.P @ self.x)
        if self.q is not None:
            val += self.q.dot(self.x)
        self.obj = val
        self.dirty_obj = False
        return val

    def _objective_gradient(self):  # FunctionManager.py:759-764
        g = self.P @ self.x
        if self.q is not None:
            g += self.q
        g *= self.t
        return g

    def hessian(self, x=None):  # FunctionManager.py:783-827
        if x is not None:
            self.update_x(x)
        if not self.dirty_hess:
            return self.hess
        inv = self._inv()
        H = self.t * self.P
        if self.C is not None:
            H += self.C.T @ ((inv[self.seg_C] ** 2)[:, None] * self.C)
        if self.bounded:
            self._bound_diag(H)
        self.hess = H
        self.dirty_hess = False
        return H

    def inv_hessian(self, x=None):
        raise ValueError("Hessian is not diagonal, cannot use inv hessian function!")


class Phase1Barrier(_BarrierBase):
    """FunctionManagerPhase1 (FunctionManager.py:359-616).

    Variables x~ = (x, s); sigma = [s + d - Cx | s + ub - x | s + x - lb];
    s0 = -min(slacks at s=0) + 1 (FunctionManager.py:390-393).
    psi  = t s - sum log(sigma + eps)
    grad = [C^T inv_C - inv_lb + inv_ub ; t - sum inv]         inv = 1/(sigma+eps)
    hess = [[C^T diag(inv_C^2) C + diag(inv_lb^2 + inv_ub^2), -C^T inv_C^2 + inv_lb^2 - inv_ub^2],
            [(same)^T, sum inv^2]]
    """

    def __init__(self, C=None, d=None, x0=None, lb=None, ub=None, t=1, n=None):
        self.C, self.d, self.lb, self.ub = C, d, lb, ub
        self.x = x0
        self.t = t
        self.s = 0
        self._refresh_slacks()
        self.s = -self.slacks.min() + 1
        self._refresh_slacks()
        self.bounded = lb is not None or ub is not None
        self.constrained = True
        nx = len(x0)
        self.seg_C = slice(0, len(C))
        off = len(C)
        self.seg_ub = self.seg_lb = None
        if ub is not None:
            self.seg_ub = slice(off, off + nx); off += nx
        if lb is not None:
            self.seg_lb = slice(off, off + nx)
        self.inv_slacks = None
        self.dirty_islacks = True
        self.obj = self.nobj = self.grad = self.hess = None
        self._mark_all()

    def _refresh_slacks(self):  # FunctionManager.py:427-449
        s = self.s + self.d - self.C @ self.x
        if self.ub is not None:
            s = np.append(s, self.s + self.ub - self.x)
        if self.lb is not None:
            s = np.append(s, self.s + self.x - self.lb)
        self.slacks = s.ravel() if s.ndim > 1 else s
        self.dirty_islacks = True

    def update_x(self, x, update_slacks=True):  # FunctionManager.py:451-470
        if len(x) == len(self.x) + 1:
            self.x = x[:-1]
            self.s = x[-1]
        elif len(x) == len(self.x):
            self.x = x
        else:
            raise ValueError("Provided x does not have the right dimensions!")
        if update_slacks:
            self._refresh_slacks()
        else:
            self.dirty_islacks = True
        self._mark_all()

    def _inv(self):
        if self.dirty_islacks:
            self.inv_slacks = 1 / (self.slacks + EPS_LOG)
            self.dirty_islacks = False
        return self.inv_slacks

    def objective(self, x=None):
        if x is not None:
            self.update_x(x)
        elif not self.dirty_obj:
            return self.obj
        self.obj = self.s
        self.dirty_obj = False
        return self.obj

    def newton_objective(self, x=None, t=None):  # FunctionManager.py:484-507
        if x is not None:
            self.update_x(x)
        if t is not None:
            self.update_t(t)
        if not self.dirty_nobj:
            return self.nobj
        self.nobj = self.t * self.objective() - np.log(self.slacks + EPS_LOG).sum()
        self.dirty_nobj = False
        return self.nobj

    def gradient(self, x=None, t=None):  # FunctionManager.py:509-545
        if x is not None:
            self.update_x(x)
        if t is not None:
            self.update_t(t)
        if not self.dirty_grad:
            return self.grad
        inv = self._inv()
        gx = self.C.T @ inv[self.seg_C]
        if self.lb is not None:
            gx -= inv[self.seg_lb]
        if self.ub is not None:
            gx += inv[self.seg_ub]
        self.grad = np.append(gx, self.t - inv.sum())
        self.dirty_grad = False
        return self.grad

    def hessian(self, x=None):  # FunctionManager.py:547-611
        if x is not None:
            self.update_x(x)
        if not self.dirty_hess:
            return self.hess
        inv2 = self._inv() ** 2
        hxx = self.C.T @ (inv2[self.seg_C][:, None] * self.C)
        hxs = -(self.C.T @ inv2[self.seg_C])
        dg = np.einsum("ii->i", hxx)
        if self.lb is not None:
            dg += inv2[self.seg_lb]
            hxs += inv2[self.seg_lb]
        if self.ub is not None:
            dg += inv2[self.seg_ub]
            hxs -= inv2[self.seg_ub]
        hss = inv2.sum()
        self.hess = np.block([[hxx, hxs.reshape(-1, 1)], [hxs.reshape(1, -1), np.array(hss).reshape(1, 1)]])
        self.dirty_hess = False
        return self.hess

    def inv_hessian(self, x=None):
        raise ValueError("Hessian is not diagonal, so inverse hessian cannot be directly computed!!")


class _LazyBlocks:
    """list-like per-cone blocks computed on access (memory-light form of the reference's caches)"""

    def __init__(self, fn, k):
        self.fn, self.k = fn, k

    def __len__(self):
        return self.k

    def __getitem__(self, i):
        return self.fn(i)


class SOCPBarrier(_BarrierBase):
    """FunctionManagerSOCP (FunctionManager.py:834-1162).

    Cone i: lhs_i = A_i x + b_i (A_i dense, or a vector a_i meaning diag(a_i)),
            rhs_i = c_i.x + d_i,  s_i = rhs_i^2 - ||lhs_i||^2.
    slacks = [s_1..s_K | ub - x | x - lb | rhs_1..rhs_K]; the trailing rhs block only
    enforces c_i.x + d_i >= 0 in the domain test (Q15); the barrier sums the rest.
    grad = t(Px+q) + sum_i 2(A_i^T lhs_i - c_i rhs_i)/(s_i+1e-12) - 1/(s_lb+1e-15) + 1/(s_ub+1e-15)
    hess = tP + sum_i [2(A_i^T A_i + c_i c_i^T)/(s_i+1e-12) + g_i g_i^T] + diag(1/(s_b+1e-12)^2)
           g_i = 2(A_i^T lhs_i - c_i rhs_i)/(s_i+1e-12)    (note +c_i c_i^T: Q5)
    """

    def __init__(self, P=None, q=None, A=None, b=None, c=None, d=None, lb=None, ub=None,
                 x0=None, t=1, n=None):
        self.P, self.q, self.A, self.b, self.c, self.d = P, q, A, b, c, d
        self.lb, self.ub = lb, ub
        self.x = x0
        self.t = t
        # the reference caches A_i^T A_i and c_i c_i^T per cone (2 K n^2 doubles: 64 GiB at the M5
        # size, FunctionManager.py:870-905); above 2 GiB they are recomputed per Hessian instead --
        # the same BLAS call on the same operands, so the blocks are bitwise the cached ones
        nx0 = len(x0) if x0 is not None else A[0].shape[-1]
        self.lazy = len(A) * nx0 * nx0 * 8 * 2 > (2 << 30)
        if self.lazy:
            self.AtA = _LazyBlocks(lambda i: np.matmul(A[i].T, A[i]) if A[i].ndim > 1 else np.diag(A[i] ** 2), len(A))
            self.cct = _LazyBlocks(lambda i: np.outer(c[i], c[i]), len(c)) if c is not None else None
        else:
            self.AtA = [np.matmul(Ai.T, Ai) if Ai.ndim > 1 else np.diag(Ai ** 2) for Ai in A]
            self.cct = [np.outer(ci, ci) for ci in c] if c is not None else None
        self.bounded = lb is not None or ub is not None
        self.constrained = True
        K = len(A)
        nx = len(x0)
        self.seg_cone = slice(0, K)
        off = K
        self.seg_ub = self.seg_lb = None
        if ub is not None:
            self.seg_ub = slice(off, off + nx); off += nx
        if lb is not None:
            self.seg_lb = slice(off, off + nx); off += nx
        self.seg_barrier = slice(0, off)
        self.slacks = self.lhs = self.rhs = None
        self.obj = self.nobj = self.grad = self.hess = None
        self._mark_all()

    def _cone_parts(self, xv):  # FunctionManager.py:933-975
        lhs = [(Ai @ xv) if Ai.ndim > 1 else Ai * xv for Ai in self.A]
        if self.b is not None:
            for i in range(len(lhs)):
                lhs[i] += self.b[i]
        if self.c is not None:
            rhs = [ci.dot(xv) for ci in self.c]
            if self.d is not None:
                for i in range(len(rhs)):
                    rhs[i] += self.d[i]
        elif self.d is not None:
            rhs = self.d
        else:
            rhs = 0
        return lhs, rhs

    def _refresh_slacks(self):  # FunctionManager.py:933-994
        lhs, rhs = self._cone_parts(self.x)
        self.lhs, self.rhs = lhs, rhs
        s = np.array([r ** 2 - (l ** 2).sum() for r, l in zip(rhs, lhs)])
        if self.ub is not None:
            s = np.append(s, self.ub - self.x)
        if self.lb is not None:
            s = np.append(s, self.x - self.lb)
        s = np.append(s, rhs)
        self.slacks = s.ravel() if s.ndim > 1 else s

    def update_x(self, x, update_slacks=True):  # FunctionManager.py:1020-1027
        self.x = x
        self._mark_all()
        if update_slacks:
            self._refresh_slacks()

    def objective(self, x=None):  # FunctionManager.py:996-1018
        if x is not None:
            self.update_x(x)
        elif not self.dirty_obj:
            return self.obj
        val = 0
        if self.P is not None:
            val += 1 / 2 * self.x.dot(self.P @ self.x)
        if self.q is not None:
            val += self.q.dot(self.x)
        self.obj = val
        self.dirty_obj = False
        return val

    def newton_objective(self, x=None, t=None):  # FunctionManager.py:1029-1053
        if x is not None:
            self.update_x(x)
        if t is not None:
            self.update_t(t)
        if not self.dirty_nobj:
            return self.nobj
        self.nobj = self.t * self.objective() - np.log(self.slacks[self.seg_barrier] + EPS_LOG).sum()
        self.dirty_nobj = False
        return self.nobj

    def _objgrad(self):
        g = 0
        if self.P is not None:
            g = self.P @ self.x
        if self.q is not None:
            g += self.q
        g *= self.t
        return g

    def gradient(self, x=None, t=None):  # FunctionManager.py:1055-1102
        if x is not None:
            self.update_x(x)
        if t is not None:
            self.update_t(t)
        if not self.dirty_grad:
            return self.grad
        g = self._objgrad()
        for i, (s, r, l) in enumerate(zip(self.slacks[self.seg_cone], self.rhs, self.lhs)):
            if self.c is not None:
                g -= 2 * self.c[i] * r / (s + EPS_CONE)
            Ai = self.A[i]
            if Ai.ndim > 1:
                g += 2 * (Ai.T @ l) / (s + EPS_CONE)
            else:
                g += 2 * Ai * l / (s + EPS_CONE)
        if self.lb is not None:
            g -= 1 / (self.slacks[self.seg_lb] + EPS_LOG)
        if self.ub is not None:
            g += 1 / (self.slacks[self.seg_ub] + EPS_LOG)
        self.grad = g
        self.dirty_grad = False
        return g

    def hessian(self, x=None, t=None):  # FunctionManager.py:1104-1158
        if x is not None:
            self.update_x(x)
        if t is not None:
            self.update_t(t)
        if not self.dirty_hess:
            return self.hess
        if self.lazy and all(Ai.ndim > 1 for Ai in self.A):
            H = self._hessian_stacked()
        else:
            H = self._hessian_blocks()
        if self.bounded:
            dg = np.einsum("ii->i", H)
            if self.lb is not None:
                dg += 1 / (self.slacks[self.seg_lb] + EPS_CONE) ** 2
            if self.ub is not None:
                dg += 1 / (self.slacks[self.seg_ub] + EPS_CONE) ** 2
        self.hess = H
        self.dirty_hess = False
        return H

    def _hessian_stacked(self):
        """The same sum as _hessian_blocks in ONE weighted Gram product (the device's layout,
        DESIGN.md §3): rows A_i (weight 2/(s_i+eps)), c_i (same weight), g_i (weight 1), so
        H = tP + X^T diag(w) X.  Used only above the 2 GiB cache size (the M5 fixture,
        tests/golden/make_golden_m5.py), where the per-cone form streams ~1 GB of n x n temporaries
        per cone and a Hessian takes minutes; it sums in another order than the reference's
        per-cone loop (rounding-level differences, covered by the fixture's perturbation envelope)."""
        rows, wts = [], []
        for i, (Ai, s) in enumerate(zip(self.A, self.slacks[self.seg_cone])):
            sc = 2 / (s + EPS_CONE)
            gt = Ai.T @ self.lhs[i]
            rows.append(Ai)
            wts.append(np.full(Ai.shape[0], sc))
            if self.c is not None:
                gt -= self.c[i] * self.rhs[i]
                rows.append(self.c[i][None, :])
                wts.append(np.array([sc]))
            gt *= sc
            rows.append(gt[None, :])
            wts.append(np.array([1.0]))
        X = np.concatenate(rows, axis=0)
        w = np.concatenate(wts)
        H = X.T @ (w[:, None] * X)
        if self.P is not None:
            H += self.t * self.P
        return H

    def _hessian_blocks(self):
        H = 0
        if self.P is not None:
            H += self.t * self.P
        for i, (Ai, s) in enumerate(zip(self.A, self.slacks[self.seg_cone])):
            gt = Ai * self.lhs[i] if Ai.ndim < 2 else Ai.T @ self.lhs[i]
            blk = 0
            blk += self.AtA[i]
            if self.c is not None:
                blk += self.cct[i]
                gt -= self.c[i] * self.rhs[i]
            blk *= 2 / (s + EPS_CONE)
            gt *= 2 / (s + EPS_CONE)
            blk += np.outer(gt, gt)
            H += blk
        return H

    def inv_hessian(self, x=None):
        raise ValueError("Hessian is not diagonal, cannot use inv hessian function!")


class SOCPPhase1Barrier(SOCPBarrier):
    """FunctionManagerSOCPPhase1 (FunctionManager.py:1165-1460): sigma = slacks + s on the
    barrier segments (cones, bounds); the appended rhs block is not shifted."""

    def __init__(self, A=None, b=None, c=None, d=None, x0=None, lb=None, ub=None, t=1, n=None):
        super().__init__(P=None, q=None, A=A, b=b, c=c, d=d, lb=lb, ub=ub, x0=x0, t=t, n=n)
        self.s = 0
        self._refresh_slacks()
        self.s = -self.slacks.min() + 1
        self._refresh_slacks()
        self.inv_slacks = None
        self.dirty_islacks = True

    def _refresh_slacks(self):  # FunctionManager.py:1258-1262
        super()._refresh_slacks()
        self.slacks[self.seg_barrier] += self.s
        self.dirty_islacks = True

    def update_x(self, x, update_slacks=True):  # FunctionManager.py:1264-1283
        if len(x) == len(self.x) + 1:
            self.x = x[:-1]
            self.s = x[-1]
        elif len(x) == len(self.x):
            self.x = x
        else:
            raise ValueError("Provided x does not have the right dimensions!")
        if update_slacks:
            self._refresh_slacks()
        # the reference's update_slacks=False branch sets a misspelled attribute
        # (FunctionManager.py:1278), so the inverse-slack cache is NOT invalidated.
        self._mark_all()

    def objective(self, x=None):
        if x is not None:
            self.update_x(x)
        elif not self.dirty_obj:
            return self.obj
        self.obj = self.s
        self.dirty_obj = False
        return self.obj

    def _inv(self):
        if self.dirty_islacks:
            self.inv_slacks = 1 / (self.slacks[self.seg_barrier] + EPS_LOG)
            self.dirty_islacks = False
        return self.inv_slacks

    def gradient(self, x=None, t=None):  # FunctionManager.py:1322-1370
        if x is not None:
            self.update_x(x)
        if t is not None:
            self.update_t(t)
        if not self.dirty_grad:
            return self.grad
        inv = self._inv()
        gx = 0
        for i, (iv, r, l) in enumerate(zip(inv[self.seg_cone], self.rhs, self.lhs)):
            if self.c is not None:
                gx -= 2 * self.c[i] * r * iv
            Ai = self.A[i]
            if Ai.ndim > 1:
                gx += 2 * (Ai.T @ l) * iv
            else:
                gx += 2 * Ai * l * iv
        if self.lb is not None:
            gx -= inv[self.seg_lb]
        if self.ub is not None:
            gx += inv[self.seg_ub]
        self.grad = np.append(gx, self.t - inv.sum())
        self.dirty_grad = False
        return self.grad

    def hessian(self, x=None):  # FunctionManager.py:1372-1453
        if x is not None:
            self.update_x(x)
        if not self.dirty_hess:
            return self.hess
        inv = self._inv()
        inv2 = inv ** 2
        hxx = 0
        hxs = 0
        for i, (Ai, iv) in enumerate(zip(self.A, inv[self.seg_cone])):
            gt = Ai * self.lhs[i] if Ai.ndim < 2 else Ai.T @ self.lhs[i]
            blk = 0
            blk += self.AtA[i]
            if self.c is not None:
                blk += self.cct[i]
                gt -= self.c[i] * self.rhs[i]
            blk *= 2 * iv
            gt *= 2 * iv
            hxs -= gt * iv
            blk += np.outer(gt, gt)
            hxx += blk
        if self.bounded:
            dg = np.einsum("ii->i", hxx)
            if self.lb is not None:
                dg += inv2[self.seg_lb]
                hxs += inv2[self.seg_lb]
            if self.ub is not None:
                dg += inv2[self.seg_ub]
                hxs -= inv2[self.seg_ub]
        hss = inv2.sum()
        self.hess = np.block([[hxx, hxs.reshape(-1, 1)], [hxs.reshape(1, -1), np.array(hss).reshape(1, 1)]])
        self.dirty_hess = False
        return self.hess


# --------------------------------------------------------------------------------------
# L2: Newton inner solvers (NewtonSolver.py, NewtonSolverInfeasibleStart.py)
# --------------------------------------------------------------------------------------

class FeasibleNewton:
    """NewtonSolver.solve / backtrack_search (NewtonSolver.py:80-206) with the
    linear-solve strategies of NewtonSolver.py:212-420.

    method: 'cholesky' (cho_factor/cho_solve; first LinAlgError -> lstsq forever, Q9),
            'diag' (H^-1 = 1/h), 'lstsq', 'solve', 'direct'.
    trace: list of dicts {step, nd} per Newton iteration (for trajectory parity).
    """

    def __init__(self, fm, method="cholesky", max_iters=50, eps=1e-5, alpha=0.2, beta=0.6,
                 phase1=False, phase1_tol=0.1, use_psd_condition=False, update_slacks_every=0):
        self.fm, self.method = fm, method
        self.max_iters, self.eps = max_iters, eps
        self.alpha, self.beta = alpha, beta
        self.phase1, self.phase1_tol = phase1, phase1_tol
        self.use_psd_condition = use_psd_condition
        self.update_slacks_every = update_slacks_every
        self.use_backup = False
        self.trace = []

    def direction(self, g):
        fm = self.fm
        if self.method == "diag":
            return -fm.inv_hessian() * g
        H = fm.hessian()
        if self.method == "lstsq":
            return np.linalg.lstsq(H, -g, rcond=None)[0]
        if self.method == "solve":
            return np.linalg.solve(H, -g)
        if self.method == "direct":
            return np.linalg.inv(H) @ -g
        # cholesky (NewtonSolver.py:277-341)
        if not self.use_backup:
            try:
                if self.use_psd_condition:
                    np.einsum("ii->i", H)[...] += 1e-9
                L = scipy.linalg.cho_factor(H, overwrite_a=True, check_finite=False)
                return scipy.linalg.cho_solve(L, -g, overwrite_b=True, check_finite=False)
            except np.linalg.LinAlgError:
                self.use_backup = True
        return np.linalg.lstsq(H, -g, rcond=None)[0]

    def backtrack(self, x, dx, g):  # NewtonSolver.py:157-206
        fm, beta = self.fm, self.beta
        step = 1
        fx = fm.newton_objective()
        nxt = x + step * dx
        gc = g.dot(x)                     # Q1: g.x, not g.dx
        fm.update_x(nxt)
        while (fm.slacks < 0).any():
            step *= beta
            if step < STEP_FLOOR:
                return step
            nxt = x + step * dx
            fm.update_x(nxt)
        attempt = 0
        K = self.update_slacks_every
        while fm.newton_objective() > fx + self.alpha * step * gc:
            attempt += 1
            nxt = x + step * dx           # Q3: the point for the PRE-update step
            if step < STEP_FLOOR:
                return step
            step *= beta
            fm.update_x(nxt, update_slacks=(K > 0 and attempt % K == K - 1))  # Q2
        fm.update_x(nxt)
        return step

    def solve(self, x, t, v0=None):  # NewtonSolver.py:80-155
        fm = self.fm
        nd = None
        it = 0
        try:
            for it in range(self.max_iters):
                g = fm.gradient(x)
                dx = self.direction(g)
                step = self.backtrack(x, dx, g)
                x += step * dx                 # Q8: in place
                fm.update_x(x)
                if self.phase1 and x[-1] < -self.phase1_tol:
                    self.trace.append({"step": step, "nd": None})
                    return x, None, it + 1, None, True
                nd = -g.dot(dx) / 2            # Q6
                self.trace.append({"step": step, "nd": nd})
                if step < STEP_FLOOR:
                    return x, None, it + 1, nd, False
                elif nd < self.eps:
                    return x, None, it + 1, nd, True
            return x, None, it + 1, nd, False
        except np.linalg.LinAlgError:
            return x, None, it + 1, nd, False


class InfeasibleNewton:
    """NewtonSolverInfeasibleStart (NewtonSolverInfeasibleStart.py:72-273) with the
    block-elimination linear solves of :279-956.

    method: 'cholesky' (dense H; fallback = np.linalg.solve x4, Q9), 'cholesky_diag'
            (H diagonal; S = A diag(1/h) A^T), 'lstsq', 'solve', 'direct', 'lstsq_diag',
            'solve_diag', 'direct_diag', 'kkt', 'kkt_diag'.
    """

    def __init__(self, A, b, fm, method="cholesky", max_iters=50, eps=1e-5, alpha=0.2, beta=0.6,
                 use_psd_condition=False, update_slacks_every=0):
        self.A, self.b, self.fm, self.method = A, b, fm, method
        self.max_iters, self.eps = max_iters, eps
        self.alpha, self.beta = alpha, beta
        self.use_psd_condition = use_psd_condition
        self.update_slacks_every = update_slacks_every
        self.use_backup = False
        self.trace = []

    def _lu_blocks(self, H, x, g, b2=None):  # NewtonSolverInfeasibleStart.py:513-538
        A = self.A
        if H.ndim < 2:
            H = np.diag(H)
        if b2 is None:
            b2 = A @ x - self.b
        HiAT = np.linalg.solve(H, A.T)
        Hig = np.linalg.solve(H, g)
        w = np.linalg.solve(A @ HiAT, b2 - A @ Hig)
        dx = -np.linalg.solve(H, g + A.T @ w)
        return dx, w

    def direction(self, x, v, g):
        A, fm, m = self.A, self.fm, self.method
        if m.endswith("_diag"):
            b2 = A @ x - self.b
            Hi = fm.inv_hessian()
            S = A @ (Hi[:, None] * A.T)
            r = b2 - A @ (Hi * g)
            if m == "cholesky_diag":
                w = scipy.linalg.cho_solve(scipy.linalg.cho_factor(S, overwrite_a=False, check_finite=False),
                                           r, overwrite_b=False, check_finite=False)
            elif m == "lstsq_diag":
                w = np.linalg.lstsq(S, r, rcond=None)[0]
            elif m == "solve_diag":
                w = np.linalg.solve(S, r)
            elif m == "direct_diag":
                w = np.linalg.inv(S) @ r
            else:
                raise ValueError(m)
            dx = -Hi * (g + A.T @ w)
            return dx, w - v
        if m in ("kkt", "kkt_diag"):
            rd = g + A.T @ v
            rp = A @ x - self.b
            p = A.shape[0]
            H = fm.hessian()
            M = np.block([[np.diag(H), A.T], [A, np.zeros((p, p))]])
            dd = np.linalg.solve(M, -np.append(rd, rp))
            return dd[: A.shape[1]], dd[A.shape[1]:]
        H = fm.hessian()
        if H.ndim < 2:
            H = np.diag(H)
        if m == "lstsq":
            b2 = A @ x - self.b
            HiAT = np.linalg.lstsq(H, A.T, rcond=None)[0]
            Hig = np.linalg.lstsq(H, g, rcond=None)[0]
            w = np.linalg.lstsq(A @ HiAT, b2 - A @ Hig, rcond=None)[0]
            dx = -np.linalg.lstsq(H, g + A.T @ w, rcond=None)[0]
            return dx, w - v
        if m == "solve":
            dx, w = self._lu_blocks(H, x, g)
            return dx, w - v
        if m == "direct":
            b2 = A @ x - self.b
            Hi = np.linalg.inv(H)
            Ki = np.linalg.inv(A @ (Hi @ A.T))
            w = Ki @ (b2 - A @ (Hi @ g))
            return -Hi @ (g + A.T @ w), w - v
        # cholesky (NewtonSolverInfeasibleStart.py:386-511)
        b2 = None
        if not self.use_backup:
            try:
                if self.use_psd_condition:
                    np.einsum("ii->i", H)[...] += 1e-9
                b2 = A @ x - self.b
                L1 = scipy.linalg.cho_factor(H, overwrite_a=False, check_finite=False)
                HiAT = scipy.linalg.cho_solve(L1, A.T, overwrite_b=False, check_finite=False)
                Hig = scipy.linalg.cho_solve(L1, g, overwrite_b=False, check_finite=False)
                L2 = scipy.linalg.cho_factor(A @ HiAT, overwrite_a=False, check_finite=False)
                w = scipy.linalg.cho_solve(L2, b2 - A @ Hig, overwrite_b=False, check_finite=False)
                dx = -scipy.linalg.cho_solve(L1, g + A.T @ w, overwrite_b=False, check_finite=False)
                return dx, w - v
            except np.linalg.LinAlgError:
                self.use_backup = True
        dx, w = self._lu_blocks(H, x, g, b2=b2)
        return dx, w - v

    def backtrack(self, x, v, dx, dv, g):  # NewtonSolverInfeasibleStart.py:170-273
        fm, A, beta = self.fm, self.A, self.beta
        step = 1
        nxt = x + step * dx
        fm.update_x(nxt)
        while (fm.slacks < 0).any():
            step *= beta
            if step < STEP_FLOOR:
                return step, None, None
            nxt = x + step * dx
            fm.update_x(nxt)
        ATv = A.T @ v
        ATdv = A.T @ dv
        Axb = A @ x - self.b
        Adx = A @ dx
        r = np.linalg.norm(np.append(g + ATv, Axb))
        gn = fm.gradient()
        rn = np.linalg.norm(np.append(gn + ATv + step * ATdv, Axb + step * Adx))
        attempt = 0
        K = self.update_slacks_every
        while rn > (1 - self.alpha * step) * r:
            attempt += 1
            step *= beta                      # no lag here (unlike the feasible solver)
            if step < STEP_FLOOR:
                break
            nxt = x + step * dx
            fm.update_x(nxt, update_slacks=(K > 0 and attempt % K == K - 1))
            gn = fm.gradient()                # stale-slack barrier gradient (Q2)
            rn = np.linalg.norm(np.append(gn + ATv + step * ATdv, Axb + step * Adx))
        fm.update_x(nxt)
        return step, gn, rn

    def solve(self, x, t, v0=None):  # NewtonSolverInfeasibleStart.py:72-168
        fm = self.fm
        v = np.zeros(self.A.shape[0]) if v0 is None else v0
        rn = None
        it = 0
        try:
            for it in range(self.max_iters):
                g = fm.gradient(x)
                dx, dv = self.direction(x, v, g)
                step, g, rn = self.backtrack(x, v, dx, dv, g)
                x += step * dx
                v += step * dv
                fm.update_x(x)
                self.trace.append({"step": step, "res": rn})
                if step < STEP_FLOOR:
                    return x, v, it + 1, rn, False
                elif rn < self.eps:             # Q7: trial residual from backtracking
                    return x, v, it + 1, rn, True
            return x, v, it + 1, rn, False
        except np.linalg.LinAlgError:
            return x, v, it + 1, rn, False


# --------------------------------------------------------------------------------------
# L3: phase one (PhaseOneSolver.py)
# --------------------------------------------------------------------------------------

class PhaseOne:
    """PhaseOneSolver (PhaseOneSolver.py:6-154): min s s.t. slacks + s > 0."""

    def __init__(self, C=None, d=None, lb=None, ub=None, x0=None, max_outer_iters=50,
                 max_inner_iters=20, epsilon=1e-8, inner_epsilon=1e-5, alpha=0.2, beta=0.6,
                 mu=15, t0=1, n=None, tol=0.1, socp=False, socp_params=None,
                 use_psd_condition=False, update_slacks_every=0):
        self.n, self.mu, self.t0, self.tol = n, mu, t0, tol
        self.epsilon = epsilon
        self.max_outer_iters, self.max_inner_iters = max_outer_iters, max_inner_iters
        if socp:
            A, b, c, d2 = socp_params
            self.fm = SOCPPhase1Barrier(A=A, b=b, c=c, d=d2, x0=x0, lb=lb, ub=ub, t=t0, n=n)
        else:
            self.fm = Phase1Barrier(C=C, d=d, x0=x0, lb=lb, ub=ub, t=t0, n=n)
        self.x = np.append(x0, self.fm.s)
        self.ns = FeasibleNewton(self.fm, "cholesky", max_inner_iters, inner_epsilon, alpha, beta,
                                 phase1=True, phase1_tol=tol, use_psd_condition=use_psd_condition,
                                 update_slacks_every=update_slacks_every)

    def solve(self, x0=None):  # PhaseOneSolver.py:112-154
        if x0 is not None:
            self.fm.update_x(x0)
        t = self.t0
        self.outer_iters = 0
        self.inner_iters = []
        obj = None
        for _ in range(self.max_outer_iters):
            self.x, _, k, _, ok = self.ns.solve(self.x, t)
            self.outer_iters += 1
            self.inner_iters.append(k)
            obj = self.fm.objective(self.x)
            if obj < -self.tol:
                break
            t = min(t * self.mu, (self.n + 1.0) / self.epsilon)
            self.fm.update_t(t)
        return self.x[:-1], obj


# --------------------------------------------------------------------------------------
# L4: problem facades (LPSolver.py, QPSolver.py, SOCPSolver.py)
# --------------------------------------------------------------------------------------

def default_x0(n, lb, ub):
    """LPSolver.py:128-143 (same in QP/SOCP): midpoint / lb+0.1 / ub-0.1 / np.random.rand."""
    if lb is not None and ub is not None:
        return (np.maximum(lb, -1e2) + np.minimum(ub, 1e2)) / 2 * np.ones(n)
    if lb is not None:
        return (np.maximum(lb, -1e2) + 1e-1) * np.ones(n)
    if ub is not None:
        return (np.minimum(ub, 1e2) - 1e-1) * np.ones(n)
    return np.random.rand(n)


def _bounds(lb, ub):
    lb = None if lb is None else np.array(lb)
    ub = None if ub is None else np.array(ub)
    return lb, ub


class _BarrierProblem:
    """Outer barrier loop shared by LP/QP/SOCP (LPSolver.py:514-653, QPSolver.py:500-638,
    SOCPSolver.py:616-753): t <- t0; centre; record objective if ||Ax-b|| small (LP: 1e-4 n,
    QP/SOCP: 1e-3); break on non-improvement after a successful centring; stop when
    num_constraints / t < epsilon; t <- mu t."""

    eq_tol_scale = None

    def _eq_ok(self, x):
        if self.A is None:
            return True
        return np.linalg.norm(self.A @ x - self.b) < self._eq_tol()

    def solve(self, resolve=True, **kw):
        if not resolve and self.optimal:
            return self.value
        t = kw.get("t0", self.t0)
        max_outer = kw.get("max_outer_iters", self.max_outer_iters)
        self.track_loss = kw.get("track_loss", self.track_loss)
        if "x0" in kw:
            x = kw["x0"]
            use_x0 = True
        else:
            x = self.x
            use_x0 = False
        self.phase1_iters = []
        if self.has_ineq and self.phase1.fm.s >= 1:            # Q11
            x, s = self.phase1.solve(x0=x) if use_x0 else self.phase1.solve()
            self.phase1_iters = list(self.phase1.inner_iters)
            if s > -self.phase1_tol:
                raise ValueError("Phase 1 Solver did not successfully find a feasible point!")
        self.outer_iters = 0
        self.inner_iters = []
        vals = []
        self.fm.update_x(x)
        self.fm.update_t(t)
        v = np.zeros(self.A.shape[0]) if self.A is not None else None
        gap = self.num_constraints
        best_x = x.copy()
        best = np.inf
        for _ in range(max_outer):
            x, v, k, _, ok = self.ns.solve(x, t, v0=v)
            self.outer_iters += 1
            self.inner_iters.append(k)
            if self._eq_ok(x):
                val = self.fm.objective()
                if self.track_loss:
                    vals.append(val)
                if val < best:
                    best = val
                    best_x = x.copy()
                elif ok:
                    break
            elif vals:
                vals.append(vals[-1])
            gap = self.num_constraints / t
            if gap < self.epsilon:
                break
            t = t * self.mu
            self.fm.update_t(t)
        self.xstar = best_x
        if self.get_dual_variables:
            if self.has_ineq or self.bounded:
                self.fm.update_x(best_x)
                self.lam_star = 1 / (t * self.fm.slacks)
            if self.A is not None:
                self.v_star = v / t
        self.optimal = True
        self.value = best
        self.optimality_gap = gap
        self.objective_vals = vals
        return best


class LPSolver(_BarrierProblem):
    """LPSolver (LPSolver.py:18-705), check_cvxpy ignored (cvxpy absent)."""

    def __init__(self, c=None, A=None, b=None, C=None, d=None, lower_bound=0, upper_bound=None,
                 t0=0.1, max_outer_iters=20, max_inner_iters=50, phase1_max_inner_iters=500,
                 epsilon=1e-10, inner_epsilon=1e-5, check_cvxpy=False, linear_solve_method="cholesky",
                 max_cg_iters=50, alpha=0.2, beta=0.6, mu=15, suppress_print=True, use_gpu=False,
                 try_diag=True, track_loss=False, get_dual_variables=False, phase1_tol=0,
                 phase1_t0=0.01, x0=None, update_slacks_every=0):
        self.c, self.A, self.b, self.C, self.d = c, A, b, C, d
        self.lb, self.ub = _bounds(lower_bound, upper_bound)
        self.n = len(c) if c is not None else (A.shape[1] if A is not None else C.shape[1])
        self.x = x0 if x0 is not None else default_x0(self.n, self.lb, self.ub)
        self.bounded = self.lb is not None or self.ub is not None
        self.has_ineq = C is not None
        self.num_constraints = (len(d) if d is not None else 0) + self.n * (self.lb is not None) + self.n * (self.ub is not None)
        self.t0, self.mu, self.epsilon = t0, mu, epsilon
        self.max_outer_iters = max_outer_iters
        self.track_loss, self.get_dual_variables = track_loss, get_dual_variables
        self.phase1_tol = phase1_tol
        self.optimal = False
        self.value = None
        if C is not None:
            self.phase1 = PhaseOne(C=C, d=d, lb=self.lb, ub=self.ub, x0=self.x, max_outer_iters=max_outer_iters,
                                   max_inner_iters=phase1_max_inner_iters, epsilon=epsilon,
                                   inner_epsilon=inner_epsilon, alpha=alpha, beta=beta, mu=mu,
                                   t0=phase1_t0, n=self.n, tol=phase1_tol,
                                   update_slacks_every=update_slacks_every)
        self.fm = LPBarrier(c=c, C=C, d=d, x0=self.x, lb=self.lb, ub=self.ub, t=1, try_diag=try_diag, n=self.n)
        diag = not (C is not None or not try_diag)
        common = dict(max_iters=max_inner_iters, eps=inner_epsilon, alpha=alpha, beta=beta,
                      update_slacks_every=update_slacks_every)
        if A is not None:
            meth = {"cholesky": "cholesky", "np_solve": "solve", "np_lstsq": "lstsq", "direct": "direct",
                    "kkt": "kkt"}[linear_solve_method]
            if diag:
                meth = meth + "_diag"
            self.ns = InfeasibleNewton(A, b, self.fm, meth, **common)
        else:
            if linear_solve_method == "kkt" and not diag:   # LPSolver.py:423-430
                raise ValueError("No KKT System non-equality-constrained problems! Please choose another solver")
            meth = "diag" if diag else {"cholesky": "cholesky", "np_solve": "solve", "np_lstsq": "lstsq",
                                        "direct": "direct"}[linear_solve_method]
            self.ns = FeasibleNewton(self.fm, meth, **common)

    def _eq_tol(self):
        return 1e-4 * self.n


class QPSolver(_BarrierProblem):
    """QPSolver (QPSolver.py:18-689)."""

    def __init__(self, P=None, q=None, A=None, b=None, C=None, d=None, lower_bound=0, upper_bound=None,
                 t0=0.1, max_outer_iters=20, max_inner_iters=50, phase1_max_inner_iters=500,
                 epsilon=1e-10, inner_epsilon=1e-5, check_cvxpy=False, linear_solve_method="cholesky",
                 max_cg_iters=50, alpha=0.2, beta=0.6, mu=15, suppress_print=True, use_gpu=False,
                 track_loss=False, get_dual_variables=False, phase1_tol=0, phase1_t0=0.01, x0=None,
                 update_slacks_every=0):
        if P is None:
            raise ValueError("Setting P to None is just an LP! Please use LP solver or set a value to P.")
        self.P, self.q, self.A, self.b, self.C, self.d = P, q, A, b, C, d
        self.lb, self.ub = _bounds(lower_bound, upper_bound)
        if q is not None:
            self.n = len(q)
        elif A is not None:
            self.n = A.shape[1]
        elif C is not None:
            self.n = C.shape[1]
        else:
            self.n = P.shape[1]
        self.x = x0 if x0 is not None else default_x0(self.n, self.lb, self.ub)
        self.bounded = self.lb is not None or self.ub is not None
        self.has_ineq = C is not None
        self.num_constraints = (len(d) if d is not None else 0) + self.n * (self.lb is not None) + self.n * (self.ub is not None)
        self.t0, self.mu, self.epsilon = t0, mu, epsilon
        self.max_outer_iters = max_outer_iters
        self.track_loss, self.get_dual_variables = track_loss, get_dual_variables
        self.phase1_tol = phase1_tol
        self.optimal = False
        self.value = None
        if C is not None:
            self.phase1 = PhaseOne(C=C, d=d, lb=self.lb, ub=self.ub, x0=self.x, max_outer_iters=max_outer_iters,
                                   max_inner_iters=phase1_max_inner_iters, epsilon=epsilon,
                                   inner_epsilon=inner_epsilon, alpha=alpha, beta=beta, mu=mu,
                                   t0=phase1_t0, n=self.n, tol=phase1_tol,
                                   update_slacks_every=update_slacks_every)
        self.fm = QPBarrier(P=P, q=q, C=C, d=d, x0=self.x, lb=self.lb, ub=self.ub, t=1, n=self.n)
        common = dict(max_iters=max_inner_iters, eps=inner_epsilon, alpha=alpha, beta=beta,
                      update_slacks_every=update_slacks_every)
        meth = {"cholesky": "cholesky", "np_solve": "solve", "np_lstsq": "lstsq", "direct": "direct",
                "kkt": "kkt"}[linear_solve_method]
        if A is not None:
            self.ns = InfeasibleNewton(A, b, self.fm, meth, **common)
        else:
            if meth == "kkt":   # QPSolver.py:417-424
                raise ValueError("No KKT System non-equality-constrained problems! Please choose another solver")
            self.ns = FeasibleNewton(self.fm, meth, **common)

    def _eq_tol(self):
        return 1e-3


def normalize_socp(A, b, c, d):
    """SOCPSolver.py:274-382 (Q16): lists, diagonal compression of 2-D A_i, broadcast of b/d."""
    if A is None:
        return A, b, c, d
    A = list(A) if isinstance(A, list) else [A]
    for i, Ai in enumerate(A):
        if Ai.ndim == 2:
            dg = np.diag(Ai).copy()
            off = Ai.copy()
            np.fill_diagonal(off, 0)
            if (off == 0).all():
                A[i] = dg
    if b is not None:
        b = list(b) if isinstance(b, list) else [b]
        if len(b) == 1:
            b = b * len(A)
    if c is not None:
        c = list(c) if isinstance(c, list) else [c]
    if d is not None:
        d = list(d) if isinstance(d, list) else [d]
        if len(d) == 1:
            d = d * len(A)
    return A, b, c, d


class SOCPSolver(_BarrierProblem):
    """SOCPSolver (SOCPSolver.py:18-833). F x = g are the equality constraints."""

    def __init__(self, P=None, q=None, A=None, b=None, c=None, d=None, F=None, g=None, lower_bound=0,
                 upper_bound=None, t0=0.1, phase1_t0=0.01, max_outer_iters=20, max_inner_iters=50,
                 phase1_max_inner_iters=500, epsilon=1e-10, inner_epsilon=1e-5, check_cvxpy=False,
                 linear_solve_method="cholesky", max_cg_iters=50, alpha=0.2, beta=0.6, mu=15,
                 suppress_print=True, use_gpu=False, try_diag=True, track_loss=False,
                 get_dual_variables=False, phase1_tol=0, use_psd_condition=False, x0=None,
                 update_slacks_every=0):
        A, b, c, d = normalize_socp(A, b, c, d)
        if A is None:
            raise ValueError("No cone contraints detected. Run with LPSolver or QPSolver for better performance.")
        self.P, self.q, self.cones, self.cb, self.cc, self.cd = P, q, A, b, c, d
        self.A, self.b = F, g                   # equality constraints drive the infeasible start
        self.lb, self.ub = _bounds(lower_bound, upper_bound)
        if q is not None:
            self.n = len(q)
        elif P is not None:
            self.n = P.shape[1]
        elif F is not None:
            self.n = F.shape[1]
        else:
            self.n = A[0].shape[-1]
        self.x = x0 if x0 is not None else default_x0(self.n, self.lb, self.ub)
        self.bounded = self.lb is not None or self.ub is not None
        self.has_ineq = True
        self.num_constraints = len(A) + self.n * (self.lb is not None) + self.n * (self.ub is not None)
        self.t0, self.mu, self.epsilon = t0, mu, epsilon
        self.max_outer_iters = max_outer_iters
        self.track_loss, self.get_dual_variables = track_loss, get_dual_variables
        self.phase1_tol = phase1_tol
        self.optimal = False
        self.value = None
        self.phase1 = PhaseOne(lb=self.lb, ub=self.ub, x0=self.x, max_outer_iters=max_outer_iters,
                               max_inner_iters=phase1_max_inner_iters, epsilon=epsilon,
                               inner_epsilon=inner_epsilon, alpha=alpha, beta=beta, mu=mu, t0=phase1_t0,
                               n=self.n, tol=phase1_tol, socp=True, socp_params=(A, b, c, d),
                               use_psd_condition=use_psd_condition, update_slacks_every=update_slacks_every)
        self.fm = SOCPBarrier(P=P, q=q, A=A, b=b, c=c, d=d, lb=self.lb, ub=self.ub, x0=self.x, t=1, n=self.n)
        common = dict(max_iters=max_inner_iters, eps=inner_epsilon, alpha=alpha, beta=beta,
                      use_psd_condition=use_psd_condition, update_slacks_every=update_slacks_every)
        meth = {"cholesky": "cholesky", "np_solve": "solve", "np_lstsq": "lstsq", "direct": "direct",
                "kkt": "kkt"}[linear_solve_method]
        if F is not None:
            self.ns = InfeasibleNewton(F, g, self.fm, meth, **common)
        else:
            if meth == "kkt":   # SOCPSolver.py dispatch, as QPSolver.py:417-424
                raise ValueError("No KKT System non-equality-constrained problems! Please choose another solver")
            self.ns = FeasibleNewton(self.fm, meth, **common)

    def _eq_tol(self):
        return 1e-3
