"""CPU oracle for the batched-ADMM Lasso solver -- TEST INFRASTRUCTURE ONLY.

NumPy/SciPy restatement of the reference's ``LassoSolver`` (fdeguire03/InteriorPoint-GPU,
LassoSolver.py) used by ``tests/`` to check the HIP path (``ipm355.lasso``); the product path never
imports it.

Parity status: PINNED.  ``tests/golden/make_golden_lasso.py`` runs the reference LassoSolver in
the build container (cvxpy stubbed, ``check_cvxpy=False``) and stores inputs and outputs under
``tests/golden/lasso_*.npz``; ``tests/test_oracle_golden.py`` checks this module against them.

Semantics restated (file:line in the reference):
* problem  min_x 1/(2m) ||A x - b||^2 + reg ||x||_1 for every column of b / entry of reg at once
  (LassoSolver.py:38-42); ``num_samples = max(b.shape[1], len(reg))`` (:110-112);
* ``normalize_A`` divides the caller's A in place by its column std (:122-123), BEFORE the bias
  column is prepended (:124-131); ``AtA_cache`` exists only with ``add_bias=True`` -- without it the
  constructor raises AttributeError at the Cholesky (:178-183), a reference bug kept as is;
* Q = (diag(m rho) + A^T A)^-1 by Cholesky + cho_solve against I (:178-189);
* one chunk (:193-221): bA = Q (A^T b); Q *= -m rho; several chunks (:339-485): the same per chunk
  of columns i::num_chunks, with Q * -m * rho evaluated left to right (two roundings) and the dual
  update written u + (x - alpha);
* ADMM step (:240-252): x = bA + Q (u - alpha); alpha = prox(x + u, reg / rho); u = u + x - alpha;
  prox (:533-558): max(v - eta, 0) - max(-v - eta, 0) (no second term when ``positive``), row 0 left
  unpenalised with ``add_bias``;
* stopping check every ``check_stop`` iterations (:270-289): ||x - alpha||_F < eps_abs sqrt(n S) +
  eps_rel ||alpha||_F and ||rho (alpha - alpha_prev)||_F < eps_abs sqrt(n S) + eps_rel rho ||u||_F;
* loss (:254-268, 305-318): 1/(2m) ||A alpha - b||^2 per column + reg ||alpha[bias:]||_1 (|.| only
  when not ``positive``);
* returns (X, solutions, gaps[:iters], iters) for one chunk (:330-337), (X, solutions, gaps,
  [iteration of each chunk]) -- the LAST index, not a count -- for several (:474-485).
"""
from __future__ import annotations

import numpy as np
import scipy.linalg


class LassoSolver:
    def __init__(self, A, b, reg=1, rho=0.4, max_iters=1000, check_stop=10, add_bias=False, normalize_A=False,
                 positive=False, compute_loss=False, adaptive_rho=False, eps_abs=1e-4, eps_rel=3e-2, use_gpu=False,
                 num_chunks=0, check_cvxpy=False):
        self.num_chunks = max(1, num_chunks)                       # LassoSolver.py:89-90 (CPU path)
        self.b = b if b.ndim >= 2 else b[:, None]
        self.reg, self.rho, self.max_iters, self.check_stop = reg, rho, max_iters, check_stop
        self.compute_loss, self.positive, self.add_bias = compute_loss, positive, add_bias
        self.eps_abs, self.eps_rel = eps_abs, eps_rel
        assert len(reg) == self.b.shape[1] or len(reg) == 1 or self.b.shape[1] == 1
        self.num_samples = max(self.b.shape[1], len(reg))
        self.gaps = np.zeros((max_iters, self.num_samples))
        self.A = A
        self.m = A.shape[0]
        if normalize_A:
            self.A /= self.A.std(axis=0)                            # in place on the caller's array
        if add_bias:
            self.A = np.hstack((np.ones((self.m, 1)), self.A))
            self.AtA_cache = self.A.T @ self.A
        self.n = self.A.shape[1]
        Mreg = np.diag(np.ones(self.n) * self.m * rho) + self.AtA_cache   # AttributeError w/o add_bias
        fac = scipy.linalg.cho_factor(Mreg, overwrite_a=False, check_finite=False)
        self.Qinv_cache = scipy.linalg.cho_solve(fac, np.eye(self.n), overwrite_b=False, check_finite=False)
        self.X = np.zeros((self.n, self.b.shape[1]))
        if self.num_chunks == 1:
            self.b = np.array(self.b)
            self.reg = np.array(reg)
            self.stop_multiplier = eps_abs * np.sqrt(self.n * self.num_samples)
            self.eta = self.reg / rho
            self.bA_cache = self.Qinv_cache @ (self.A.T @ self.b)
            self.Qinv_cache *= -self.m * rho

    def prox(self, v, eta):
        out = np.maximum(v - eta, 0)
        if not self.positive:
            out -= np.maximum(-v - eta, 0)
        if self.add_bias:
            out[0] = v[0]
        return out

    def _loss(self, alpha, b, reg):
        f = 1 / (2 * self.m) * ((self.A @ alpha - b) ** 2).sum(axis=0)
        xa = alpha if self.positive else np.abs(alpha)
        f += reg * (xa[1:] if self.add_bias else xa).sum(axis=0)
        return f

    def solve(self):
        if self.num_chunks == 1:
            return self._one()
        return self._chunks()

    def _stop(self, x, alpha, last, u, mult):
        rn = np.linalg.norm(x - alpha)
        dn = np.linalg.norm(self.rho * (alpha - last))
        return rn < mult + self.eps_rel * np.linalg.norm(alpha) and dn < mult + self.eps_rel * self.rho * np.linalg.norm(u)

    def _one(self):
        S = self.num_samples
        x = np.zeros((self.n, S))
        alpha = np.zeros((self.n, S))
        u = np.zeros((self.n, S))
        for it in range(self.max_iters):
            x = self.bA_cache + self.Qinv_cache @ (u - alpha)
            last = alpha
            alpha = self.prox(x + u, self.eta)
            u = u + x - alpha
            if self.compute_loss:
                self.gaps[it] = self._loss(alpha, self.b, self.reg)
            if it % self.check_stop == self.check_stop - 1 and self._stop(x, alpha, last, u, self.stop_multiplier):
                break
        self.x, self.alpha, self.u = x, alpha, u
        self.solutions = self._loss(alpha, self.b, self.reg)
        self.X = alpha
        self.num_iterations = [it + 1]
        return self.X, self.solutions, self.gaps[: it + 1], it + 1

    def _chunks(self):
        self.num_iterations = []
        self.solutions = np.empty(self.num_samples)
        reg_arr = isinstance(self.reg, np.ndarray)
        idx = np.array(range(self.b.shape[1]))
        for c in range(self.num_chunks):
            cols = idx[c::self.num_chunks]
            bc = np.array(self.b[..., cols])
            S = bc.shape[1]
            regc = np.array(self.reg[cols]) if reg_arr else np.array(self.reg)
            mult = self.eps_abs * np.sqrt(self.n * S)
            x = np.zeros((self.n, S))
            alpha = np.zeros((self.n, S))
            u = np.zeros((self.n, S))
            eta = regc / self.rho
            bA = self.Qinv_cache @ (self.A.T @ bc)
            Q = self.Qinv_cache * -self.m * self.rho
            for it in range(self.max_iters):
                x = bA + Q @ (u - alpha)
                last = alpha
                alpha = self.prox(x + u, eta)
                u = u + (x - alpha)
                if self.compute_loss:
                    self.gaps[it, cols] = self._loss(alpha, bc, regc)
                if it % self.check_stop == self.check_stop - 1 and self._stop(x, alpha, last, u, mult):
                    break
            self.solutions[cols] = self._loss(alpha, bc, regc)
            self.X[:, cols] = alpha
            self.num_iterations.append(it)
        return self.X, self.solutions, self.gaps, self.num_iterations
