"""Batch group: independent instances on ONE GPU factor their Newton matrices in one grid.

SURVEY.md §8(e) config 4 (8 x n=2048 QPs per GPU).  Each instance is solved by its own host thread
on its own HIP stream (the solver facades are unchanged); the members of a group meet at every
Newton-step Cholesky inside libipm355.so and one of them launches the factorisations of all that
arrived as ONE grid of the fused Cholesky kernel (instances interleaved over the workgroups, so the
panel-chain roles of every instance are dispatched first).  A member that is elsewhere -- phase
change, LU fallback, finished -- is not waited for longer than `timeout_us`.

    group = BatchGroup()
    for s in solvers:
        group.attach(s)
    def run(s):                         # one host thread per solver, each under its own stream
        with group.member():
            s.solve()
"""
from __future__ import annotations

import contextlib
import ctypes as C

from . import _lib as L


def _problems(solver):
    out = []
    fm = getattr(solver, "fm", None)
    if fm is not None and getattr(fm, "prob", None) is not None:
        out.append(fm.prob)
    p1 = getattr(solver, "phase1_solver", None)
    if p1 is not None and getattr(p1.phase1_fm, "prob", None) is not None:
        out.append(p1.phase1_fm.prob)
    return out


class BatchGroup:
    def __init__(self, timeout_us: float = 300.0):
        self.lib = L.load_library()
        p = L.P()
        rc = self.lib.ipm_batch_create(float(timeout_us), C.byref(p))
        if rc != L.IPM_OK:
            raise L.IPMBackendError(f"ipm_batch_create failed ({rc})")
        self.ptr = p

    def attach(self, solver):
        for prob in _problems(solver):
            prob.check(self.lib.ipm_problem_set_batch(prob.ptr, self.ptr))

    @staticmethod
    def detach(solver):
        for prob in _problems(solver):
            prob.check(prob.handle.lib.ipm_problem_set_batch(prob.ptr, L.P(0)))

    @contextlib.contextmanager
    def member(self):
        self.lib.ipm_batch_join(self.ptr)
        try:
            yield self
        finally:
            self.lib.ipm_batch_leave(self.ptr)

    def stats(self):
        """(leader launches, member factorisations) so far: their ratio is the mean batch size."""
        a, b = L.I64(), L.I64()
        self.lib.ipm_batch_stats(self.ptr, C.byref(a), C.byref(b))
        return a.value, b.value

    def close(self):
        if self.ptr:
            self.lib.ipm_batch_destroy(self.ptr)
            self.ptr = None
