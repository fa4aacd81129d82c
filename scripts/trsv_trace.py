"""Backward-solve chain timeline (trace builds, -DIPM_ROLE_TRACE): per ticket, when its pre sum was
done, when x_{B+1} had been polled, when x_B was stored (s_memrealtime, 100 MHz).
    IPM355_LIB=build/r6ab/trace.so python scripts/trsv_trace.py [n ...]"""
import ctypes, sys, os
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "interiorpoint-gpu_amd"),
                os.path.join(os.path.dirname(__file__), "..", "tests")]
from gpu_util import dev, handle, potrf, potrs   # noqa: E402

for n in [int(a) for a in sys.argv[1:]] or [4096]:
    h = handle()
    rng = np.random.default_rng(3)
    M = rng.normal(size=(n + 8, n)) * 2.0 ** -4
    A = M.T @ M + n * np.eye(n)
    Hm = dev(A)
    rc, info = potrf(Hm, n, n)
    assert rc == 0 and info == 0
    b = rng.normal(size=n)
    for _ in range(3):
        potrs(Hm, n, n, b.copy())
    nb = (n + 127) // 128
    buf = (ctypes.c_ulonglong * (4 * nb))()
    assert h.lib.ipm_debug_trsv_trace(buf, nb) == 0
    tr = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 4).astype(np.float64)
    t0 = tr[0, 2]
    pre, got, st = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0, (tr[:, 2] - t0) / 100.0
    det = got[1:] - st[:-1]           # x_{B+1} stored -> polled by the next ticket
    comp = st[1:] - got[1:]           # polled -> x_B stored
    wait = got[1:] - pre[1:]          # pre sum done -> x_{B+1} polled
    step = np.diff(st)
    print("n=%d: %d tickets, chain %.1f us, per step median %.2f us (mean %.2f)" % (n, nb, st[-1], np.median(step), step.mean()))
    print("  store -> next ticket polled: median %.2f  min %.2f  max %.2f us" % (np.median(det), det.min(), det.max()))
    print("  polled -> stored (the chain step's work): median %.2f  min %.2f  max %.2f us" % (np.median(comp), comp.min(), comp.max()))
    print("  pre sum done -> x_{B+1} polled: median %.2f  min %.2f us (small: the pre sum is on the chain)" % (np.median(wait), wait.min()))
    print("  pre sum done after the predecessor's store by: median %.2f us" % np.median(pre[1:] - st[:-1]))
