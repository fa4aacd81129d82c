"""in-process repro of the r3e bench core dump (CPU only).  Run with OMP_NUM_THREADS=2
and a larger limit, e.g.  OMP_NUM_THREADS=2 python -X faulthandler scripts/openblas_thread_repro.py 8"""
import numpy as np, scipy.linalg as sl, threadpoolctl, sys
for i in threadpoolctl.threadpool_info(): print(i['prefix'], i['num_threads'], i['version'])
n = 3000
a = np.random.rand(n, n); a = a @ a.T + n * np.eye(n)
for lim in [int(x) for x in sys.argv[1:]]:
    with threadpoolctl.threadpool_limits(lim):
        for i in threadpoolctl.threadpool_info(): print(' set', lim, '->', i['prefix'], i['num_threads'])
        c = sl.cho_factor(a, lower=True); x = sl.cho_solve(c, np.ones(n)); b = a @ a; e = np.linalg.eigvalsh(a[:500,:500])
print("ok")
