"""Full-solve probe (tests/test_gpu_large.py test_m3_full_solve without the assertions): solves the
fixture while a watchdog prints the elapsed time every 10 s, then reports steps, timing, whether a
problem fell to the least-squares backup (Q9) and the distance to the reference.
   python scripts/full_probe.py m3_qp_full"""
import sys, threading, time
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import numpy as np
from test_gpu_large import _fixture, _instance, _cls, _device_trace, rel
name = sys.argv[1]
z = _fixture(name)
spec, kw = _instance(z)
s = _cls(spec)(check_cvxpy=False, suppress_print=True, **kw)
t0 = time.perf_counter()
done = []
def watch():
    while not done:
        time.sleep(10)
        if not done:
            p1 = s.phase1_solver
            n1 = len(p1.phase1_ns.trace) if p1 is not None and hasattr(p1, "phase1_ns") else -1
            n2 = len(s.ns.trace) if hasattr(s, "ns") else -1
            print(f"  [{time.perf_counter() - t0:6.1f} s] phase-1 steps {n1}, barrier steps {n2}", flush=True)
threading.Thread(target=watch, daemon=True).start()
v = s.solve()
done.append(1)
steps, nds = _device_trace(s)
p1 = s.phase1_solver
bk = [getattr(getattr(fm, "prob", None), "use_backup", None) for fm in (getattr(s, "fm", None), getattr(p1, "phase1_fm", None)) if fm is not None]
ref = z["trace_step"]
k = min(len(steps), len(ref))
first = int(np.argmax(steps[:k] != ref[:k])) if np.any(steps[:k] != ref[:k]) else k
print(f"[{name}] {time.perf_counter() - t0:.1f} s, {len(steps)} steps (ref {len(ref)}), x* rel {rel(s.xstar, z['xstar']):.2e}, "
      f"backup {bk}, first differing step {first}", flush=True)
