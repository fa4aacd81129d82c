"""Run-to-run determinism of a truncated M3 trajectory (tests/test_gpu_large.py
test_m3_truncated_trajectory): solve the same fixture `reps` times in one process and print x_K's
distance to the reference and a digest of its bytes.   python scripts/traj_repeat.py NAME REPS"""
import hashlib, sys, time
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import numpy as np
from test_gpu_large import _fixture, _instance, _cls, _device_trace, rel
name, reps = sys.argv[1], int(sys.argv[2])
z = _fixture(name)
spec, kw = _instance(z)
K = int(z["k_steps"])
for r in range(reps):
    t0 = time.perf_counter()
    s = _cls(spec)(check_cvxpy=False, suppress_print=True, **kw)
    s.solve(iteration_budget=K)
    steps, nds = _device_trace(s)
    xk = (s.phase1_solver.x if len(z["x_k"]) == spec["n"] + 1 else s.x_last).cpu().numpy()
    print(f"[{name}] run {r}: x_K rel {rel(xk, z['x_k']):.3e} digest {hashlib.sha1(xk.tobytes()).hexdigest()[:12]} "
          f"nd digest {hashlib.sha1(np.asarray(nds).tobytes()).hexdigest()[:12]} ({time.perf_counter() - t0:.1f} s)",
          flush=True)
