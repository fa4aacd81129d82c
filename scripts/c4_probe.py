"""Config-4 concurrency probe: the eight M4 instances solved concurrently through ipm355.dist.Shard,
each instance's completion time, Newton iterations and backup-path flag printed as it finishes
(flushed), so a slow or stuck run names the instance.  python scripts/c4_probe.py [budget_s]"""
import os, sys, time, threading
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import numpy as np
from test_gpu_large import _fixture, _instance, rel
from ipm355 import dist, QPSolver
zs = [_fixture(f"m4_qp_{sd}") for sd in range(1000, 1008)]
insts = [_instance(z)[1] for z in zs]
sh = dist.Shard(lambda i: dict(insts[i]), range(8), QPSolver, device=0, concurrent=True)
t0 = time.perf_counter()
orig = sh.solvers
done = {}
def watch():
    while len(done) < 8 and time.perf_counter() - t0 < float(sys.argv[1] if len(sys.argv) > 1 else 60):
        time.sleep(5)
        print(f"  [{time.perf_counter() - t0:6.1f} s] finished {sorted(done)}", flush=True)
threading.Thread(target=watch, daemon=True).start()
import ipm355.dist as D
one_orig = None
out = {}
def solve_one(k):
    s = sh.solvers[k]
    with D._on(sh.streams[k]):
        v = s.solve()
        sh.streams[k].synchronize()
    p1 = getattr(s, "phase1_solver", None)
    it = int(sum(s.inner_iters)) + (int(sum(p1.inner_iters)) if p1 is not None else 0)
    bk = [getattr(getattr(fm, "prob", None), "use_backup", None) for fm in (getattr(s, "fm", None), getattr(p1, "phase1_fm", None)) if fm is not None]
    done[k] = time.perf_counter() - t0
    ref = int(sum(zs[k]["inner_iters"]) + sum(zs[k]["phase1_inner_iters"]))
    print(f"instance {k}: {done[k]:.2f} s, iters {it} (ref {ref}), x* rel {rel(s.xstar, zs[k]['xstar']):.2e}, backup {bk}", flush=True)
from concurrent.futures import ThreadPoolExecutor
with ThreadPoolExecutor(8) as ex:
    list(ex.map(solve_one, range(8)))
print(f"all done in {time.perf_counter() - t0:.2f} s", flush=True)
