"""KKT SYRK launch time (HIP events, median of 15) at the headline shape, for the tail mode the
process runs with (IPM_STREAMK=0|1|2|3, see ipm_mfma.h).   python scripts/syrk_tail_bench.py"""
import os, sys
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import torch
from gpu_util import handle
from ipm355 import _lib as L
h = handle()
mode = os.environ.get("IPM_STREAMK", "1")
for n, k in [(8192, 2048), (8100, 2050)]:
    g = torch.Generator(device="cuda").manual_seed(n)
    X = torch.rand(k, n, dtype=torch.float64, device="cuda", generator=g)
    w = torch.rand(k, dtype=torch.float64, device="cuda", generator=g) + 0.5
    H = torch.zeros(n, n, dtype=torch.float64, device="cuda")
    ts = []
    for r in range(16):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        h.check(h.lib.ipm_syrk(h.ptr, n, k, L.dptr(X), n, L.dptr(w), 1.0, 0.0, L.dptr(H), n), h.ptr)
        e.record(); torch.cuda.synchronize()
        if r: ts.append(s.elapsed_time(e))
    ts.sort()
    t = ts[len(ts) // 2]
    cs = float(torch.tril(H).sum())
    print(f"mode={mode} syrk n={n} k={k}: {t*1e3:8.1f} us  {k*n*(n+1)/t/1e9:6.1f} TF/s  checksum {cs:.15e}", flush=True)
