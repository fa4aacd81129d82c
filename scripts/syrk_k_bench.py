"""Standalone SYRK rate vs K and n (HIP events): is a K=256 trailing update intrinsically slower
than the K=2048 KKT SYRK?   python scripts/syrk_k_bench.py"""
import ctypes, sys
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import torch
from gpu_util import handle
from ipm355 import _lib as L
h = handle()
for n, k in [(8192, 2048), (8192, 256), (7680, 256), (6144, 256), (4096, 256), (2048, 256), (7680, 512), (4096, 512)]:
    X = torch.rand(k, n, dtype=torch.float64, device="cuda")
    H = torch.zeros(n, n, dtype=torch.float64, device="cuda")
    ts = []
    for r in range(6):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        h.check(h.lib.ipm_syrk(h.ptr, n, k, L.dptr(X), n, None, 1.0, 0.0, L.dptr(H), n), h.ptr)
        e.record(); torch.cuda.synchronize()
        if r: ts.append(s.elapsed_time(e))
    ts.sort()
    t = ts[len(ts) // 2]
    print(f"syrk n={n} k={k}: {t*1e3:8.1f} us  {k*n*(n+1)/t/1e9:6.1f} TF/s", flush=True)
