"""Role timeline of ONE fused Cholesky launch (block b) from the diagnostic library.
   make trace && IPM_TRACE_BLOCK=b python scripts/role_trace.py [n]
Prints, per role, count / first start / last end / mean duration (us from the launch's first start)."""
import ctypes, os, sys
os.environ.setdefault("IPM355_LIB", "/root/repo/build/trace/libipm355_trace.so")
sys.path[:0] = ["/root/repo/interiorpoint-gpu_amd", "/root/repo/tests"]
import numpy as np
import torch
from gpu_util import handle
from ipm355 import _lib as L
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
h = handle()
torch.manual_seed(0)
M = torch.rand(n, n, dtype=torch.float64, device="cuda")
A = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
for _ in range(2):
    Hc = A.clone(); torch.cuda.synchronize()
    info = ctypes.c_int(0)
    h.lib.ipm_potrf(h.ptr, n, L.dptr(Hc), n, ctypes.byref(info))
    torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (4 * 8192))()
rc = h.lib.ipm_debug_role_trace(buf, 8192)
a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4).astype(np.int64)
a = a[a[:, 1] > 0]
t0 = a[:, 1].min()
names = {0: "LA tile", 1: "P(a) diag", 2: "P(a) row<nchd", 3: "P(b) diag", 4: "S tile", 5: "P(a) row", 6: "P(b) row",
         7: "S sleep@Pa", 8: "S sleep@Pb", 9: "NF fold tile", 12: "ragged rows", 13: "tail"}
print(f"block {os.environ.get('IPM_TRACE_BLOCK')} n={n}: {len(a)} workgroups, span {(a[:, 2].max() - t0) / 100:.1f} us")
for r in sorted(set((a[:, 0] >> 32).tolist())):
    s = a[(a[:, 0] >> 32) == r]
    d = (s[:, 2] - s[:, 1]) / 100
    print(f"  {str(names.get(r, r)):14s} n={len(s):5d} start {(s[:, 1].min() - t0) / 100:7.1f}..{(s[:, 1].max() - t0) / 100:7.1f}"
          f"  end {(s[:, 2].min() - t0) / 100:7.1f}..{(s[:, 2].max() - t0) / 100:7.1f}  dur mean {d.mean():6.1f} max {d.max():6.1f}")
print(f"  distinct CU keys {len(set(a[:, 3].tolist()))}")
# S-tile durations by start time (are mid-launch tiles, with no panel work beside them, slower?)
s = a[(a[:, 0] >> 32) == 4]
st = (s[:, 1] - t0) / 100
du = (s[:, 2] - s[:, 1]) / 100
for lo in range(0, int(st.max()) + 50, 50):
    m = (st >= lo) & (st < lo + 50)
    if m.any():
        print(f"    S tiles starting {lo:4d}-{lo + 50:4d} us: n={m.sum():4d} dur mean {du[m].mean():6.1f} min {du[m].min():6.1f}")
# NF fold tiles (diagnostic build): spin end (wake), operands loaded, end -- us from the launch start
s = a[(a[:, 0] >> 32) == 9]
for row in s[np.argsort(s[:, 3])]:
    wake, loaded = row[3], row[1] + (row[0] & 0xFFFFFFFF)
    if 0 < wake - t0 < 10 ** 9:
        print(f"    NF tile wake {(wake - t0) / 100:6.1f}  loaded {(loaded - t0) / 100:6.1f}  end {(row[2] - t0) / 100:6.1f}")

# the traced launch's P(a) diagonal role, stamped inside the fused kernel (s_memtime cycles; the
# same phases as tools/leaf2_lab.hip prints for the role alone)
st = (ctypes.c_ulonglong * 128)()
if hasattr(h.lib, "ipm_debug_diag_stamps") and h.lib.ipm_debug_diag_stamps(st) == 0:
    s = np.frombuffer(st, dtype=np.uint64).astype(np.int64)
    if s[0] > 0 and s[26] > s[0]:
        print(f"  P(a) diagonal role in the launch: {s[26] - s[0]} cycles to its last progress word, "
              f"panel load {s[1] - s[0]}")
        print("   leaf phases per J: operands landed / sweep / stores:",
              "  ".join(f"{s[48 + J] - s[2 + 3 * J]}/{s[56 + J] - s[48 + J]}/{s[32 + J] - s[56 + J]}" for J in range(8)))
        print("   J  step1+bar  leaf(w0)  bar-wait  progress | inv(w3)  free waves done (w1 w2 w3), from step-1 end")
        for J in range(8):
            st0 = s[1] if J == 0 else s[4 + 3 * (J - 1)]
            b = s[2 + 3 * J]
            fw = " ".join(f"{s[80 + 8 * w + J] - b:7d}" for w in (1, 2, 3)) if J else ""
            print(f"  {J:2d} {b - st0:9d} {s[32 + J] - b:9d} {s[3 + 3 * J] - s[32 + J]:9d} "
                  f"{s[4 + 3 * J] - s[3 + 3 * J]:9d} | {(s[40 + J] - b) if J else 0:7d}  {fw}")

# look-ahead fold tiles (the P(a) diagonal block's 32-tiles): per tile, us from the launch start
ft = (ctypes.c_ulonglong * (32 * 12))()
if hasattr(h.lib, "ipm_debug_fold_trace") and h.lib.ipm_debug_fold_trace(ft) == 0:
    f = np.frombuffer(ft, dtype=np.uint64).reshape(32, 12).astype(np.int64)
    for i in range(32):
        r = f[i]
        if r[0] <= 0 or not (0 <= r[0] - t0 < 10 ** 8):
            continue
        npass = int(r[11])
        us = lambda v: f"{(v - t0) / 100:6.1f}" if v > 0 else "   -  "
        ps = "  ".join(f"p{p} ld {us(r[2 + 2 * p])} mf {us(r[3 + 2 * p])}" for p in range(min(npass, 4)))
        print(f"    {'fold' if i < 16 else 'NF  '} tile {i % 16:2d} K={128 * npass:4d} start {us(r[0])} wake {us(r[1])}  {ps}  done {us(r[10])}")
