"""Per-launch durations of the last Cholesky (k_potrf_block launches between the last two KKT SYRKs)
from a rocprofv3 kernel trace.   python scripts/launch_timeline.py <run_kernel_trace.csv>"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted([(r["Kernel_Name"][:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows],
            key=lambda k: k[1])
sy = [i for i, k in enumerate(ks) if "k_mfma_gemm<128, true" in k[0]]
a, b = sy[-2], len(ks)
seq = [k for k in ks[a:b] if "potrf_block" in k[0]]
seq = seq[:40]
t0 = seq[0][1]
print(" ".join(f"{(k[2] - k[1]) / 1e3:.0f}" for k in seq))
print("sum", sum(k[2] - k[1] for k in seq) / 1e3, "span", (seq[-1][2] - t0) / 1e3, "n", len(seq))
