"""Per-launch durations and inter-launch gaps of the LAST factorization in a rocprofv3 kernel trace
of scripts/potrf_time.py.   python scripts/potrf_launches.py <run_kernel_trace.csv> [nlaunch]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted([(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "potrf_block" in r["Kernel_Name"]],
            key=lambda k: k[1])
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 32
seq = ks[-nl:]
t0 = seq[0][1]
tot = 0
for i, (nm, s, e) in enumerate(seq):
    gap = (s - seq[i - 1][2]) / 1e3 if i else 0.0
    inst = nm[nm.find("<") + 1:nm.find(">")]
    print(f"{i:3d} {inst:18s} start {(s - t0) / 1e3:8.1f} dur {(e - s) / 1e3:7.1f} gap {gap:5.1f}")
    tot += e - s
print(f"sum of launches {tot / 1e3:.1f} us, span {(seq[-1][2] - t0) / 1e3:.1f} us")
