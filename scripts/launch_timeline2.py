"""Per-launch durations of the last Cholesky of a potrf-only run (scripts/potrf_once.py) from a
rocprofv3 kernel trace: the last `count` k_potrf_block launches.
    python scripts/launch_timeline2.py <run_kernel_trace.csv> [count]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
cnt = int(sys.argv[2]) if len(sys.argv) > 2 else 32
ks = sorted([(r["Kernel_Name"][:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
             if "potrf_block" in r["Kernel_Name"]], key=lambda k: k[1])[-cnt:]
print(" ".join(f"{(k[2] - k[1]) / 1e3:.0f}" for k in ks))
gaps = [(ks[i + 1][1] - ks[i][2]) / 1e3 for i in range(len(ks) - 1)]
print("sum %.1f us, span %.1f us, gaps %.1f us, n %d" % (sum(k[2] - k[1] for k in ks) / 1e3,
                                                        (ks[-1][2] - ks[0][1]) / 1e3, sum(gaps), len(ks)))
