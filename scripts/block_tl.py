"""Per-launch durations of the fused Cholesky (k_potrf_block) in a kernel trace (last potrf)."""
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'k_potrf_block' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
rows = rows[len(rows) // 2:]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
t0 = int(rows[0]['Start_Timestamp']); prev = t0
for b, r in enumerate(rows):
    s = int(r['Start_Timestamp']); e = int(r['End_Timestamp'])
    m = n - 256 * (b + 1); t = -(-m // 128); tiles = t * (t + 1) // 2 if b > 0 and m > 0 else 0
    print(f"b={b:2d} start={(s - t0) / 1e3:8.1f} gap={(s - prev) / 1e3:5.1f} dur={(e - s) / 1e3:7.1f}us  S tiles={tiles}")
    prev = e
print("total", (prev - t0) / 1e3)
