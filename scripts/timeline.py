"""Timeline of the LAST potrf in a kernel trace: per-kernel-type busy time, critical-path view."""
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if "ipm::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# last potrf = kernels after the last k_potrf_diag with k0 == 0 ... approximate: take the second half
starts = [i for i, r in enumerate(rows) if "k_potrf_diag" in r["Kernel_Name"] or "k_potrf_panel" in r["Kernel_Name"]]
half = starts[len(starts) // 2]
rows = rows[half:]
t0 = int(rows[0]["Start_Timestamp"]); t1 = max(int(r["End_Timestamp"]) for r in rows)
print(f"span {(t1 - t0) / 1e6:.3f} ms, {len(rows)} kernels")
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    k = r["Kernel_Name"].split("(")[0][-40:] + " q" + r["Queue_Id"] if "Queue_Id" in r else r["Kernel_Name"][:40]
    agg[k][0] += 1; agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:50s} {c:5d} {t:8.3f} ms  avg {t / c * 1e3:7.1f} us")
# first 12 blocks' events
for r in rows[:40]:
    print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {(int(r['End_Timestamp']) - t0) / 1e3:9.1f}  q{r.get('Queue_Id','?')} {r['Kernel_Name'][:50]}")
print("... last blocks")
for r in rows[-30:]:
    print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {(int(r['End_Timestamp']) - t0) / 1e3:9.1f}  q{r.get('Queue_Id','?')} {r['Kernel_Name'][:50]}")
