"""Summarise a rocprofv3 kernel-trace CSV: per-kernel count / total / mean (ms)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
tot = sum(sum(v) for v in agg.values())
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{k:70s} {len(v):6d} {sum(v):9.3f} {sum(v) / len(v):8.4f}  {100 * sum(v) / tot:5.1f}%")
