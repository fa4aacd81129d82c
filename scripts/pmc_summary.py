"""Per-dispatch PMC summary for one kernel from rocprofv3 --pmc CSV outputs (separate passes).

usage: pmc_summary.py <kernel-substring> <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json> [n m]

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: rocprofv3 reports both in KiB;
on gfx950 FETCH_SIZE reads exactly half the bytes of a wide coalesced stream
(MI355X_MICROARCH.md, HBM section) -> doubled.  Averaged over every dispatch of the kernel.
"""
import csv
import json
import sys


def per_dispatch(path, kname, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if kname in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


kname, fpath, wpath, out = sys.argv[1:5]
f = per_dispatch(fpath, kname, "FETCH_SIZE")
w = per_dispatch(wpath, kname, "WRITE_SIZE")
fetch = sum(f) / len(f) * 1024
write = sum(w) / len(w) * 1024
rec = {"kernel": kname, "dispatches": [len(f), len(w)], "fetch_size_bytes_raw": fetch,
       "write_size_bytes": write, "hbm_bytes_per_launch": 2 * fetch + write,
       "note": "FETCH_SIZE doubled (gfx950 reports half of wide coalesced reads); separate --pmc passes; "
               "Infinity-Cache hits are counted by FETCH_SIZE"}
if len(sys.argv) > 6:
    rec["n"], rec["m"] = int(sys.argv[5]), int(sys.argv[6])
rec["command"] = "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- python3 bench.py --no-cpu --steps 3 --warmup 1"
json.dump(rec, open(out, "w"), indent=1)
print(json.dumps(rec))
