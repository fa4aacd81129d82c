"""Per-dispatch PMC summary for one kernel from rocprofv3 --pmc CSV outputs (separate passes).

usage: pmc_summary.py <kernel-substring> <out.json> n m <pass.csv> [<pass.csv> ...]

Every counter found in the pass files for dispatches of the kernel is averaged per dispatch.
Derived:
* HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: rocprofv3 reports both in KiB;
  on gfx950 FETCH_SIZE reads exactly half the bytes of a wide coalesced stream
  (MI355X_MICROARCH.md, HBM section) -> doubled.  FETCH_SIZE counts Infinity-Cache hits as well.
* MFMA: SQ_VALU_MFMA_BUSY_CYCLES per launch; the effective clock GRBM_GUI_ACTIVE / 8 XCDs / kernel
  duration (MI355X_MICROARCH.md, DVFS), and busy cycles / (256 CUs x 4 SIMDs x active cycles) as
  the MFMA-pipe busy fraction.
The record carries the sha256 of libipm355.so and the git commit it was collected on; bench.py
refuses a summary whose library hash differs from the library it runs.
"""
import csv
import hashlib
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "interiorpoint-gpu_amd", "ipm355", "libipm355.so")


def per_dispatch(path, kname):
    """{counter: [value per dispatch]} and {dispatch: duration ns} (if the row carries timestamps)"""
    vals = {}
    for r in csv.DictReader(open(path)):
        if kname not in r.get("Kernel_Name", ""):
            continue
        c = r.get("Counter_Name")
        vals.setdefault(c, {})
        vals[c][r["Dispatch_Id"]] = vals[c].get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {c: list(v.values()) for c, v in vals.items()}


def durations(trace_csv, kname):
    out = []
    try:
        for r in csv.DictReader(open(trace_csv)):
            if kname in r.get("Kernel_Name", ""):
                out.append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    except Exception:
        pass
    return out


def main():
    kname, out, n, m = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    counters, dur = {}, []
    for p in sys.argv[5:]:
        for c, v in per_dispatch(p, kname).items():
            counters[c] = {"mean": sum(v) / len(v), "dispatches": len(v)}
        tr = os.path.join(os.path.dirname(p), os.path.basename(p).replace("counter_collection", "kernel_trace"))
        if os.path.exists(tr) and "GRBM_GUI_ACTIVE" in per_dispatch(p, kname):
            dur = durations(tr, kname)
    rec = {"kernel": kname, "n": n, "m": m, "counters": counters}
    if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
        fetch = counters["FETCH_SIZE"]["mean"] * 1024
        write = counters["WRITE_SIZE"]["mean"] * 1024
        rec.update(fetch_size_bytes_raw=fetch, write_size_bytes=write, hbm_bytes_per_launch=2 * fetch + write)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in counters:
        mf = {"busy_cycles_per_launch": counters["SQ_VALU_MFMA_BUSY_CYCLES"]["mean"]}
        if "GRBM_GUI_ACTIVE" in counters:
            act = counters["GRBM_GUI_ACTIVE"]["mean"] / 8.0
            mf["active_cycles_per_xcd"] = act
            mf["busy_frac_of_simd_cycles"] = mf["busy_cycles_per_launch"] / (256 * 4 * act)
            if dur:
                d = sum(dur) / len(dur)
                mf["kernel_ns_profiled"] = d
                mf["effective_clock_ghz"] = act / d
        rec["mfma"] = mf
    rec["note"] = ("separate --pmc passes of `python3 bench.py --no-cpu` (profiled runs clock lower than "
                   "unprofiled ones); FETCH_SIZE doubled (gfx950 reports half of wide coalesced reads) and "
                   "counts Infinity-Cache hits")
    rec["lib_sha256"] = hashlib.sha256(open(LIB, "rb").read()).hexdigest()
    try:
        rec["commit"] = os.environ.get("IPM_COMMIT") or subprocess.run(["git", "-C", REPO, "rev-parse", "HEAD"], capture_output=True,
                                       text=True).stdout.strip() or None
    except Exception:
        rec["commit"] = None
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
