#!/bin/bash
# A/B of two variant libraries (build/r5ab/lib_A.so vs lib_B.so, trace builds tr_A / tr_B):
# bitwise factor check, role timelines, POTRF times.   scripts/r5_dl.sh OUTDIR A B
set -o pipefail
o=$1; A=$2; B=$3; mkdir -p $o
for n in 2048 4100; do
  for v in $A $B; do
    IPM355_LIB=$PWD/build/r5ab/lib_$v.so timeout -k 10 120 python scripts/potrf_dump.py $n $o/f_${v}_$n.npy || exit 1
  done
done
O=$o A=$A B=$B python - <<'PY' || exit 1
import numpy as np, os
o, A, B = os.environ["O"], os.environ["A"], os.environ["B"]
for n in (2048, 4100):
    a = np.load(f"{o}/f_{A}_{n}.npy"); b = np.load(f"{o}/f_{B}_{n}.npy")
    print(n, "bitwise equal" if np.array_equal(a, b) else f"DIFF max {np.abs(a-b).max():.3e}", flush=True)
PY
rm -f $o/*.npy
for v in $A $B; do
  [ -f build/r5ab/tr_$v.so ] || continue
  IPM355_LIB=$PWD/build/r5ab/tr_$v.so IPM_TRACE_BLOCK=4 timeout -k 10 120 python scripts/role_trace.py 2048 > $o/st_${v}_n2048_b4.txt 2>&1 || exit 1
done
REPS=${REPS:-2} scripts/potrf_ab.sh $o/potrf_ab.txt build/r5ab/lib_$A.so build/r5ab/lib_$B.so
