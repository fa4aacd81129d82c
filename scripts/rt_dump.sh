#!/bin/bash
# raw role timelines for several (n, block) pairs: scripts/rt_dump.sh OUTDIR LIB "n:b n:b ..."
set -o pipefail
o=$1; lib=$2; mkdir -p $o
for nb in $3; do
  n=${nb%:*}; b=${nb#*:}
  IPM355_LIB=$PWD/$lib IPM_TRACE_BLOCK=$b timeout -k 10 120 python scripts/role_dump.py $n $o/n${n}_b$b.npz || exit 1
  IPM355_LIB=$PWD/$lib IPM_TRACE_BLOCK=$b timeout -k 10 120 python scripts/role_trace.py $n > $o/n${n}_b$b.txt 2>&1 || exit 1
done
