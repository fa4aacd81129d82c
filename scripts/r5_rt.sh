#!/bin/bash
# role timelines of one library (trace build): scripts/r5_rt.sh OUTDIR LIB "n:b n:b ..."
set -o pipefail
o=$1; lib=$2; mkdir -p $o
for nb in ${3:-2048:4 2048:6 8192:20 8192:28}; do
  n=${nb%:*}; b=${nb#*:}
  IPM355_LIB=$PWD/$lib IPM_TRACE_BLOCK=$b timeout -k 10 120 python scripts/role_trace.py $n > $o/n${n}_b$b.txt 2>&1 || exit 1
done
