#!/bin/bash
# raw role timelines of several launches: scripts/rt_dump.sh OUTDIR LIB n "b b b ..."
set -o pipefail
o=$1; lib=$2; n=$3; mkdir -p $o
for b in $4; do
  IPM355_LIB=$PWD/$lib IPM_TRACE_BLOCK=$b timeout -k 10 120 python scripts/role_dump.py $n $o/n${n}_b$b.npz || exit 1
done
