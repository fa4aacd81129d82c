#!/bin/bash
# Round 4: per-role timelines of single fused Cholesky launches (diagnostic library with role
# stamps, build/rtr) at n = 2048 (blocks 2, 4, 6) and n = 8192 (blocks 4, 20, 28).
set -o pipefail
OUT=gpurun_out/${TAG:-r4t}
mkdir -p $OUT
export IPM355_LIB=$PWD/build/rtr/libipm355_trace.so
for nb in "2048 2" "2048 4" "2048 6" "8192 4" "8192 20" "8192 28"; do
  set -- $nb
  IPM_TRACE_BLOCK=$2 timeout -k 10 120 python scripts/role_trace.py $1 2>&1 | grep -v amdgpu.ids > $OUT/n$1_b$2.txt || exit 1
done
cat $OUT/n2048_b4.txt $OUT/n8192_b28.txt
