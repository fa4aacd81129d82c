#!/bin/bash
# race_check.py over several shapes for each library: scripts/race_run.sh OUT "lib lib ..." [REPS]
set -o pipefail
out=$1; mkdir -p $(dirname $out); : > $out
for lib in $2; do
  for shp in "8194 8193 8194" "8193 8192 8194" "8192 8192 8192" "2049 2048 2050" "4097 4096 4098"; do
    echo "== $lib $shp" >> $out
    IPM355_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/race_check.py $shp ${3:-30} 2>&1 | grep -v amdgpu.ids >> $out || exit 1
  done
done
