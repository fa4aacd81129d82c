#!/bin/bash
# race_check.py for several library specs (VAR=v@lib or lib) over SHAPES ("n:ncols:lda ...")
#   scripts/race_ab.sh OUT REPS "spec spec ..."
set -o pipefail
out=$1; mkdir -p $(dirname $out); : > $out
for spec in $3; do
  envs=""; lib=$spec
  if [[ "$spec" == *@* ]]; then envs=${spec%@*}; lib=${spec##*@}; fi
  for shp in ${SHAPES:-8194:8193:8208 8193:8192:8208 2049:2048:2064}; do
    echo "== $spec $shp" >> $out
    env $envs IPM355_LIB=$PWD/$lib timeout -k 10 150 python -u scripts/race_check.py ${shp//:/ } $2 2>&1 | grep -v amdgpu.ids >> $out || exit 1
    tail -1 $out
  done
done
