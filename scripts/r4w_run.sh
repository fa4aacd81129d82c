#!/bin/bash
# Round 4: the look-ahead 32-tiles through the LDS-staged fold (this tree; IPM_LA32F=0 selects the
# slab loop in the same library) against the r4v library (NF fold only), POTRF at n = 8193 / 4096 /
# 2048, two pairs; then the Cholesky GPU tests on this tree.
set -o pipefail
OUT=gpurun_out/r4w
mkdir -p $OUT
NEW=interiorpoint-gpu_amd/ipm355/libipm355.so
for r in 1 2; do
  for cfg in "build/abh/r4v/libipm355.so 1" "$NEW 1" "$NEW 0"; do
    set -- $cfg
    for n in "8193 9 8194" "4096 15" "2048 25"; do
      IPM_LA32F=$2 IPM355_LIB=$PWD/$1 timeout -k 10 120 python scripts/potrf_time.py $n | sed "s|^|$1 la32f=$2 |" || exit $?
    done
  done
done 2>&1 | grep -v amdgpu.ids | tee $OUT/potrf_ab.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "potrf or chol or block or potrs" --timeout 120 --timeout-method thread > $OUT/pytest_potrf.log 2>&1
rc=$?; echo "pytest potrf rc=$rc"; tail -2 $OUT/pytest_potrf.log
exit $rc
