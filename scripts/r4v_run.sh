#!/bin/bash
# Round 4: the next-diagonal-block fold tiles staged through LDS with 16-byte direct loads (this
# tree) against the r4s library (build/abh/r4s): POTRF at n = 8193 / 4096 / 2048, two pairs; the
# Cholesky GPU tests; role traces of the new fold (n = 2048 block 4, n = 8192 block 28).
set -o pipefail
OUT=gpurun_out/r4v
mkdir -p $OUT
NEW=interiorpoint-gpu_amd/ipm355/libipm355.so
for r in 1 2; do
  for lib in build/abh/r4s/libipm355.so $NEW; do
    for n in "8193 9 8194" "4096 15" "2048 25"; do
      IPM355_LIB=$PWD/$lib timeout -k 10 120 python scripts/potrf_time.py $n | sed "s|^|$lib |" || exit $?
    done
  done
done 2>&1 | grep -v amdgpu.ids | tee $OUT/potrf_ab.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "potrf or chol or block or potrs" --timeout 120 --timeout-method thread > $OUT/pytest_potrf.log 2>&1
rc=$?; echo "pytest potrf rc=$rc"; tail -2 $OUT/pytest_potrf.log
[ $rc -ne 0 ] && exit $rc
export IPM355_LIB=$PWD/build/rtr/libipm355_trace.so
for nb in "2048 4" "8192 28"; do
  set -- $nb
  IPM_TRACE_BLOCK=$2 timeout -k 10 120 python scripts/role_trace.py $1 2>&1 | grep -v amdgpu.ids > $OUT/n$1_b$2.txt || exit 1
done
head -12 $OUT/n2048_b4.txt
