#!/bin/bash
# quick GPU pass: the named test files/expressions, then the LU timing
set -o pipefail
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
timeout -k 10 ${TT:-900} python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/lu_time.py > $OUT/lu_time.json 2> $OUT/lu_time.err; rc=$?; cat $OUT/lu_time.json; exit $rc
