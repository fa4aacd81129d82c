#!/bin/bash
# kernel tests of one library, then an A/B of library specs on the Cholesky alone:
#   scripts/ab_run.sh OUTDIR TESTLIB "spec spec ..."   (spec: lib or VAR=v@lib; env SIZES, REPS)
set -o pipefail
o=$1; mkdir -p $o
IPM355_LIB=$PWD/$2 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "potrf or chol" > $o/kernels.log 2>&1
rc=$?; tail -2 $o/kernels.log; [ $rc -ne 0 ] && exit $rc
REPS=${REPS:-2} SIZES=${SIZES:-"8193:7:8194 4096:11 2048:15"} scripts/potrf_ab.sh $o/ab.txt $3
