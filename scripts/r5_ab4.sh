#!/bin/bash
set -o pipefail
o=gpurun_out/r5q; mkdir -p $o
IPM355_LIB=$PWD/build/r5ab/tr_fa4.so IPM_TRACE_BLOCK=4 timeout -k 10 120 python scripts/role_trace.py 2048 > $o/st_fa4_n2048_b4.txt 2>&1 || exit 1
REPS=2 scripts/potrf_ab.sh $o/potrf_ab.txt build/r5ab/lib_fp2.so build/r5ab/lib_fa2.so build/r5ab/lib_fa4.so \
  HIP_FORCE_DEV_KERNARG=1@build/r5ab/lib_fp2.so HIP_FORCE_DEV_KERNARG=0@build/r5ab/lib_fp2.so
