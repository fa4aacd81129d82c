#!/bin/bash
set -o pipefail
o=gpurun_out/r5ts; mkdir -p $o
IPM355_LIB=$PWD/build/r5ab/lib_ts.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py > $o/kern.txt 2>&1; echo "kernels rc=$?"; tail -1 $o/kern.txt
REPS=2 scripts/r5_dl.sh $o/ab base ts 2>&1 | grep -v amdgpu.ids | grep -E "bitwise|DIFF"
sort $o/ab/potrf_ab.txt | awk '{print $1, $3, $6, $7}'
