#!/bin/bash
set -o pipefail
o=gpurun_out/r5b3; mkdir -p $o
IPM_FUSED_GRAD=0 timeout -k 10 150 python -u -m pytest -x -v -s --timeout 140 --timeout-method thread tests/test_gpu_large.py -k "batched_cholesky_bitwise" > $o/batch_f0.txt 2>&1; echo "batch fused0 rc=$?"
grep -E "passed|failed|assert |Timeout" $o/batch_f0.txt | head -3
IPM355_LIB=$PWD/build/r5ab/lib_cc29a9f.so timeout -k 10 150 python -u -m pytest -x -v -s --timeout 140 --timeout-method thread tests/test_gpu_large.py -k "batched_cholesky_bitwise" > $o/batch_cc.txt 2>&1; echo "batch cc29a9f rc=$?"
grep -E "passed|failed|assert |Timeout" $o/batch_cc.txt | head -3
