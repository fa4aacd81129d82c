#!/bin/bash
set -o pipefail
o=gpurun_out/r5bs; mkdir -p $o
for c in 91310d7 cc29a9f a0570e0; do
  IPM355_LIB=$PWD/build/r5ab/lib_$c.so timeout -k 10 100 python -u -m pytest -x -q -s --timeout 90 --timeout-method thread tests/test_gpu_large.py -k batched_cholesky_bitwise > $o/$c.txt 2>&1
  echo "$c rc=$?"; grep -E "assert|passed|failed|Timeout|batched cholesky" $o/$c.txt | head -5
done
