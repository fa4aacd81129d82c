#!/bin/bash
set -o pipefail
o=gpurun_out/r5bf; mkdir -p $o
IPM355_LIB=$PWD/build/r5ab/lib_bf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_kernels.py > $o/tests.txt 2>&1; echo "tests rc=$?"; tail -2 $o/tests.txt
for v in base bf; do
  if [ $v = bf ]; then export IPM355_LIB=$PWD/build/r5ab/lib_bf.so; else unset IPM355_LIB; fi
  scripts/cfg_quick.sh $o/cfg_$v | sed "s/^/$v /"
done
