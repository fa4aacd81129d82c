#!/bin/bash
# border/flag fusion (lib_bf) tests + configs A/B; step-1 pair (lib_s1) bitwise + POTRF A/B
set -o pipefail
o=gpurun_out/r5fa; mkdir -p $o
IPM355_LIB=$PWD/build/r5ab/lib_bf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_kernels.py > $o/tests_bf.txt 2>&1; echo "tests bf rc=$?"; tail -1 $o/tests_bf.txt
REPS=2 scripts/r5_dl.sh $o/s1 base s1 2>&1 | grep -v amdgpu.ids | grep -E "bitwise|DIFF"
sort $o/s1/potrf_ab.txt | awk '{print $1, $3, $6, $7}'
for v in base bf; do
  if [ $v = bf ]; then export IPM355_LIB=$PWD/build/r5ab/lib_bf.so; else unset IPM355_LIB; fi
  scripts/cfg_quick.sh $o/cfg_$v | sed "s/^/$v /"
done
