#!/bin/bash
# one-stream leaf (build/v1, IPM_DIAG_V=32898) vs the shipped two-stream leaf: bitwise factor
# comparison, then POTRF timings alternating
set -o pipefail
V1=/root/repo/build/v1/libipm355.so
mkdir -p gpurun_out/one
for n in 2048 4100; do
  timeout -k 10 120 python scripts/potrf_dump.py $n gpurun_out/one/f0_$n.npy || exit $?
  IPM355_LIB=$V1 timeout -k 10 120 python scripts/potrf_dump.py $n gpurun_out/one/f1_$n.npy || exit $?
  python3 -c "
import numpy as np; a=np.load('gpurun_out/one/f0_$n.npy'); b=np.load('gpurun_out/one/f1_$n.npy')
print('n=$n bitwise identical:', np.array_equal(a,b), 'max diff', np.abs(a-b).max())"
done
rm -f gpurun_out/one/*.npy
for r in 1 2; do
  for n in 8192 2048; do
    timeout -k 10 120 python scripts/potrf_time.py $n 9 || exit $?
    IPM355_LIB=$V1 timeout -k 10 120 python scripts/potrf_time.py $n 9 | sed 's/^/V1 /' || exit $?
  done
done
