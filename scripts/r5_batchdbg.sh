#!/bin/bash
set -o pipefail
o=gpurun_out/r5bd; mkdir -p $o
IPM_TAIL=0 timeout -k 10 150 python -u -m pytest -x -v -s --timeout 140 --timeout-method thread tests/test_gpu_large.py -k batched_cholesky_bitwise > $o/tail0.txt 2>&1; echo "tail0 rc=$?"
tail -5 $o/tail0.txt
IPM_FUSED_GRAD=0 timeout -k 10 150 python -u -m pytest -x -v -s --timeout 140 --timeout-method thread tests/test_gpu_large.py -k batched_cholesky_bitwise > $o/fused0.txt 2>&1; echo "fused0 rc=$?"
tail -5 $o/fused0.txt
