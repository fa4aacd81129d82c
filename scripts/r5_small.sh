#!/bin/bash
set -o pipefail
o=gpurun_out/r5sm; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_kernels.py > $o/tests.txt 2>&1; echo "tests rc=$?"; tail -2 $o/tests.txt
scripts/cfg_quick.sh $o/cfg
