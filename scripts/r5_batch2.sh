#!/bin/bash
set -o pipefail
o=gpurun_out/r5b2; mkdir -p $o
timeout -k 10 150 python -u -m pytest -x -v -s --timeout 140 --timeout-method thread tests/test_gpu_large.py -k "batched_cholesky_bitwise or shard_on_one_gpu" > $o/batch.txt 2>&1; echo "batch rc=$?"
grep -E "passed|failed|assert |Timeout|batched cholesky" $o/batch.txt | head -5
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_kernels.py -k "tail" > $o/tail.txt 2>&1; echo "tail rc=$?"; tail -2 $o/tail.txt
