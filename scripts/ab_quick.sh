#!/bin/bash
# kernel tests (potrf) with the current library, then A/B bench vs build/old/libipm355.so
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q -k "${KSEL:-potrf}" --timeout 120 --timeout-method thread > gpurun_out/k.log 2>&1
rc=$?; echo "kernels rc=$rc"; tail -3 gpurun_out/k.log
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_bench.sh
