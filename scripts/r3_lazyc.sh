#!/bin/bash
# lazy C reads in the Cholesky's K = 256 trailing tiles (IPM_LAZYC) vs the C-read burst
set -o pipefail
for r in 1 2; do
  for cfg in "IPM_LAZYC=0" "IPM_LAZYC=1"; do
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8192 9 || exit $?
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8193 9 8194 || exit $?
  done
done
IPM_LAZYC=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "potrf or chol" --timeout 120 --timeout-method thread 2>&1 | tail -3
