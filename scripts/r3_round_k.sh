#!/bin/bash
# lazy-C for the pair tiles (K = 512) A/B, the GPU suite, then bench + rocprof + PMC
set -o pipefail
for r in 1 2; do
  for cfg in "IPM_LAZYC=2" "IPM_LAZYC=1"; do
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8193 9 8194 || exit $?
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8192 9 || exit $?
  done
done
mkdir -p gpurun_out/r3k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3k/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 gpurun_out/r3k/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 TAG=r3k bash scripts/gpu_round.sh
