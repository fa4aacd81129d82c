#!/bin/bash
# block pairs for the first launches only: threshold sweep, then the GPU suite with pairs on
set -o pipefail
mkdir -p gpurun_out/pairs
for r in 1 2; do
  for cfg in "IPM_PAIR=0" "IPM_PAIR=1 IPM_PAIR_MIN=6656" "IPM_PAIR=1 IPM_PAIR_MIN=6144" "IPM_PAIR=1 IPM_PAIR_MIN=5632"; do
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8192 9 || exit $?
  done
done
export IPM_PAIR=1 IPM_PAIR_MIN=6144
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pairs/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu (pairs) rc=$rc"; tail -3 gpurun_out/pairs/pytest_gpu.log; exit $rc
