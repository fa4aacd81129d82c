#!/bin/bash
# lazy-C tiles vs the K-split planner (a launch with split tiles runs the non-lazy kernel)
set -o pipefail
for r in 1 2; do
  for cfg in "IPM_SPLIT=1" "IPM_SPLIT=0" "IPM_LAZYC=0"; do
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8193 9 8194 || exit $?
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8192 9 || exit $?
  done
done
