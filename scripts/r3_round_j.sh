#!/bin/bash
# final round: GPU suite + bench + rocprof + PMC (gpu_round.sh), then the lazy-C A/B at the solver sizes
set -o pipefail
TAG=r3j bash scripts/gpu_round.sh || exit $?
for r in 1 2; do
  for cfg in "IPM_LAZYC=1" "IPM_LAZYC=0"; do
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8193 9 8194 || exit $?
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8192 9 || exit $?
  done
done
