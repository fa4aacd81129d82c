#!/bin/bash
# Block pairs only while the far region is large (IPM_PAIR_MIN sweep)
set -o pipefail
for r in 1 2; do
  for cfg in "IPM_PAIR=0" "IPM_PAIR=1 IPM_PAIR_MIN=3072" "IPM_PAIR=1 IPM_PAIR_MIN=4096" "IPM_PAIR=1 IPM_PAIR_MIN=5120" "IPM_PAIR=1 IPM_PAIR_MIN=6144" "IPM_PAIR=1 IPM_PAIR_MIN=7168"; do
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8192 9 || exit $?
  done
done
