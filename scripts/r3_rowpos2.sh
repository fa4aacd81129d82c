#!/bin/bash
# Row-chunk placement A/B with XCD-phase padding (IPM_ROWPAD)
set -o pipefail
for r in 1 2; do
  for cfg in "IPM_ROWPOS=0" "IPM_ROWPOS=1" "IPM_ROWPOS=1 IPM_ROWPAD=0" "IPM_ROWPOS=1 IPM_ROW_TB=9" "IPM_ROWPOS=1 IPM_ROW_TA=1.5 IPM_ROW_TB=2.5"; do
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8192 9 || exit $?
  done
done
