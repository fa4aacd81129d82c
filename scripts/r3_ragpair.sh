#!/bin/bash
# pairs vs plain at the solver's shapes (bordered n = N+1, even ldh) + the leaf lab
set -o pipefail
for r in 1 2; do
  for cfg in "IPM_PAIR=0" "IPM_PAIR=1"; do
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8192 9 || exit $?
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8193 9 8194 || exit $?
    env $cfg timeout -k 10 120 python scripts/potrf_time.py 8194 9 8194 || exit $?
  done
done
timeout -k 10 60 build/lab/leaf2_lab || exit $?
