#!/bin/bash
# far-region threshold of the block pairs, with lazy-C pair tiles (solver's bordered size)
set -o pipefail
for r in 1 2; do
  for mn in 6144 5632 5120 4096; do
    IPM_PAIR_MIN=$mn timeout -k 10 120 python scripts/potrf_time.py 8193 9 8194 || exit $?
  done
done
