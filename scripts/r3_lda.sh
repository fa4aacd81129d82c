#!/bin/bash
# Cholesky time vs leading dimension at the solver's bordered size (column alignment)
set -o pipefail
for r in 1 2; do
  for lda in 8194 8200 8208 8224 8256; do
    timeout -k 10 120 python scripts/potrf_time.py 8193 9 $lda || exit $?
  done
  timeout -k 10 120 python scripts/potrf_time.py 8192 9 8192 || exit $?
  timeout -k 10 120 python scripts/potrf_time.py 8192 9 8208 || exit $?
done
