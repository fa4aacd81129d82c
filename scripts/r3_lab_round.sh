#!/bin/bash
# r3 GPU pass: tile / leaf labs, then the Lasso ADMM step at three split widths (each step under
# its own time limit; stops at the first failure)
set -o pipefail
OUT=gpurun_out/${TAG:-r3e}
mkdir -p $OUT
timeout -k 10 150 build/lab/tile_lab > $OUT/tile.txt 2>&1 || exit 1
timeout -k 10 60 build/lab/leaf2_lab > $OUT/leaf2.txt 2>&1 || exit 1
for sl in 512 1024 2048; do
  IPM_ADMM_SLOTS=$sl timeout -k 10 300 python scripts/lasso_bench.py 4096 30 300 > $OUT/lasso_$sl.json 2> $OUT/lasso_$sl.err || exit 1
  echo "slots $sl: $(cat $OUT/lasso_$sl.json)"
done
timeout -k 10 300 python -u -m pytest tests/test_lasso.py -q -x --timeout 120 --timeout-method thread -m gpu > $OUT/lasso_tests.log 2>&1
rc=$?; tail -2 $OUT/lasso_tests.log; exit $rc
