#!/bin/bash
# ADMM step with the tile-blocked Qs: kernel time under rocprofv3 and the Lasso parity tests
set -o pipefail
OUT=gpurun_out/admmblk
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 scripts/lasso_bench.py 4096 30 600 > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/bench.json
timeout -k 10 300 python -u -m pytest tests/test_lasso.py -q -m gpu --timeout 200 --timeout-method thread 2>&1 | tail -3
