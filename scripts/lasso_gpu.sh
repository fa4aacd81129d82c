#!/bin/bash
set -o pipefail
OUT=gpurun_out/${TAG:-lasso}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for cfg in "1024 30 500" "4096 30 300" "4096 128 200"; do
  timeout -k 10 300 python scripts/lasso_bench.py $cfg >> $OUT/lasso_bench.jsonl 2> $OUT/lasso_bench.err || exit 1
done
cat $OUT/lasso_bench.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 scripts/lasso_bench.py 4096 30 300 > $OUT/prof.json 2> $OUT/prof.err || exit 1
