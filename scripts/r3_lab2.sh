#!/bin/bash
# leaf-lab variants; Lasso ADMM step kernel time under rocprofv3 (n = 4097, S = 30)
set -o pipefail
OUT=gpurun_out/${TAG:-r3f}
mkdir -p $OUT
timeout -k 10 60 build/lab/leaf2_lab > $OUT/leaf2.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lasso_prof -o run -- \
    python3 scripts/lasso_bench.py 4096 30 300 > $OUT/lasso_prof.json 2> $OUT/lasso_prof.err || exit 1
f=$(find $OUT/lasso_prof -name '*kernel_stats.csv' | head -1); grep -i "admm" $f
