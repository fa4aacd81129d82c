#!/bin/bash
# ADMM step kernel vs the K-split workgroup target (IPM_ADMM_WG), n = 4097, S = 30
set -o pipefail
OUT=gpurun_out/admm
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for wg in 512 1032 2064 768; do
  IPM_ADMM_WG=$wg timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/w$wg -o run -- \
    python3 scripts/lasso_bench.py 4096 30 600 > $OUT/w$wg.json 2> $OUT/w$wg.err || exit 1
  f=$(find $OUT/w$wg -name '*kernel_stats.csv' | head -1)
  echo "WG=$wg"; grep -i "admm_step" $f | cut -d, -f1-4
done
