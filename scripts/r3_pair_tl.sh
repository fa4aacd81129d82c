#!/bin/bash
# per-launch Cholesky timelines (n = 8192): plain vs block pairs at several far-region thresholds
set -o pipefail
OUT=gpurun_out/pairtl3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for cfg in "IPM_PAIR=0" "IPM_PAIR=1 IPM_PAIR_MIN=6144" "IPM_PAIR=1 IPM_PAIR_MIN=3072"; do
  i=$((i+1))
  env $cfg timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 scripts/potrf_once.py 8192 > $OUT/p$i.out 2>&1 || { tail -5 $OUT/p$i.out; exit 1; }
  f=$(find $OUT/p$i -name '*kernel_trace.csv' | head -1)
  echo "$cfg"; python3 scripts/launch_timeline2.py $f 33
done
