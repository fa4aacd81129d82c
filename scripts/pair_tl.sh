#!/bin/bash
# per-launch Cholesky timelines (n = 8192): plain vs block pairs
set -o pipefail
OUT=gpurun_out/${TAG:-pairtl}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for cfg in 0 1; do
  IPM_PAIR=$cfg timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p$cfg -o run -- python3 scripts/potrf_once.py 8192 > $OUT/p$cfg.out 2>&1 || { tail -5 $OUT/p$cfg.out; exit 1; }
  f=$(find $OUT/p$cfg -name '*kernel_trace.csv' | head -1)
  echo "IPM_PAIR=$cfg"; python3 scripts/launch_timeline2.py $f 32
done
