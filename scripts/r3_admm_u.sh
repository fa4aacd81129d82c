#!/bin/bash
# ADMM step kernel: slabs in flight per wave (IPM_ADMM_U) x workgroup target, n = 4097, S = 30
set -o pipefail
OUT=gpurun_out/admmu
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for cfg in "IPM_ADMM_U=4" "IPM_ADMM_U=8" "IPM_ADMM_U=16" "IPM_ADMM_U=8 IPM_ADMM_WG=1032" "IPM_ADMM_U=16 IPM_ADMM_WG=260"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- \
    python3 scripts/lasso_bench.py 4096 30 600 > $OUT/$tag.json 2> $OUT/$tag.err || exit 1
  echo "$cfg done"
done
