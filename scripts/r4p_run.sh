#!/bin/bash
# Round 4: the pair threshold (IPM_PAIR_MIN) and the look-ahead 128-tile threshold around their
# defaults on the headline (n = 8192), env A/B, two pairs.
set -o pipefail
OUT=gpurun_out/r4p
mkdir -p $OUT
CF="IPM_PAIR_MIN=6144;IPM_PAIR_MIN=5120;IPM_PAIR_MIN=7168;IPM_LA128_MIN=2560;IPM_LA128_MIN=3584"
CFGS="$CF" BENCH_ARGS="--steps 20 --warmup 2" bash scripts/env_ab.sh 2>&1 | tee $OUT/head.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
exit 0
