#!/bin/bash
# Round 4: config 4 (8 concurrent n = 2048 QPs) with the two-stream panel Cholesky
# (IPM_POTRF_LA=1: panel launches + trailing GEMM launches, no waiting workgroups holding CU slots)
# against the fused one-launch-per-block form; config 2 alongside.  env A/B, two pairs.
set -o pipefail
OUT=gpurun_out/r4o
mkdir -p $OUT
CF="IPM_POTRF_LA=0;IPM_POTRF_LA=1;IPM_POTRF_LA=1 IPM_NO_LOOKAHEAD=1"
CFGS="$CF" BENCH_ARGS="--n 2048 --m 512 --instances 8 --concurrent --steps 20 --warmup 2" bash scripts/env_ab.sh 2>&1 | tee $OUT/c4.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
CFGS="$CF" BENCH_ARGS="--n 2048 --m 512 --steps 40 --warmup 4" bash scripts/env_ab.sh 2>&1 | tee $OUT/c2.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
exit 0
