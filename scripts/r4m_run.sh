#!/bin/bash
# Round 4: look-ahead 128-tiles only while more than IPM_LA128_MIN rows remain (r4l: IPM_LA128=0
# took n = 2048's factorization 0.865 -> 0.816 ms); env A/B, two pairs, on the headline (n = 8192),
# config 2 (QP n = 2048) and config 5 (SOCP n = 4096).
set -o pipefail
OUT=gpurun_out/r4m
mkdir -p $OUT
CF="IPM_LA128_MIN=0;IPM_LA128_MIN=2048;IPM_LA128_MIN=3072;IPM_LA128_MIN=4096;IPM_LA128_MIN=99999"
CFGS="$CF" BENCH_ARGS="--n 2048 --m 512 --steps 40 --warmup 4" bash scripts/env_ab.sh 2>&1 | tee $OUT/c2.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
CFGS="$CF" BENCH_ARGS="--problem socp --n 4096 --m 256 --steps 12 --warmup 2" bash scripts/env_ab.sh 2>&1 | tee $OUT/c5.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
CFGS="$CF" BENCH_ARGS="--steps 20 --warmup 2" bash scripts/env_ab.sh 2>&1 | tee $OUT/head.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
exit 0
