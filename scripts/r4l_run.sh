#!/bin/bash
# Round 4: the Cholesky's run-time knobs (tuned on one n = 8192 instance) on configs 2 (one
# n = 2048 QP) and 4 (8 concurrent n = 2048 QPs through ipm355.dist.Shard), env A/B, two pairs.
set -o pipefail
OUT=gpurun_out/r4l
mkdir -p $OUT
CF="IPM_NONE=0;IPM_PAIR=0;IPM_SPLIT=0;IPM_LA128=0;IPM_RAG=0;IPM_LAZYC=0"
CFGS="$CF" BENCH_ARGS="--n 2048 --m 512 --instances 8 --concurrent --steps 20 --warmup 2" bash scripts/env_ab.sh 2>&1 | tee $OUT/c4_knobs.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
CFGS="$CF" BENCH_ARGS="--n 2048 --m 512 --steps 40 --warmup 4" bash scripts/env_ab.sh 2>&1 | tee $OUT/c2_knobs.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
# rotations per outer sweep of the blocked Jacobi (n = 2048)
IPM_BJ_DEBUG=1 HOST_MAX=0 timeout -k 10 120 python scripts/lstsq_time.py 2048 > $OUT/bj_sweeps.txt 2>&1 || exit 1
grep -c "rotations" $OUT/bj_sweeps.txt
exit 0
