#!/bin/bash
# Round 4: the KKT SYRK's stream-K tail modes on config 5 (SOCP n = 4096: 528 128-tiles on 512
# slots, 16 tiles split) -- IPM_STREAMK 3 (default: pieces first, <= 8 per tile), 1 (pieces first,
# <= 16), 2 (pieces last, <= 16); env A/B, two pairs.
set -o pipefail
OUT=gpurun_out/r4q
mkdir -p $OUT
CF="IPM_STREAMK=3;IPM_STREAMK=1;IPM_STREAMK=2"
CFGS="$CF" BENCH_ARGS="--problem socp --n 4096 --m 256 --steps 12 --warmup 2" bash scripts/env_ab.sh 2>&1 | tee $OUT/c5.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
exit 0
