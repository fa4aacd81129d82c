#!/bin/bash
# Row-chunk placement A/B (IPM_ROWPOS / IPM_ROWPRIO): POTRF time per configuration (one process
# each), the planner's choice, then the default bench line (CPU baseline children included).
set -o pipefail
mkdir -p gpurun_out/rowpos
IPM_ROWPOS=1 IPM_SPLIT_DEBUG=1 timeout -k 10 120 python scripts/potrf_time.py 8192 1 2> gpurun_out/rowpos/plan8192.txt || exit $?
for r in 1 2; do
  for cfg in "IPM_ROWPOS=0" "IPM_ROWPOS=1" "IPM_ROWPOS=1 IPM_ROWPRIO=2" "IPM_ROWPRIO=2" "IPM_ROWPOS=1 IPM_ROW_TB=9"; do
    for n in 8192 2048; do
      env $cfg timeout -k 10 120 python scripts/potrf_time.py $n 9 || exit $?
    done
  done
done
timeout -k 10 600 python bench.py > gpurun_out/rowpos/bench.json 2> gpurun_out/rowpos/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/rowpos/bench.json; exit $rc
