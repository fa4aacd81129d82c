#!/bin/bash
# A/B/C on the headline bench: "LIB|ENV" configurations (CFGS, ';'-separated), alternating, same box
set -o pipefail
mkdir -p gpurun_out/ab3
IFS=';' read -ra C <<< "${CFGS}"
for r in 1 2; do
  for cfg in "${C[@]}"; do
    lib=${cfg%%|*}; ev=${cfg#*|}
    env IPM355_LIB=$PWD/$lib $ev timeout -k 10 300 python bench.py --no-cpu --steps ${STEPS:-20} --warmup 2 ${BENCH_ARGS} \
        2>gpurun_out/ab3/err.txt > gpurun_out/ab3/out.json || { echo "fail $cfg"; tail -5 gpurun_out/ab3/err.txt; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab3/out.json').read().strip().splitlines()[-1])
print('$cfg', round(d['value'],2), 'kkt', round(d['kkt_syrk']['avg_launch_ms'],3), 'potrf', round(d['potrf']['avg_ms'],3), flush=True)"
  done
done
