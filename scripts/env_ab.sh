#!/bin/bash
# bench A/B over env configurations (CFGS, ';'-separated), alternating, same box
set -o pipefail
IFS=';' read -ra C <<< "${CFGS}"
for r in 1 2; do
  for cfg in "${C[@]}"; do
    env $cfg timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS} 2>/dev/null > gpurun_out/envab.json || { echo "fail $cfg"; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/envab.json').read().strip().splitlines()[-1])
print('$cfg', round(d['value'],2), 'kkt', round(d['kkt_syrk']['avg_launch_ms'],3), 'potrf', round(d['potrf']['avg_ms'],3))"
  done
done
