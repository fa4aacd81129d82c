#!/bin/bash
# A/B: bench.py with the current library and with build/old/libipm355.so, alternating, same box
set -o pipefail
for r in 1 2; do
  for lib in interiorpoint-gpu_amd/ipm355/libipm355.so build/old/libipm355.so; do
    IPM355_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS} 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib'.split('/')[-2], round(d['value'],2), 'kkt', round(d['kkt_syrk']['avg_launch_ms'],3), 'potrf', round(d['potrf']['avg_ms'],3))" || exit 1
  done
done
