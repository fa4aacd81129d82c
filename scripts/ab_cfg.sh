#!/bin/bash
# A/B of library builds (IPM355_LIB) on the headline bench and the n=2048 config, alternating, two pairs
set -o pipefail
mkdir -p gpurun_out/abcfg
for rep in 1 2; do
  for lib in "$@"; do
    IPM355_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 2 > gpurun_out/abcfg/h.json 2>/dev/null || exit 1
    IPM355_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --n 2048 --m 512 --steps 40 --warmup 4 > gpurun_out/abcfg/s.json 2>/dev/null || exit 1
    python3 -c "
import json;h=json.load(open('gpurun_out/abcfg/h.json'));s=json.load(open('gpurun_out/abcfg/s.json'))
print('$lib', 'n8192', round(h['value'],2), 'potrf', round(h['potrf']['avg_ms'],3), '| n2048', round(s['value'],1), 'potrf', round(s['potrf']['avg_ms'],4))"
  done
done
