#!/bin/bash
# A/B of library builds on the headline bench (IPM355_LIB override), alternating
set -o pipefail
mkdir -p gpurun_out/ablibs
for rep in 1 2; do
  for lib in "$@"; do
    IPM355_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 2 > gpurun_out/ablibs/out.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ablibs/out.json'));print('$lib', round(d['value'],2), round(d['potrf']['avg_ms'],3))"
  done
done
