#!/bin/bash
# A/B of the KKT SYRK tail modes (IPM_STREAMK=0..3): launch times alternating, then bench lines
set -o pipefail
mkdir -p gpurun_out/sk
for rep in 1 2; do
  for m in 0 1 2 3; do
    IPM_STREAMK=$m timeout -k 10 120 python scripts/syrk_tail_bench.py >> gpurun_out/sk/syrk.log 2>&1 || exit $?
  done
done
cat gpurun_out/sk/syrk.log
for m in ${BMODES:-0 1 2}; do
  IPM_STREAMK=$m timeout -k 10 300 python bench.py --no-cpu --steps 30 > gpurun_out/sk/bench_$m.json 2> gpurun_out/sk/bench_$m.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/sk/bench_$m.json'));print('mode $m', round(d['value'],2), 'it/s kkt', round(d['kkt_syrk']['avg_launch_ms'],3), 'ms potrf', round(d['potrf']['avg_ms'],3))"
done
