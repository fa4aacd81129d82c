#!/bin/bash
# Bench-level A/B of the KKT SYRK tail (IPM_STREAMK=0: K-halves split, 3: stream-K pieces), two pairs
set -o pipefail
OUT=gpurun_out/${TAG:-r2}
mkdir -p $OUT
for rep in 1 2; do
  for m in 0 3; do
    IPM_STREAMK=$m timeout -k 10 300 python bench.py --no-cpu --steps 30 > $OUT/ab_$m.json 2> $OUT/ab_$m.err || exit $?
    python -c "import json;d=json.load(open('$OUT/ab_$m.json'));print('mode $m', round(d['value'],2), 'it/s kkt', round(d['kkt_syrk']['avg_launch_ms'],3), 'ms potrf', round(d['potrf']['avg_ms'],3))" | tee -a $OUT/ab.txt
  done
done
