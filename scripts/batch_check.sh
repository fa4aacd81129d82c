#!/bin/bash
# batch group: the bit-identity test, then config 4 concurrent with and without the batch group
set -o pipefail
OUT=gpurun_out/${TAG:-batch}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s --timeout 240 --timeout-method thread -k "batch_group or concurrent" > $OUT/test.log 2>&1
rc=$?; tail -4 $OUT/test.log; [ $rc -ne 0 ] && exit $rc
for mode in "" "--batch" "" "--batch"; do
  timeout -k 10 300 python bench.py --no-cpu --n 2048 --m 512 --instances 8 --concurrent $mode --steps 20 --warmup 2 > $OUT/c4$mode.json 2> $OUT/c4$mode.err || { tail -5 $OUT/c4$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c4$mode.json'));print('$mode', round(d['value'],1), 'it/s potrf', round(d['potrf']['avg_ms'],3), d.get('batch_group'))"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --no-cpu --n 2048 --m 512 --instances 8 --concurrent --batch --steps 20 --warmup 2 > $OUT/prof.json 2> $OUT/prof.err
