#!/bin/bash
# Round 4: least squares with one inner sweep (tests + timing vs host gelsd), the other BASELINE
# configurations (bench + rocprof each), config-4 hardware-queue sweep, PMC passes for the library.
set -o pipefail
OUT=gpurun_out/r4f
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s -k "lstsq" --timeout 300 --timeout-method thread > $OUT/pytest_lstsq.log 2>&1
rc=$?; echo "pytest lstsq rc=$rc"; grep -E "lstsq n=|passed|failed|FAILED" $OUT/pytest_lstsq.log | tail -14
[ $rc -ne 0 ] && exit $rc
HOST_MAX=8193 timeout -k 10 400 python scripts/lstsq_time.py 1025 2048 4096 8193 2>&1 | tee $OUT/lstsq_time.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
for q in 8 32; do
  IPM_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu --n 2048 --m 512 --instances 8 --concurrent --steps 20 --warmup 2 > $OUT/c4_q$q.json 2> $OUT/c4_q$q.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/c4_q$q.json'));print('c4 queues $q', round(d['value'],1))"
done
timeout -k 10 300 python bench.py --no-cpu --n 2048 --m 512 --instances 16 --concurrent --steps 20 --warmup 2 > $OUT/c4_i16.json 2> $OUT/c4_i16.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/c4_i16.json'));print('c4 16 instances', round(d['value'],1))"
SKIP_TESTS=1 TAG=r4f PT=400 BT=400 bash scripts/gpu_round.sh
