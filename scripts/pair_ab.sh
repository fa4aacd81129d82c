#!/bin/bash
# block-pair Cholesky: kernel tests, then bench A/B (IPM_PAIR=0 vs pairs at two thresholds), then the
# full-solve parity tests; every GPU step under its own time limit, stop at the first failure
set -o pipefail
OUT=gpurun_out/${TAG:-pair}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "potrf or chol" -x -q --timeout 120 --timeout-method thread > $OUT/k.log 2>&1
rc=$?; tail -3 $OUT/k.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for cfg in ${CFGS:-"IPM_PAIR=0" "IPM_PAIR_MIN=3072" "IPM_PAIR_MIN=2048"}; do
    env ${cfg//,/ } timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 2 > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
    python3 -c "
import json;h=json.load(open('$OUT/b.json'))
print('$cfg', round(h['value'],2), 'potrf', round(h['potrf']['avg_ms'],3), 'frac', round(h['roofline']['frac'],4), 'parity', h.get('parity'))"
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -k "m3_full or m2_qp or truncated" -x -v -s --timeout 300 --timeout-method thread > $OUT/large.log 2>&1
rc=$?; grep -E "x\* rel|PASS|FAIL" $OUT/large.log | head -20; exit $rc
