#!/bin/bash
# GPU: deferred-KKT parity test, then the bench with several deferral plans (A/B on one box).
set -o pipefail
mkdir -p gpurun_out/defer
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "deferred or full_solve" --timeout 200 \
    --timeout-method thread > gpurun_out/defer/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/defer/pytest.log
[ $rc -ne 0 ] && exit $rc
for cfg in ${CFGS:-"IPM_DEFER=0" "IPM_DEFER=1" "IPM_DEFER_FILL=1" "IPM_DEFER_FILL=1.5" \
           "IPM_DEFER_FILL=2.5" "IPM_DEFER=0"}; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu --steps 8 > gpurun_out/defer/b.json 2> gpurun_out/defer/b.err
  rc=$?
  [ $rc -ne 0 ] && { echo "$cfg bench rc=$rc"; tail -5 gpurun_out/defer/b.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/defer/b.json').read().strip().splitlines()[-1])
print('$cfg', round(d['value'],2), 'kkt', round(d['kkt_syrk']['avg_launch_ms'],3), 'potrf', round(d['potrf']['avg_ms'],3))"
done
