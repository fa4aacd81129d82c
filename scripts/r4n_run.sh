#!/bin/bash
# Round 4 checkpoint after the look-ahead 128-tile threshold (IPM_LA128_MIN=3072 default) and the
# stream-K 128-tile KKT for grids just past a round (SOCP n = 4096): config 5 first (the changed
# KKT), the GPU suite, the headline bench + rocprofv3 + PMC (gpu_round.sh), then configs 2-5 with
# their rocprofv3 summaries (gpu_configs.sh).
set -o pipefail
OUT=gpurun_out/${TAG:-r4n}
mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu --problem socp --n 4096 --m 256 --steps 12 --warmup 2 > $OUT/c5_first.json 2> $OUT/c5_first.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/c5_first.json'));print('c5', round(d['value'],1), 'kkt', round(d['kkt_syrk']['avg_launch_ms'],3), 'potrf', round(d['potrf']['avg_ms'],3))"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 TAG=${TAG:-r4n} PT=400 BT=400 bash scripts/gpu_round.sh || exit $?
TAG=${TAG:-r4n}_configs bash scripts/gpu_configs.sh || exit $?
