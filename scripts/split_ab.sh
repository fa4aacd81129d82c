#!/bin/bash
# A/B of the K-split trailing tiles: potrf kernel tests, then the headline bench with IPM_SPLIT=0/1
# (kernel-trace summaries of both), planner decisions in split_debug.txt.
set -o pipefail
OUT=gpurun_out/${TAG:-split}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -s --timeout 200 --timeout-method thread -k "potrf" > $OUT/kernels.log 2>&1
rc=$?; tail -3 $OUT/kernels.log; [ $rc -ne 0 ] && exit $rc
IPM_SPLIT_DEBUG=1 timeout -k 10 200 python bench.py --no-cpu --steps 4 --warmup 0 > /dev/null 2> $OUT/split_debug.txt || exit 1
for sp in 0 1 0 1; do
  IPM_SPLIT=$sp timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS} > $OUT/bench_s$sp.json 2> $OUT/bench_s$sp.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/bench_s$sp.json'));print('split',$sp,round(d['value'],2),'it/s potrf',round(d['potrf']['avg_ms'],3),'ms frac',round(d['roofline']['frac'],4))"
done
for sp in 0 1; do
  IPM_SPLIT=$sp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_s$sp -o run -- \
      python3 bench.py --no-cpu --steps 8 --warmup 2 > $OUT/prof_s$sp.json 2> $OUT/prof_s$sp.err || exit 1
done
