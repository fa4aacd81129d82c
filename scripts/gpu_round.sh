#!/bin/bash
# One GPU-box pass: build, GPU tests, default bench line, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
OUT=gpurun_out/${TAG:-r1}
mkdir -p $OUT
make -j8 > $OUT/build.log 2>&1 || { echo "build failed"; tail -20 $OUT/build.log; exit 1; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${TT:-700} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -15 $OUT/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 ${BT:-600} python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -5 $OUT/bench.err
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 ${PT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --no-cpu ${BENCH_ARGS} > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; echo "rocprof rc=$rc"; cat $OUT/prof_bench.json; tail -3 $OUT/prof.err
find $OUT/prof -name '*stats*' | head
exit $rc
