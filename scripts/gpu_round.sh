#!/bin/bash
# One GPU-box pass: build, GPU tests, default bench line, rocprofv3 kernel-trace summary, and the
# PMC HBM-traffic passes (FETCH_SIZE / WRITE_SIZE in separate runs) for the two MFMA kernels.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
OUT=gpurun_out/${TAG:-r1}
mkdir -p $OUT
make -j8 > $OUT/build.log 2>&1 || { echo "build failed"; tail -20 $OUT/build.log; exit 1; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${TT:-700} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -3 $OUT/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 ${BT:-600} python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -2 $OUT/bench.err
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 ${PT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --no-cpu ${BENCH_ARGS} > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; echo "rocprof rc=$rc"; cat $OUT/prof_bench.json
[ $rc -ne 0 ] && exit $rc
[ -n "$SKIP_PMC" ] && exit 0
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_$c -o run -- \
      python3 bench.py --no-cpu --steps 3 --warmup 1 > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err
  rc=$?; echo "pmc $c rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/pmc_$c.err; exit $rc; }
done
F=$(find $OUT/pmc_FETCH_SIZE -name '*counter_collection.csv' | head -1)
W=$(find $OUT/pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_summary.py "k_potrf_block" $F $W $OUT/pmc_potrf_block.json 8192 2048
python3 scripts/pmc_summary.py "k_mfma_gemm<128, true, true" $F $W $OUT/pmc_kkt_syrk.json 8192 2048
