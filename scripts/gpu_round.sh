#!/bin/bash
# One GPU-box pass (the library is built in-tree beforehand, on the CPU side): GPU tests, default bench line, rocprofv3 kernel-trace summary, and the
# PMC passes (FETCH_SIZE / WRITE_SIZE / MFMA busy cycles, each in its own run) for the two MFMA
# kernels.  Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
OUT=gpurun_out/${TAG:-r2}
mkdir -p $OUT
# (the library is built in-tree on the CPU side; nothing is compiled on the box)
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${TT:-900} python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -3 $OUT/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 ${BT:-600} python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -2 $OUT/bench.err
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 ${PT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --no-cpu ${BENCH_ARGS} > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; echo "rocprof rc=$rc"; cat $OUT/prof_bench.json
[ $rc -ne 0 ] && exit $rc
[ -n "$SKIP_PMC" ] && exit 0
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1
MF="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES"
i=0
for c in FETCH_SIZE WRITE_SIZE "$MF"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_$i -o run -- \
      python3 bench.py --no-cpu --steps 6 --warmup 2 ${BENCH_ARGS} > $OUT/pmc_$i.json 2> $OUT/pmc_$i.err
  rc=$?; echo "pmc pass $i ($c) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/pmc_$i.err; exit $rc; }
done
P=$(find $OUT/pmc_1 $OUT/pmc_2 $OUT/pmc_3 -name '*counter_collection.csv' | tr '\n' ' ')
python3 scripts/pmc_summary.py "k_potrf_block" $OUT/pmc_potrf_block.json ${PMC_N:-8192} ${PMC_M:-2048} $P
python3 scripts/pmc_summary.py "k_mfma_gemm_streamk<true, true" $OUT/pmc_kkt_syrk.json ${PMC_N:-8192} ${PMC_M:-2048} $P
