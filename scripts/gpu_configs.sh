#!/bin/bash
# Bench lines + rocprofv3 kernel-trace summaries for the other BASELINE configurations:
# config 2 (QP n=2048, m=512, one instance), config 3 (LP n=8192, m=2048), config 4 (8 x n=2048 per
# GPU, sequential and concurrent), config 5 (SOCP n=4096, 256 cones).  Each GPU step has its own
# time limit; the script stops at the first failure.
set -o pipefail
OUT=gpurun_out/${TAG:-r2cfg}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {   # name, bench args
  local nm=$1; shift
  timeout -k 10 300 python bench.py --no-cpu "$@" > $OUT/$nm.json 2> $OUT/$nm.err
  local rc=$?; echo "$nm rc=$rc"; cat $OUT/$nm.json
  [ $rc -ne 0 ] && { tail -5 $OUT/$nm.err; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$nm -o run -- \
      python3 bench.py --no-cpu "$@" > $OUT/prof_$nm.json 2> $OUT/prof_$nm.err
  rc=$?; echo "rocprof $nm rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/prof_$nm.err; exit $rc; }
  return 0
}
want() { [ -z "$CFGS" ] || [[ " $CFGS " == *" $1 "* ]]; }
want c2 && { run c2_qp2048 --n 2048 --m 512 --steps 40 --warmup 4 || exit 1; }
want c4s && { run c4_seq --n 2048 --m 512 --instances 8 --steps 20 --warmup 2 || exit 1; }
want c4 && { run c4_conc --n 2048 --m 512 --instances 8 --concurrent --steps 20 --warmup 2 || exit 1; }
want c3 && { run c3_lp8192 --problem lp --n 8192 --m 2048 --steps 12 --warmup 2 || exit 1; }
want c5 && { run c5_socp --problem socp --n 4096 --m 256 --steps 12 --warmup 2 || exit 1; }
exit 0
