#!/bin/bash
# bench.py A/B of library builds, alternated REPS times:
#   scripts/bench_ab.sh OUT "spec spec ..." [bench args]     (env REPS=2)
# spec: a library path, or VAR=value@library (an environment knob for that run)
# prints one line per run: library, it/s, KKT SYRK ms, Cholesky ms
set -o pipefail
out=$1; libs=$2; shift 2
mkdir -p $(dirname $out)
for r in $(seq 1 ${REPS:-2}); do
  for spec in $libs; do
    lib=${spec#*@}; kv=""; [ "$lib" != "$spec" ] && kv=${spec%@*}
    env $kv IPM355_LIB=$PWD/$lib timeout -k 10 240 python bench.py --no-cpu "$@" > $out.tmp 2> $out.err || { tail -5 $out.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('$out.tmp'))
print('%-34s %8.2f it/s  syrk %.3f ms  potrf %.3f ms' % ('$spec', d['value'], d['kkt_syrk']['avg_launch_ms'], d['potrf']['avg_ms']))" | tee -a $out
  done
done
rm -f $out.tmp
