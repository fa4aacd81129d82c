#!/bin/bash
# A/B of library builds on bench.py (IPM355_LIB override), alternating builds, REPS pairs.
#   scripts/ab.sh OUTDIR "BENCH ARGS" LIB1 LIB2 ...      (env: REPS=2, T=300 seconds per run)
# Prints one line per run: library, Newton it/s, Cholesky ms, KKT SYRK ms.  Replaces the one-off
# r3_*.sh wrappers of round 3 (knob A/B: pass the same library twice and set the knob per entry as
# VAR=value@lib, e.g.  IPM_PAIR=0@interiorpoint-gpu_amd/ipm355/libipm355.so).
set -o pipefail
out=$1; shift
args=$1; shift
mkdir -p "$out"
for rep in $(seq 1 ${REPS:-2}); do
  for spec in "$@"; do
    envs=""; lib=$spec
    if [[ "$spec" == *@* ]]; then envs=${spec%@*}; lib=${spec##*@}; fi
    env $envs IPM355_LIB=$PWD/$lib timeout -k 10 ${T:-300} python bench.py --no-cpu $args > "$out/run.json" 2> "$out/run.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "$spec: bench rc=$rc"; tail -5 "$out/run.err"; exit $rc; fi
    python3 -c "import json;d=json.load(open('$out/run.json'));p=d.get('parity') or {};print('$spec', round(d['value'],2), 'potrf', round(d['potrf']['avg_ms'],3), 'syrk', round(d['kkt_syrk']['avg_launch_ms'],3), 'steps_identical', [v.get('steps_identical') for v in p.values() if v])"
  done
done
