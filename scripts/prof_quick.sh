#!/bin/bash
# rocprofv3 kernel trace of a short bench; prints per-kernel avg durations (top 16)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/pq
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pq -o run -- \
    python3 bench.py --no-cpu --steps ${STEPS:-6} ${BENCH_ARGS} > gpurun_out/pq_bench.json 2> gpurun_out/pq.err || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/pq/**/run_kernel_stats.csv', recursive=True) + glob.glob('gpurun_out/pq/run_kernel_stats.csv')
rows = list(csv.DictReader(open(f[0])))
for r in rows[:16]:
    print(f"{r['Name'][:70]:70s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs'])/1e3:9.1f} pct {r['Percentage']}")
PY
