#!/bin/bash
# bench lines only (no profiler): headline + configs 2 / 4-concurrent / 5.   scripts/cfg_quick.sh OUTDIR
set -o pipefail
o=$1; mkdir -p $o
run() { local nm=$1; shift
  timeout -k 10 300 python bench.py --no-cpu "$@" > $o/$nm.json 2> $o/$nm.err || { echo "$nm failed"; tail -5 $o/$nm.err; exit 1; }
  echo "$nm $(python -c "import json,sys; d=json.load(open('$o/$nm.json')); print(d['value'], d.get('roofline',{}).get('frac'))")"
}
run c1 --steps 20 --warmup 4
run c2 --n 2048 --m 512 --steps 40 --warmup 4
run c4_conc --n 2048 --m 512 --instances 8 --concurrent --steps 20 --warmup 2
run c5 --problem socp --n 4096 --m 256 --steps 12 --warmup 2
